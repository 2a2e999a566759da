set -e
cd "$GRAFT_REPO_ROOT"; OUT="$GRAFT_REPO_ROOT/gpurun_out/cfg5prof"; mkdir -p "$OUT"
for nt in ${NTS:-softras gaussian}; do
  (cd /tmp && export TMPDIR=/tmp PYTHONPATH="$GRAFT_REPO_ROOT" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$nt" -o p -- \
     python -m pertrenderer_amd.pose_opt --mode graph -np 4 -sn $nt > "$OUT/$nt.log" 2>&1)
  find "$OUT/$nt" -name "*kernel_trace.csv" -delete
done
echo done
