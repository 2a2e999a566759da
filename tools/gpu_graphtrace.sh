# kernel trace of the graph-mode bench (for the per-replay kernel list: tools/replay.py)
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG="${1:-gt}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$TAG" -o g -- \
  python "$R/bench.py" --no-cpu-baseline --no-dense --steps 20 --warmup 5 > "$OUT/$TAG.json" 2> "$OUT/$TAG.err"
rc=$?; echo "graphtrace rc=$rc"; cut -c1-300 "$OUT/$TAG.json"
exit $rc
