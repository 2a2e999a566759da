# GPU tests for each rasterizer wave count, then the sweep
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
cd "$R"
for w in 4 2 1; do
  PR_RAST_WAVES=$w timeout -k 10 300 python -m pytest tests/test_gpu_rast.py -q -x --timeout 120 -p no:cacheprovider > "$OUT/trast_$w.log" 2>&1
  rc=$?; echo "waves=$w pytest rc=$rc"; tail -2 "$OUT/trast_$w.log"
  [ $rc -ne 0 ] && exit $rc
done
bash tools/gpu_sweep.sh
