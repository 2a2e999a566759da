# rasterizer GPU tests for each wave count, phase profile, then the bench sweep
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG="${1:-ra}"
cd "$R"
for w in 1 2 4; do
  PR_RAST_WAVES=$w timeout -k 10 300 python -m pytest tests/test_gpu_rast.py -q -x --timeout 120 -p no:cacheprovider > "$OUT/trast_$w.log" 2>&1
  rc=$?; echo "waves=$w pytest rc=$rc $(tail -1 $OUT/trast_$w.log)"
  [ $rc -ne 0 ] && { tail -20 "$OUT/trast_$w.log"; exit $rc; }
done
bash tools/gpu_rprof.sh "$TAG" || exit $?
bash tools/gpu_sweep.sh
