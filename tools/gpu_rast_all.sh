# rasterizer GPU tests for every slice count (and the separate fragment pass), then a bench sweep
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
cd "$R"
for cfg in "PR_RAST_SLICES=1" "PR_RAST_SLICES=2" "PR_RAST_SLICES=4" "PR_RAST_SLICES=8" "PR_RAST_SLICES=4 PR_RAST_FRAG=0"; do
  env $cfg timeout -k 10 300 python -u -m pytest tests/test_gpu_rast.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/trast.log" 2>&1
  rc=$?; echo "$cfg rc=$rc $(tail -1 $OUT/trast.log)"
  if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" "$OUT/trast.log" | head -10; exit $rc; fi
done
bash tools/gpu_sweep.sh "$@"
