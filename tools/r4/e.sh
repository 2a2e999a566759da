# round 4: fused blend finalize + rast_bwd LDS layout: tests, sweep, PMC (through gpurun)
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/r4e"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_fused_finalize.py tests/test_gpu_segments.py tests/test_gpu_rast.py tests/test_gpu_deterministic.py \
  tests/test_gpu_rast_kat.py tests/test_gpu_headline_parity.py tests/test_gpu_blend.py tests/test_gpu_scalar_link.py \
  tests/test_gpu_graph.py > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" "$OUT/tests.log" | tail -8; [ $rc -ne 0 ] && exit $rc
bash tools/gpu.sh sweep r4e cfg2 "base|PR_X=0|" "nosync|PR_BLEND_SYNC=0|" "base2|PR_X=0|" "nosync2|PR_BLEND_SYNC=0|" || exit 1
bash tools/gpu.sh pmc r4e || exit 1
