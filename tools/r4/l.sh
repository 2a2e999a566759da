# round 4: per-tile compacted / walk fragment output (PR_RAST_FRAGC_DENSE): parity, then sweeps
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_rast.py tests/test_gpu_rast_kat.py tests/test_gpu_headline_parity.py tests/test_gpu_fullsize.py \
  tests/test_gpu_counts.py tests/test_gpu_deterministic.py > gpurun_out/tests_r4l.log 2>&1
rc=$?; tail -n 2 gpurun_out/tests_r4l.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu.sh sweep r4l cfg2 "d101|PR_RAST_FRAGC_DENSE=101|" "d85|PR_RAST_FRAGC_DENSE=85|" "d60|PR_RAST_FRAGC_DENSE=60|" \
  "d0|PR_RAST_FRAGC_DENSE=0|" "d101b|PR_RAST_FRAGC_DENSE=101|" "d85b|PR_RAST_FRAGC_DENSE=85|" || exit 1
bash tools/gpu.sh sweep r4le eval "d101|PR_RAST_FRAGC_DENSE=101|" "d85|PR_RAST_FRAGC_DENSE=85|" "d0|PR_RAST_FRAGC_DENSE=0|" || exit 1
bash tools/gpu.sh sweep r4l3 cfg3 "d101|PR_RAST_FRAGC_DENSE=101|" "d85|PR_RAST_FRAGC_DENSE=85|" || exit 1
bash tools/gpu.sh sweep r4l4 cfg4 "d101|PR_RAST_FRAGC_DENSE=101|" "d85|PR_RAST_FRAGC_DENSE=85|" || exit 1
