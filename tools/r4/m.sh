# round 4: face-range split of the rasterizer tiles (PR_RAST_SPLIT=1): bit-exactness, then sweeps
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
PR_RAST_SPLIT=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_rast.py tests/test_gpu_rast_kat.py tests/test_gpu_headline_parity.py tests/test_gpu_counts.py \
  tests/test_gpu_pipeline_ref.py tests/test_gpu_host_layer.py > gpurun_out/tests_r4m.log 2>&1
rc=$?; tail -n 2 gpurun_out/tests_r4m.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu.sh sweep r4m cfg2 "base|PR_X=0|" "split|PR_RAST_SPLIT=1|" "base2|PR_X=0|" "split2|PR_RAST_SPLIT=1|" || exit 1
bash tools/gpu.sh sweep r4me eval "base|PR_X=0|" "split|PR_RAST_SPLIT=1|" || exit 1
