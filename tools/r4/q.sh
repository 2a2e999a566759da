# round 4: rasterizer forward with div_rn (PR_RAST_FASTDIV): GPU division check, bit-exact tests, A/B sweeps
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 120 ./tools/fastdiv_check > gpurun_out/fastdiv_check.txt 2>&1; rc=$?; cat gpurun_out/fastdiv_check.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_rast.py tests/test_gpu_rast_kat.py tests/test_gpu_headline_parity.py tests/test_gpu_counts.py \
  tests/test_gpu_pipeline_ref.py tests/test_gpu_fullsize.py tests/test_gpu_deterministic.py > gpurun_out/tests_r4q.log 2>&1
rc=$?; tail -n 3 gpurun_out/tests_r4q.log; [ $rc -ne 0 ] && exit $rc
PR_NATIVE_LIB=$R/pertrenderer_amd/libpertrender_nofd.so timeout -k 10 300 python -u -m pytest -x -q --timeout 250 \
  --timeout-method thread -p no:cacheprovider tests/test_gpu_rast.py > gpurun_out/tests_r4q_nofd.log 2>&1
rc=$?; tail -n 2 gpurun_out/tests_r4q_nofd.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu.sh sweep r4q cfg2 "fd|PR_X=0|" "ieee|PR_X=0|libpertrender_nofd" "fd2|PR_X=0|" "ieee2|PR_X=0|libpertrender_nofd" || exit 1
bash tools/gpu.sh sweep r4qe eval "fd|PR_X=0|" "ieee|PR_X=0|libpertrender_nofd" || exit 1
bash tools/gpu.sh sweep r4q4 cfg4 "fd|PR_X=0|" "ieee|PR_X=0|libpertrender_nofd" || exit 1
