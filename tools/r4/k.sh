# round 4: 512-thread forward blend workgroups (PR_BLEND_FWD_THREADS=512): parity, then cfg2/eval/cfg3/cfg4 sweeps
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
PR_BLEND_FWD_THREADS=512 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_blend.py tests/test_gpu_headline_parity.py tests/test_gpu_variants.py tests/test_gpu_empty_blocks.py \
  tests/test_gpu_counts.py tests/test_gpu_host_layer.py > gpurun_out/tests_r4k.log 2>&1
rc=$?; tail -n 2 gpurun_out/tests_r4k.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu.sh sweep r4k cfg2 "base|PR_X=0|" "nt512|PR_BLEND_FWD_THREADS=512|" "base2|PR_X=0|" "nt512b|PR_BLEND_FWD_THREADS=512|" || exit 1
bash tools/gpu.sh sweep r4ke eval "base|PR_X=0|" "nt512|PR_BLEND_FWD_THREADS=512|" || exit 1
bash tools/gpu.sh sweep r4k3 cfg3 "base|PR_X=0|" "nt512|PR_BLEND_FWD_THREADS=512|" || exit 1
bash tools/gpu.sh sweep r4k4 cfg4 "base|PR_X=0|" "nt512|PR_BLEND_FWD_THREADS=512|" || exit 1
