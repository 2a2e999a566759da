# round 4: blend backward with 16-bit win counts (LDS <= 20 KB at cfg 2: 8 workgroups per CU), tests + A/B
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_blend.py tests/test_gpu_empty_blocks.py tests/test_gpu_fused_finalize.py tests/test_gpu_headline_parity.py \
  tests/test_gpu_segments.py tests/test_gpu_variants.py tests/test_gpu_cfg4_blend.py tests/test_gpu_host_layer.py \
  tests/test_gpu_deterministic.py > gpurun_out/tests_r4u.log 2>&1
rc=$?; tail -n 3 gpurun_out/tests_r4u.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu.sh sweep r4u cfg2 "cn16|PR_X=0|" "base|PR_X=0|libpertrender_base" "cn16b|PR_X=0|" "baseb|PR_X=0|libpertrender_base" || exit 1
bash tools/gpu.sh sweep r4ue eval "cn16|PR_X=0|" "base|PR_X=0|libpertrender_base" || exit 1
bash tools/gpu.sh sweep r4u3 cfg3 "cn16|PR_X=0|" "base|PR_X=0|libpertrender_base" || exit 1
bash tools/gpu.sh sweep r4u4 cfg4 "cn16|PR_X=0|" "base|PR_X=0|libpertrender_base" || exit 1
