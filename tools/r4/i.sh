# round 4: low-priority scalar link node, fused finalize by default: tests + eager / graph rows
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_host_layer.py tests/test_gpu_fused_finalize.py tests/test_gpu_scalar_link.py tests/test_gpu_shading.py \
  tests/test_gpu_once_differentiable.py tests/test_gpu_blend.py > gpurun_out/tests_r4i.log 2>&1
rc=$?; tail -n 3 gpurun_out/tests_r4i.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  bash tools/gpu.sh bench "eager_cpp_r4i$i" --mode eager --no-cpu-baseline --no-dense || exit 1
done
HIP_LAUNCH_BLOCKING=1 bash tools/gpu.sh bench eager_blocking_cpp_r4i --mode eager --no-cpu-baseline --no-dense || exit 1
bash tools/gpu.sh bench eager_eval_cpp_r4i --config eval --mode eager --no-cpu-baseline --no-dense || exit 1
bash tools/gpu.sh bench graph_r4i --no-cpu-baseline --no-dense || exit 1
