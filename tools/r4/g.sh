# round 4: full GPU suite through the C++ layer, eager rows C++ vs Python layer (alternating)
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"
bash tools/gpu.sh tests r4g || exit 1
for i in 1 2; do
  bash tools/gpu.sh bench "eager_cpp_r4g$i" --mode eager --no-cpu-baseline --no-dense || exit 1
  PR_TORCH_EXT=0 bash tools/gpu.sh bench "eager_py_r4g$i" --mode eager --no-cpu-baseline --no-dense || exit 1
done
HIP_LAUNCH_BLOCKING=1 bash tools/gpu.sh bench eager_blocking_cpp_r4g --mode eager --no-cpu-baseline --no-dense || exit 1
HIP_LAUNCH_BLOCKING=1 PR_TORCH_EXT=0 bash tools/gpu.sh bench eager_blocking_py_r4g --mode eager --no-cpu-baseline --no-dense || exit 1
bash tools/gpu.sh bench eager_eval_cpp_r4g --config eval --mode eager --no-cpu-baseline --no-dense || exit 1
