# round 4: HIP runtime knobs for the launch floor (HIP_FORCE_DEV_KERNARG) -- probe + cfg2 / eager rows
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out/r4p
timeout -k 10 120 python tools/launch_overhead.py > gpurun_out/r4p/lo_base.json 2>&1 || exit 1
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 120 python tools/launch_overhead.py > gpurun_out/r4p/lo_devkernarg.json 2>&1 || exit 1
cat gpurun_out/r4p/lo_base.json gpurun_out/r4p/lo_devkernarg.json | grep -v amdgpu
bash tools/gpu.sh sweep r4p cfg2 "base|PR_X=0|" "dka|HIP_FORCE_DEV_KERNARG=1|" "base2|PR_X=0|" "dka2|HIP_FORCE_DEV_KERNARG=1|" || exit 1
bash tools/gpu.sh bench eager_base_r4p --mode eager --no-cpu-baseline --no-dense || exit 1
HIP_FORCE_DEV_KERNARG=1 bash tools/gpu.sh bench eager_dka_r4p --mode eager --no-cpu-baseline --no-dense || exit 1
