set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/reuse
timeout -k 10 200 python tools/scratch/reuse_main.py n3 --mode graph -np 3 > gpurun_out/reuse/main_n3.log 2>&1
timeout -k 10 200 python tools/scratch/reuse_main.py r3 --mode graph -np 3 --graph-reuse > gpurun_out/reuse/main_r3.log 2>&1
timeout -k 10 200 python tools/scratch/reuse_main.py n30 --mode graph -np 30 > gpurun_out/reuse/main_n30.log 2>&1
timeout -k 10 200 python tools/scratch/reuse_main.py r30 --mode graph -np 30 --graph-reuse > gpurun_out/reuse/main_r30.log 2>&1
