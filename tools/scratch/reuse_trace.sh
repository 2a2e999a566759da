set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/reuse
for m in new ses ses_warm; do timeout -k 10 200 python tools/scratch/reuse_trace.py $m softras > gpurun_out/reuse/trace_$m.log 2>&1; done
for m in new ses; do timeout -k 10 200 python tools/scratch/reuse_trace.py $m softras,gaussian > gpurun_out/reuse/trace2_$m.log 2>&1; done
