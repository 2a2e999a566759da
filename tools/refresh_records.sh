# Copy a `tools/gpu.sh final TAG` run's outputs (merged under gpurun_out/) into the committed round-4
# records: profiles/r4_final/*, profiles/rocprof_kernels.json, profiles/pmc_traffic.json.
#   bash tools/refresh_records.sh TAG
set -eu
T="$1"; O=gpurun_out; F=profiles/r4_final
for k in "" eager_ eager_blocking_ eval_ cfg3_ cfg4_ eager_eval_; do cp "$O/bench_${k}$T.json" "$F/bench_${k}r4.json"; done
cp "$O/launch_blocking_$T.txt" "$F/launch_blocking_r4.txt"
cp "$O/pmc_summary_pmc_$T.txt" "$F/pmc_summary_pmc_r4.txt"
cp "$O/tests_$T.log" "$F/tests_r4.log"; cp "$O/smoke_$T.log" "$F/smoke_r4.log"
cp "$(find "$O/prof_$T" -name '*kernel_stats.csv' | sort | head -n 1)" "$F/graph_kernel_stats.csv"
tail -n 1 "$O/cfg5_$T.log" > "$F/cfg5.json"
cp "$O/rocprof_kernels_$T.json" profiles/rocprof_kernels.json
cp "$O/pmc_traffic_pmc_$T.json" profiles/pmc_traffic.json
python - <<'PY'
import json
for f in ("profiles/rocprof_kernels.json", "profiles/pmc_traffic.json"):
    print(f, json.load(open(f)).get("source_sha"))
PY
