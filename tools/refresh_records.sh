# Copy a `tools/gpu.sh final TAG` (+ `final2 TAG`) run's outputs (merged under gpurun_out/) into the
# committed records: profiles/<DEST>/*, profiles/rocprof_kernels.json, profiles/pmc_traffic.json
# (and, after final2, profiles/rocprof_dense.json).
#   bash tools/refresh_records.sh TAG [DEST]        (DEST default: r6_final)
set -eu
T="$1"; D="${2:-r6_final}"; O=gpurun_out; F="profiles/$D"
mkdir -p "$F"
for k in "" eager_ eager_blocking_ eval_ cfg3_ cfg4_ eager_eval_; do
  [ -f "$O/bench_${k}$T.json" ] && cp "$O/bench_${k}$T.json" "$F/bench_${k}$T.json"
done
[ -f "$O/launch_blocking_$T.txt" ] && cp "$O/launch_blocking_$T.txt" "$F/"
[ -f "$O/pmc_summary_pmc_$T.txt" ] && cp "$O/pmc_summary_pmc_$T.txt" "$F/"
cp "$O/tests_$T.log" "$F/"; cp "$O/smoke_$T.log" "$F/"
cp "$(find "$O/prof_$T" -name '*kernel_stats.csv' | sort | head -n 1)" "$F/graph_kernel_stats_$T.csv"
cp "$O/cfg5_$T.log" "$F/"
cp "$O/rocprof_kernels_$T.json" profiles/rocprof_kernels.json
cp "$O/pmc_traffic_pmc_$T.json" profiles/pmc_traffic.json
for f in bench_eager_blocking_eval_$T.json cfg5_eager_$T.log cfg5_eager_blocking_$T.log; do
  [ -f "$O/$f" ] && cp "$O/$f" "$F/"
done
if [ -f "$O/rocprof_dense_$T.json" ]; then cp "$O/rocprof_dense_$T.json" profiles/rocprof_dense.json; fi
if [ -f "$O/pmc_traffic_pmcdense_$T.json" ]; then cp "$O/pmc_traffic_pmcdense_$T.json" profiles/pmc_dense.json; fi
python - <<'PY'
import json, os
for f in ("profiles/rocprof_kernels.json", "profiles/pmc_traffic.json", "profiles/rocprof_dense.json",
          "profiles/pmc_dense.json"):
    if os.path.exists(f):
        print(f, json.load(open(f)).get("source_sha"))
PY
