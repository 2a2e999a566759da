# Round-end refresh of every measured artefact, in dependency order:
#   PMC passes -> profiles/pmc_traffic.json (read by bench.py's roofline.traffic) ->
#   GPU tests -> bench (graph) + eager bench + rocprofv3 kernel trace of the bench ->
#   batch-config bench lines.  Copy gpurun_out/* of TAG into profiles/ afterwards.
#     bash tools/gpu_refresh.sh TAG
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG="${1:-rf}"
cd "$R"
bash tools/gpu_pmc.sh "pmc_$TAG" || exit $?
python tools/pmc_summary.py "$OUT/pmc_${TAG}_p1" "$OUT/pmc_${TAG}_p2" "$OUT/pmc_${TAG}_p3" "$OUT/pmc_${TAG}_p4" \
  --traffic-out "$OUT/pmc_traffic_$TAG.json" > "$OUT/pmc_counters_$TAG.txt" || exit $?
cp "$OUT/pmc_traffic_$TAG.json" profiles/pmc_traffic.json
bash tools/gpu_test_bench.sh "$TAG" || exit $?
cd "$R"
bash tools/gpu_configs.sh "$TAG" || exit $?
exit 0
