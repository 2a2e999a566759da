# bench lines for the batch configurations (cfg3, cfg4) on one GPU
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG="${1:-cf}"
cd "$R"
for c in cfg3 cfg4; do
  timeout -k 10 400 python -u bench.py --config $c --steps ${STEPS:-10} --warmup 3 > "$OUT/bench_${c}_$TAG.json" 2> "$OUT/bench_${c}_$TAG.err"
  rc=$?; echo "$c rc=$rc"; cut -c1-600 "$OUT/bench_${c}_$TAG.json"; tail -3 "$OUT/bench_${c}_$TAG.err"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
