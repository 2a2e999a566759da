# multi-device tests, cfg3/cfg4 bench, PMC passes
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG="${1:-b2}"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_multidevice.py > "$OUT/md_$TAG.log" 2>&1
rc=$?; tail -n 15 "$OUT/md_$TAG.log"; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
for c in cfg3 cfg4; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dense --steps 20 > "$OUT/bench_${TAG}_$c.json" 2>> "$OUT/bench_$TAG.err" || exit 1
  python -c "import json;d=json.load(open('$OUT/bench_${TAG}_$c.json'));print('$c',d['value'],d['ms_per_step'],{k:v['ms'] for k,v in d['kernels'].items()})"
done
bash tools/gpu_pmc.sh pmc_$TAG || exit 1
python tools/pmc_summary.py $OUT/pmc_${TAG}_p* --traffic-out $OUT/pmc_traffic_$TAG.json > $OUT/pmc_summary_$TAG.txt 2>&1; echo pmcsum rc=$?
head -40 $OUT/pmc_summary_$TAG.txt
