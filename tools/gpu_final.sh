# round-end measurement: GPU suite, smoke, bench lines (graph + CPU baseline, eager, eval row, cfg3, cfg4),
# rocprofv3 kernel stats of the bench command, PMC passes and their summary
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG="${1:-fin}"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests_$TAG.log" 2>&1
rc=$?; grep -E "passed|failed" "$OUT/tests_$TAG.log" | tail -3; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1 || { tail -5 "$OUT/smoke_$TAG.log"; exit 1; }
tail -n 1 "$OUT/smoke_$TAG.log"
timeout -k 10 600 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || exit 1
python -c "import json;d=json.load(open('$OUT/bench_$TAG.json'));print('graph',d['value'],d['ms_per_step'],{k:v['ms'] for k,v in d['kernels'].items()},d['roofline']['kernel'],d['roofline']['frac'],d['cpu_baseline']['value'])"
timeout -k 10 300 python bench.py --mode eager --no-cpu-baseline --no-dense > "$OUT/bench_eager_$TAG.json" 2>> "$OUT/bench_$TAG.err" || exit 1
timeout -k 10 300 python bench.py --config eval --no-cpu-baseline --no-dense > "$OUT/bench_eval_$TAG.json" 2>> "$OUT/bench_$TAG.err" || exit 1
for c in cfg3 cfg4; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dense > "$OUT/bench_${c}_$TAG.json" 2>> "$OUT/bench_$TAG.err" || exit 1
done
for f in eager eval cfg3 cfg4; do python -c "import json;d=json.load(open('$OUT/bench_${f}_$TAG.json'));print('$f',d['value'],d['ms_per_step'],{k:v['ms'] for k,v in d['kernels'].items()})"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o prof -- \
  python "$R/bench.py" --no-cpu-baseline --no-dense > "$OUT/bench_prof_$TAG.json" 2> "$OUT/prof_$TAG.err" || exit 1
echo rocprof ok
cd "$R"
bash tools/gpu_pmc.sh pmc_$TAG || exit 1
python tools/pmc_summary.py $OUT/pmc_${TAG}_p* --traffic-out $OUT/pmc_traffic_$TAG.json > $OUT/pmc_summary_$TAG.txt 2>&1; echo pmcsum rc=$?
