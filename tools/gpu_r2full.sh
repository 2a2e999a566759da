# full GPU suite, smoke, bench (graph with CPU baseline, eager, eval row), rocprofv3 kernel stats of the bench
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG="${1:-full}"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests_$TAG.log" 2>&1
rc=$?; grep -E "passed|failed|Error" "$OUT/tests_$TAG.log" | tail -12
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1 || { tail -5 "$OUT/smoke_$TAG.log"; exit 1; }
tail -n 1 "$OUT/smoke_$TAG.log"
timeout -k 10 600 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || exit 1
python -c "import json;d=json.load(open('$OUT/bench_$TAG.json'));print('graph',d['value'],d['ms_per_step'],{k:v['ms'] for k,v in d['kernels'].items()},d['roofline']['frac'],d['cpu_baseline']['value'])"
timeout -k 10 300 python bench.py --mode eager --no-cpu-baseline --no-dense > "$OUT/bench_eager_$TAG.json" 2>> "$OUT/bench_$TAG.err" || exit 1
python -c "import json;d=json.load(open('$OUT/bench_eager_$TAG.json'));print('eager',d['value'],d['ms_per_step'])"
timeout -k 10 300 python bench.py --config eval --no-cpu-baseline --no-dense > "$OUT/bench_eval_$TAG.json" 2>> "$OUT/bench_$TAG.err" || exit 1
python -c "import json;d=json.load(open('$OUT/bench_eval_$TAG.json'));print('eval',d['value'],d['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o prof -- \
  python "$R/bench.py" --no-cpu-baseline --no-dense > "$OUT/bench_prof_$TAG.json" 2> "$OUT/prof_$TAG.err"
rc=$?; echo "rocprof rc=$rc"
exit $rc
