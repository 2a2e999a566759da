# smoke + GPU tests + graph bench (no profiler)
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG="${1:-q}"
cd "$R"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$OUT/smoke_$TAG.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 180 -p no:cacheprovider > "$OUT/tests_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" "$OUT/tests_$TAG.log" | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python "$R/bench.py" --no-cpu-baseline > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench_$TAG.err"
python -c "import json;d=json.load(open('$OUT/bench_$TAG.json'));print(d['value'],d['ms_per_step'],d['config']['execution'],d.get('note'));print({k:v['ms'] for k,v in d['kernels'].items()});print({k:(v['ms'],v['frac']) for k,v in d['roofline_dense'].items()})"
exit $rc
