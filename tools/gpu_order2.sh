# blend order default check: blend tests, cfg2 / cfg3 / cfg4 bench
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_blend.py tests/test_gpu_fullsize.py tests/test_gpu_counts.py > "$OUT/bt_o.log" 2>&1
rc=$?; tail -n 2 "$OUT/bt_o.log"; [ $rc -ne 0 ] && exit $rc
for c in cfg2 cfg3 cfg4; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dense > "$OUT/bench_${c}_o.json" 2>> "$OUT/bo2.err" || exit 1
  python -c "import json;d=json.load(open('$OUT/bench_${c}_o.json'));print('$c',d['value'],d['ms_per_step'],{k:v['ms'] for k,v in d['kernels'].items()})"
done
