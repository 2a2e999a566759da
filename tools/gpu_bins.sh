# coarse bins: rasterizer parity tests, bins timing tool, cfg2 / cfg4 bench with and without bins, eager host profile
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG="${1:-bn}"
cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_rast.py tests/test_gpu_rast_kat.py tests/test_gpu_fullsize.py > "$OUT/rt_$TAG.log" 2>&1
rc=$?; tail -n 4 "$OUT/rt_$TAG.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/rast_bins_bench.py "$OUT/bins_$TAG.json" > "$OUT/bins_$TAG.log" 2>&1; rc=$?
cat "$OUT/bins_$TAG.log" | grep faces; [ $rc -ne 0 ] && exit $rc
for c in cfg2 cfg4; do
  for b in 0 1; do
    PR_RAST_BINS=$b timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-dense --steps 20 > "$OUT/bench_${TAG}_${c}_$b.json" 2>> "$OUT/bench_$TAG.err" || exit 1
    python -c "import json;d=json.load(open('$OUT/bench_${TAG}_${c}_$b.json'));print('$c bins=$b',d['value'],d['ms_per_step'],{k:v['ms'] for k,v in d['kernels'].items()})"
  done
done
timeout -k 10 200 python tools/eager_host_prof.py 50 > $OUT/eager_prof.log 2>&1; echo eager rc=$?
