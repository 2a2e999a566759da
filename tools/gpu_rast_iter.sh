# rasterizer iteration: parity tests, per-tile profile (-DPR_RAST_PROFILE variant), bench kernel times
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG="${1:-ri}"
cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_rast.py tests/test_gpu_rast_kat.py tests/test_gpu_fullsize.py tests/test_gpu_counts.py > "$OUT/rt_$TAG.log" 2>&1
rc=$?; tail -n 4 "$OUT/rt_$TAG.log"; [ $rc -ne 0 ] && exit $rc
PR_NATIVE_LIB=$R/pertrenderer_amd/libpertrender_prof.so timeout -k 10 120 python tools/rast_prof.py $OUT/rp_$TAG.npy > $OUT/rp_$TAG.log 2>&1 || exit 1
python tools/rast_timeline.py $OUT/rp_$TAG.npy
timeout -k 10 300 python bench.py --no-cpu-baseline --no-dense > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err" || exit 1
python -c "import json;d=json.load(open('$OUT/bench_$TAG.json'));print(d['value'],d['ms_per_step']);print({k:v['ms'] for k,v in d['kernels'].items()})"
PR_RAST_BINS=0 timeout -k 10 300 python bench.py --no-cpu-baseline --no-dense > "$OUT/bench_${TAG}_nobins.json" 2>> "$OUT/bench_$TAG.err" || exit 1
python -c "import json;d=json.load(open('$OUT/bench_${TAG}_nobins.json'));print('nobins',d['value'],d['ms_per_step']);print({k:v['ms'] for k,v in d['kernels'].items()})"
