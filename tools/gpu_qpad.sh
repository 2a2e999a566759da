# queue-padding variants + rast_bwd rows default: rasterizer tests, cfg2 / cfg4 kernel times
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rast.py tests/test_gpu_fullsize.py > "$OUT/rt_q.log" 2>&1
rc=$?; tail -n 2 "$OUT/rt_q.log"; [ $rc -ne 0 ] && exit $rc
for c in cfg2 cfg4; do
  for v in libpertrender libpr_q1 libpr_q2 libpertrender; do
    PR_NATIVE_LIB=$R/pertrenderer_amd/$v.so timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-dense --steps 20 > $OUT/q_${v}_$c.json 2>> $OUT/q.err || exit 1
    python -c "import json;d=json.load(open('$OUT/q_${v}_$c.json'));k=d['kernels'];print('$v $c',d['value'],k['rast_fwd']['ms'],k['rast_fwd']['ms_median'],k['rast_bwd']['ms'])"
  done
done
