# rasterizer compile-variant sweep: bench kernel times per library (PR_NATIVE_LIB)
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; cd "$R"
for v in libpertrender libpr_v1 libpr_v2 libpr_v3; do
  for c in cfg2 cfg4; do
    PR_NATIVE_LIB=$R/pertrenderer_amd/$v.so timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-dense --steps 20 > $OUT/sw_${v}_$c.json 2>> $OUT/sw.err || exit 1
    python -c "import json;d=json.load(open('$OUT/sw_${v}_$c.json'));print('$v $c',d['value'],d['ms_per_step'],{k:v['ms'] for k,v in d['kernels'].items()})"
  done
done
