# rasterizer tile order on batches (PR_RAST_ORDER: bit 0 forward ring, bit 1 backward centre-out rows)
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; cd "$R"
for c in cfg4 cfg3; do
  for o in 3 0 1 2; do
    PR_RAST_ORDER=$o timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-dense --steps 10 --warmup 3 > $OUT/ro_${o}_$c.json 2>> $OUT/ro.err || exit 1
    python -c "import json;d=json.load(open('$OUT/ro_${o}_$c.json'));k=d['kernels'];print('order $o $c',d['value'],k['rast_fwd']['ms'],k['rast_bwd']['ms'])"
  done
done
