# rast_bwd rows-per-tile sweep at cfg3 / cfg4 (runtime knob PR_RAST_BWD_ROWS)
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; cd "$R"
for c in cfg4 cfg3; do
  for r in 2 1 4 8; do
    PR_RAST_BWD_ROWS=$r timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --no-dense --steps 10 --warmup 3 > $OUT/br_${r}_$c.json 2>> $OUT/br.err || exit 1
    python -c "import json;d=json.load(open('$OUT/br_${r}_$c.json'));k=d['kernels'];print('rows $r $c',d['value'],k['rast_bwd']['ms'])"
  done
done
