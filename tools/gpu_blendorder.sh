# blend block order / lanes-per-pixel sweep at cfg3 / cfg4 (runtime knobs)
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; cd "$R"
run() {
  env $2 timeout -k 10 200 python bench.py --config $3 --no-cpu-baseline --no-dense --steps 10 --warmup 3 > $OUT/bo_$1_$3.json 2>> $OUT/bo.err || exit 1
  python -c "import json;d=json.load(open('$OUT/bo_$1_$3.json'));k=d['kernels'];print('$1 $3',d['value'],k['blend_fwd']['ms'],k['blend_bwd']['ms'])"
}
for c in cfg4 cfg3; do
  run o1 PR_X=0 $c
  run o0 PR_BLEND_ORDER=0 $c
  run o3 PR_BLEND_ORDER=3 $c
  run o2 PR_BLEND_ORDER=2 $c
  run l16 PR_BLEND_LPP=16 $c
  run l32 PR_BLEND_LPP=32 $c
done
