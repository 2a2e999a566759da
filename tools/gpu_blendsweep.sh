# blend shape sweep at cfg4 / cfg3 (runtime knobs: LDS target and pixels per block)
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; cd "$R"
run() {  # tag env config
  env $2 timeout -k 10 200 python bench.py --config $3 --no-cpu-baseline --no-dense --steps 10 --warmup 3 > $OUT/bs_$1_$3.json 2>> $OUT/bs.err || exit 1
  python -c "import json;d=json.load(open('$OUT/bs_$1_$3.json'));k=d['kernels'];print('$1 $3',d['value'],k['rast_fwd']['ms'],k['blend_fwd']['ms'],k['blend_bwd']['ms'])"
}
for c in cfg4 cfg3; do
  run base PR_X=0 $c
  run b12 PR_BLEND_LDS_KB_BWD=12 $c
  run b16 PR_BLEND_LDS_KB_BWD=16 $c
  run b32 PR_BLEND_LDS_KB_BWD=32 $c
  run pb16 PR_BLEND_PB_BWD=16 $c
  run pb8 PR_BLEND_PB_BWD=8 $c
  run f12 PR_BLEND_LDS_KB_FWD=12 $c
  run f32 PR_BLEND_LDS_KB_FWD=32 $c
  run fpb16 PR_BLEND_PB_FWD=16 $c
done
run sl4 PR_RAST_SLICES=4 cfg3
