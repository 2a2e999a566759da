# blend LDS-target sweep at cfg2 (resident blocks vs passes)
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; cd "$R"
run() {
  env $2 timeout -k 10 200 python bench.py --config $3 --no-cpu-baseline --no-dense --steps 30 > $OUT/b2s_$1_$3.json 2>> $OUT/b2s.err || exit 1
  python -c "import json;d=json.load(open('$OUT/b2s_$1_$3.json'));k=d['kernels'];print('$1 $3',d['value'],k['blend_fwd']['ms'],k['blend_bwd']['ms'])"
}
run base PR_X=0 cfg2
run f16 PR_BLEND_LDS_KB_FWD=16 cfg2
run f12 PR_BLEND_LDS_KB_FWD=12 cfg2
run f8 PR_BLEND_LDS_KB_FWD=8 cfg2
run b20 PR_BLEND_LDS_KB_BWD=20 cfg2
run b16 PR_BLEND_LDS_KB_BWD=16 cfg2
run b12 PR_BLEND_LDS_KB_BWD=12 cfg2
run fpb16 PR_BLEND_PB_FWD=16 cfg2
run fpb16f12 "PR_BLEND_PB_FWD=16 PR_BLEND_LDS_KB_FWD=12" cfg2
run base2 PR_X=0 cfg2
