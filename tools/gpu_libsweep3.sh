# rasterizer: parity tests on the product build, then slice-count / chunk variants at cfg2 and cfg4
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_rast.py tests/test_gpu_rast_kat.py tests/test_gpu_fullsize.py > "$OUT/rt_s3.log" 2>&1
rc=$?; tail -n 2 "$OUT/rt_s3.log"; [ $rc -ne 0 ] && exit $rc
run() {  # tag env lib config
  env $2 PR_NATIVE_LIB=$R/pertrenderer_amd/$3.so timeout -k 10 200 python bench.py --config $4 --no-cpu-baseline --no-dense --steps 20 > $OUT/s3_$1_$4.json 2>> $OUT/s3.err || exit 1
  python -c "import json;d=json.load(open('$OUT/s3_$1_$4.json'));print('$1 $4',d['value'],d['ms_per_step'],{k:v['ms'] for k,v in d['kernels'].items()})"
}
for c in cfg2 cfg4; do
  run ch16 PR_X=0 libpertrender $c
  run sl8 PR_RAST_SLICES=8 libpertrender $c
  run sl2 PR_RAST_SLICES=2 libpertrender $c
  run ch8 PR_X=0 libpr_v4 $c
done
