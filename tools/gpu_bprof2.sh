# blend per-block phase profile (cfg2, cfg4) with the -DPR_BLEND_PROFILE variant
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; cd "$R"
for c in cfg2 cfg4; do
  PR_NATIVE_LIB=$R/pertrenderer_amd/libpertrender_bprof.so timeout -k 10 200 python tools/blend_prof.py --config $c > $OUT/bprof_$c.log 2>&1 || { tail -5 $OUT/bprof_$c.log; exit 1; }
  tail -n 30 $OUT/bprof_$c.log
done
