# Blend phase profiles of the in-tree profiling build vs LIB_B (default the previous commit's
# profiling build), CONFIG (default cfg2) (run through gpurun).
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/abprof"; mkdir -p "$OUT"
cd "$R"
B="${LIB_B:-$R/pertrenderer_amd/libpertrender_oldprof.so}"; C="${CONFIG:-cfg2}"
for v in new old new old; do
  L="$R/pertrenderer_amd/libpertrender_prof.so"; [ $v = old ] && L="$B"
  PR_NATIVE_LIB=$L timeout -k 10 200 python tools/blend_prof.py --config $C > "$OUT/$v.log" 2>&1 || { tail -5 "$OUT/$v.log"; exit 1; }
  echo "== $v"; grep -A 2 "^blend_" "$OUT/$v.log" | grep -v histogram
done
