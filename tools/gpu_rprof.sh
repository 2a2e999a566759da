# rasterizer phase profile (-DPR_RAST_PROFILE variant) for each wave count
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG="${1:-rp}"
cd "$R"
for w in ${WVS:-1 2 4}; do
  PR_RAST_WAVES=$w PR_NATIVE_LIB=$R/pertrenderer_amd/libpertrender_prof.so timeout -k 10 120 python tools/rast_prof.py > "$OUT/rprof_${TAG}_$w.log" 2>&1
  rc=$?; echo "WV=$w rc=$rc"; grep "^tile" "$OUT/rprof_${TAG}_$w.log" | sort -t'|' -k2 | tail -3
  [ $rc -ne 0 ] && exit $rc
done
exit 0
