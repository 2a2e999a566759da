set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
cd "$R"
PR_NATIVE_LIB=$R/pertrenderer_amd/libpertrender_prof.so timeout -k 10 120 python tools/rast_prof.py > "$OUT/rast_prof_r2b.log" 2>&1
rc=$?; echo "rast_prof rc=$rc"; sort -t'|' -k2 "$OUT/rast_prof_r2b.log" | tail -12
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_quick.sh r2b
