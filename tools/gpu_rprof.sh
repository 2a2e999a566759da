set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG="${1:-rp}"
cd "$R"
PR_NATIVE_LIB=$R/pertrenderer_amd/libpertrender_prof.so timeout -k 10 120 python tools/rast_prof.py > "$OUT/rast_prof_$TAG.log" 2>&1
rc=$?; echo "rast_prof rc=$rc"; grep "^tile" "$OUT/rast_prof_$TAG.log" | sort -t'|' -k2 | tail -3; grep "^bwd" "$OUT/rast_prof_$TAG.log" | sort -t'|' -k2 | tail -8
exit $rc
