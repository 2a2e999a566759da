set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG="${1:-bp}"
cd "$R"
PR_NATIVE_LIB=$R/pertrenderer_amd/libpertrender_prof.so timeout -k 10 120 python tools/rast_prof.py > "$OUT/prof_$TAG.log" 2>&1
rc=$?; echo "prof rc=$rc"; grep "^fwd blk" "$OUT/prof_$TAG.log" | head -8; grep "^bwd blk" "$OUT/prof_$TAG.log" | head -8; grep "^bwd tile" "$OUT/prof_$TAG.log" | sort -t'|' -k2 | tail -4
exit $rc
