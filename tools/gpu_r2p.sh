set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; cd "$R"
PR_NATIVE_LIB=$R/pertrenderer_amd/libpertrender_prof.so timeout -k 10 120 python tools/rast_prof.py $OUT/rp_a.npy > $OUT/rp_a.log 2>&1 || exit 1
python tools/rast_timeline.py $OUT/rp_a.npy
timeout -k 10 200 python tools/eager_host_prof.py 50 > $OUT/eager_prof.log 2>&1; echo eager rc=$?
