# rasterizer per-tile timeline + phase profile (-DPR_RAST_PROFILE variant) per slice count
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG="${1:-rp}"; shift || true
cd "$R"
for cfg in "$@"; do
  env $cfg PR_NATIVE_LIB=$R/pertrenderer_amd/libpertrender_prof.so timeout -k 10 120 python tools/rast_prof.py "$OUT/rprof_${TAG}_${cfg// /_}.npy" > "$OUT/rprof_${TAG}_${cfg// /_}.log" 2>&1
  rc=$?; echo "$cfg rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$OUT/rprof_${TAG}_${cfg// /_}.log"; exit $rc; }
done
exit 0
