# Interleaved bench A/B of two native libraries on one box: LIB_B (default libpertrender_old.so)
# against the in-tree build, CONFIG (default cfg2), 3 rounds (run through gpurun).
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/ablib"; mkdir -p "$OUT"
cd "$R"
B="${LIB_B:-$R/pertrenderer_amd/libpertrender_old.so}"; C="${CONFIG:-cfg2}"
for i in 1 2 3; do
  for v in new old; do
    L="$R/pertrenderer_amd/libpertrender.so"; [ $v = old ] && L="$B"
    PR_NATIVE_LIB=$L timeout -k 10 200 python bench.py --config $C --no-cpu-baseline --no-dense > "$OUT/$v$i.json" 2> "$OUT/$v$i.err" || { tail -5 "$OUT/$v$i.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_forward'], d['ms_backward'], {k: v['ms'] for k, v in d['kernels'].items()})" "$OUT/$v$i.json" $v
  done
done
