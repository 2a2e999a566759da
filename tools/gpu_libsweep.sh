# bench over (library x env) at CONFIGS (default "cfg2 cfg4"): LIBS = in-tree .so names,
# ENVS = env settings ("X=0" = none) (run through gpurun).
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
cd "$R"
for C in ${CONFIGS:-cfg2 cfg4}; do
  for L in $LIBS; do
    for E in "$@"; do
      env $E PR_NATIVE_LIB=$R/pertrenderer_amd/$L timeout -k 10 200 python bench.py --config $C --no-cpu-baseline --no-dense --steps 20 --warmup 5 > "$OUT/ls.json" 2> "$OUT/ls.err" || { echo "FAIL $L $E"; tail -3 "$OUT/ls.err"; exit 1; }
      python -c "import json;d=json.load(open('$OUT/ls.json'));print('$C $L $E', d['value'], {k:v['ms'] for k,v in d['kernels'].items() if k.startswith('blend')})"
    done
  done
done
