# bench sweeps over tuning env vars (no profiler): prints ms/step and kernel times
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
cd "$R"
run() {
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-dense --steps 30 --warmup 5 > "$OUT/sw.json" 2> "$OUT/sw.err" || { echo "FAIL $*"; tail -3 "$OUT/sw.err"; return 1; }
  python -c "import json;d=json.load(open('$OUT/sw.json'));print('$*', d['ms_per_step'], {k:v['ms'] for k,v in d['kernels'].items()})"
}
for r in 2 1 4; do run PR_RAST_BWD_ROWS=$r || exit 1; done
