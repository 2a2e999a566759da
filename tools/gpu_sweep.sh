# bench sweeps over tuning env vars (no profiler): prints ms/step and kernel times.
#   bash tools/gpu_sweep.sh "PR_RAST_BWD_ROWS=4" "PR_RAST_BWD_ROWS=8" ...
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
cd "$R"
run() {
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-dense --steps 30 --warmup 5 > "$OUT/sw.json" 2> "$OUT/sw.err" || { echo "FAIL $*"; tail -3 "$OUT/sw.err"; return 1; }
  python -c "import json;d=json.load(open('$OUT/sw.json'));print('$*', d['ms_per_step'], {k:v['ms'] for k,v in d['kernels'].items()})"
}
for cfg in "$@"; do run $cfg || exit 1; done
