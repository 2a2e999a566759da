# bench sweeps over tuning env vars at one config (no profiler):
#   CONFIG=cfg4 bash tools/gpu_sweep_cfg.sh "PR_BLEND_LDS_KB_FWD=24" "PR_BLEND_LDS_KB_FWD=48" ...
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
cd "$R"
C="${CONFIG:-cfg2}"
run() {
  env "$@" timeout -k 10 200 python bench.py --config $C --no-cpu-baseline --no-dense --steps 20 --warmup 5 > "$OUT/sw.json" 2> "$OUT/sw.err" || { echo "FAIL $*"; tail -3 "$OUT/sw.err"; return 1; }
  python -c "import json;d=json.load(open('$OUT/sw.json'));print('$C $*', d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['kernels'].items()})"
}
for cfg in "$@"; do run $cfg || exit 1; done
