# bench sweeps over tuning env vars on a batch configuration:
#   bash tools/gpu_sweep_cfg.sh cfg3 "PR_BLEND_LPP=16" ...
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; CFG="$1"; shift
cd "$R"
for cfg in "$@"; do
  env $cfg timeout -k 10 300 python bench.py --config "$CFG" --no-cpu-baseline --no-dense --steps 10 --warmup 3 > "$OUT/swc.json" 2> "$OUT/swc.err" || { echo "FAIL $cfg"; tail -3 "$OUT/swc.err"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/swc.json'));print('$CFG $cfg', d['ms_per_step'], {k:v['ms'] for k,v in d['kernels'].items()})"
done
