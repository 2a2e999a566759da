# Same-lease A/B of two trees' bench lines and rocprofv3 kernel stats (through gpurun):
#   bash tools/ab.sh TAG DIR_A DIR_B [ROUNDS] [bench.py args]
# DIR_A / DIR_B are repository trees with their own built libpertrender.so (e.g. a git worktree of an
# older HEAD under ab_r2/). Each round runs A then B (bench line, then a rocprofv3 --stats pass), so box
# drift shows up as A/A and B/B spread. Outputs: gpurun_out/ab_TAG/{A,B}_r<i>.json, {A,B}_prof_r<i>/.
set -u
R="$GRAFT_REPO_ROOT"; TAG="$1"; A="$2"; B="$3"; ROUNDS="${4:-2}"; shift 4 || shift $#
OUT="$R/gpurun_out/ab_$TAG"; mkdir -p "$OUT"
for i in $(seq 1 "$ROUNDS"); do
  for side in A B; do
    d="$A"; [ "$side" = B ] && d="$B"
    (cd "$R/$d" && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dense "$@" \
       > "$OUT/${side}_r$i.json" 2> "$OUT/${side}_r$i.err") || { echo "bench $side r$i failed"; tail -5 "$OUT/${side}_r$i.err"; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'], {k:v['ms'] for k,v in d['kernels'].items()})" "$OUT/${side}_r$i.json" "$side r$i"
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
       -d "$OUT/${side}_prof_r$i" -o prof -- python "$R/$d/bench.py" --steps 200 --warmup 20 --no-cpu-baseline --no-dense "$@" \
       > "$OUT/${side}_prof_r$i.json" 2> "$OUT/${side}_prof_r$i.err") || { echo "prof $side r$i failed"; tail -5 "$OUT/${side}_prof_r$i.err"; exit 1; }
    f=$(find "$OUT/${side}_prof_r$i" -name "*kernel_stats.csv" | sort | sed -n 1p)
    python - "$f" "$side r$i" <<'EOF'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2], {r["Name"].split("(")[0][-40:]: round(float(r["AverageNs"]) / 1e3, 1) for r in rows[:8]})
EOF
  done
done
