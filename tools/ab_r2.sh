# Same-lease A/B of the cfg 2 headline: A = round-2 HEAD (f965279, a worktree at ./ab_r2 built in this
# container: git worktree add ab_r2 f965279 && (cd ab_r2 && python -c "import __graft_entry__ as g; g.build()")),
# B = this tree.  bench.py --steps 50 --warmup 10, alternating A B A B A B, each under its own timeout.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/ab"; mkdir -p "$OUT"
for i in 1 2 3; do
  for side in A B; do
    if [ $side = A ]; then d="$R/ab_r2"; else d="$R"; fi
    (cd "$d" && timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-dense \
       > "$OUT/${side}_$i.json" 2> "$OUT/${side}_$i.err") || { echo "FAIL $side $i"; tail -3 "$OUT/${side}_$i.err"; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'])" "$OUT/${side}_$i.json" "$side$i"
  done
done
# kernel level: rocprofv3 --kernel-trace --stats of each side's bench (200 steps)
for side in A B; do
  if [ $side = A ]; then d="$R/ab_r2"; else d="$R"; fi
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$side" -o p -- \
     python "$d/bench.py" --steps 200 --warmup 20 --no-cpu-baseline --no-dense > "$OUT/prof_$side.json" 2> "$OUT/prof_$side.err") \
     || { echo "FAIL prof $side"; tail -3 "$OUT/prof_$side.err"; exit 1; }
  find "$OUT/prof_$side" -name "*kernel_trace.csv" -delete
done
echo prof done
