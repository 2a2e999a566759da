# A/B of the backward's masked-tail draw (PR_BLEND_TAIL=1 default vs 0): blend phase
# profiles at cfg2 / cfg4 and interleaved cfg2 bench lines on one box (run through gpurun).
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/tail_ab"; mkdir -p "$OUT"
cd "$R"
for c in cfg2 cfg4; do
  for t in 1 0; do
    PR_BLEND_TAIL=$t PR_NATIVE_LIB=$R/pertrenderer_amd/libpertrender_prof.so timeout -k 10 200 \
      python tools/blend_prof.py --config $c > "$OUT/bprof_${c}_t$t.log" 2>&1 || { tail -20 "$OUT/bprof_${c}_t$t.log"; exit 1; }
    echo "== $c tail=$t"; grep -A 2 blend_bwd "$OUT/bprof_${c}_t$t.log"
  done
done
for i in 1 2; do
  for t in 1 0; do
    PR_BLEND_TAIL=$t timeout -k 10 200 python bench.py --no-cpu-baseline --no-dense > "$OUT/b_t${t}_$i.json" 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('tail', sys.argv[2], d['value'], {k: v['ms'] for k, v in d['kernels'].items()})" "$OUT/b_t${t}_$i.json" $t
  done
done
