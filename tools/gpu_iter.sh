# One build -> measure iteration on the blend kernels (run through gpurun):
#   blend tests, fragment statistics, blend phase profiles (cfg2, cfg4), cfg2 + cfg4 bench lines.
# Extra env for the profiled/benched runs: $AB (e.g. "PR_BLEND_LPP=8") is run as a B variant.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/iter"; mkdir -p "$OUT"
cd "$R"
AB="${AB:-}"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_blend.py tests/test_gpu_variants.py > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
if [ -n "${STATS:-}" ]; then
  for c in cfg2 cfg4; do timeout -k 10 120 python tools/frag_stats.py --config $c 2>&1 | grep -v amdgpu.ids || exit 1; done
fi
for c in cfg2 cfg4; do
  for v in A B; do
    [ "$v" = B ] && [ -z "$AB" ] && continue
    E=""; [ "$v" = B ] && E="$AB"
    env $E PR_NATIVE_LIB=$R/pertrenderer_amd/libpertrender_prof.so timeout -k 10 200 \
      python tools/blend_prof.py --config $c > "$OUT/bprof_${c}_$v.log" 2>&1 || { tail -20 "$OUT/bprof_${c}_$v.log"; exit 1; }
    echo "== $c $v $E"; grep -A 2 "^blend_" "$OUT/bprof_${c}_$v.log" | grep -v histogram
  done
done
for c in cfg2 cfg4; do
  for v in A B; do
    [ "$v" = B ] && [ -z "$AB" ] && continue
    E=""; [ "$v" = B ] && E="$AB"
    env $E timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-dense \
      > "$OUT/b_${c}_$v.json" 2> "$OUT/b_${c}_$v.err" || { tail -20 "$OUT/b_${c}_$v.err"; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_forward'], d['ms_backward'], {k: v['ms'] for k, v in d['kernels'].items()})" "$OUT/b_${c}_$v.json" "$c $v"
  done
done
