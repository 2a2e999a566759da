# round 4 (re-entry): interleaved blend pixel blocks (PR_BLEND_INTERLEAVE, default on): full GPU suite,
# then A/B sweeps against the consecutive blocks (same library, env switch) at cfg2 / eval / cfg3 / cfg4
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"
bash tools/gpu.sh tests r4b || exit 1
bash tools/gpu.sh sweep r4b cfg2 "il|PR_BLEND_INTERLEAVE=1|" "cons|PR_BLEND_INTERLEAVE=0|" "il2|PR_BLEND_INTERLEAVE=1|" "cons2|PR_BLEND_INTERLEAVE=0|" \
  "il_pb32|PR_BLEND_INTERLEAVE=1 PR_BLEND_PB_BWD=32|" "il_lpp16|PR_BLEND_INTERLEAVE=1 PR_BLEND_LPP=16|" || exit 1
for c in eval cfg3 cfg4; do
  bash tools/gpu.sh sweep r4b_$c $c "il|PR_BLEND_INTERLEAVE=1|" "cons|PR_BLEND_INTERLEAVE=0|" || exit 1
done
bash tools/gpu.sh prof r4b --steps 200 --warmup 20 --no-cpu-baseline --no-dense || exit 1
