# round 4 (re-entry): interleave debug (where the layouts differ), then the A/B sweeps of b.sh
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"
timeout -k 10 200 python tools/interleave_debug.py > gpurun_out/il_debug.txt 2>&1; cat gpurun_out/il_debug.txt | tail -40
bash tools/gpu.sh sweep r4b cfg2 "il|PR_BLEND_INTERLEAVE=1|" "cons|PR_BLEND_INTERLEAVE=0|" "il2|PR_BLEND_INTERLEAVE=1|" "cons2|PR_BLEND_INTERLEAVE=0|" \
  "il_pb32|PR_BLEND_INTERLEAVE=1 PR_BLEND_PB_BWD=32|" "il_lds16|PR_BLEND_INTERLEAVE=1 PR_BLEND_LDS_KB_BWD=16|" || exit 1
for c in eval cfg3 cfg4; do
  bash tools/gpu.sh sweep r4b_$c $c "il|PR_BLEND_INTERLEAVE=1|" "cons|PR_BLEND_INTERLEAVE=0|" || exit 1
done
