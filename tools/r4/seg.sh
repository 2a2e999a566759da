# round 4: segment-plan correctness + segment-size sweep at cfg2 (through gpurun)
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/r4c"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_segments.py tests/test_gpu_empty_blocks.py tests/test_gpu_counts.py > "$OUT/tests.log" 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" "$OUT/tests.log" | tail -8; [ $rc -ne 0 ] && exit $rc
bash tools/gpu.sh sweep r4c cfg2 "seg512|PR_X=0|" "static|PR_BLEND_SEG=0|" "seg768|PR_BLEND_SEG_FWD=768 PR_BLEND_SEG_BWD=768|" \
  "seg1024|PR_BLEND_SEG_FWD=1024 PR_BLEND_SEG_BWD=1024|" "seg384|PR_BLEND_SEG_FWD=384 PR_BLEND_SEG_BWD=384|" \
  "seglpp|PR_BLEND_SEG_LPP=32 PR_BLEND_SEG_LPP_BWD=16|" "static2|PR_BLEND_SEG=0|" "seg512b|PR_X=0|" || exit 1
bash tools/gpu.sh prof r4c_seg --steps 200 --warmup 20 --no-cpu-baseline --no-dense || exit 1
python tools/ab_table.py "$OUT" 2>/dev/null | head -3
