# round 4 (re-entry): banded blend blocks (PR_BLEND_INTERLEAVE=2|4): parity vs consecutive, then cfg2 / eval A/B
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_interleave.py tests/test_gpu_blend.py tests/test_gpu_empty_blocks.py tests/test_gpu_headline_parity.py > gpurun_out/tests_r4d.log 2>&1
rc=$?; tail -n 3 gpurun_out/tests_r4d.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu.sh sweep r4d cfg2 "cons|PR_BLEND_INTERLEAVE=0|" "b2|PR_BLEND_INTERLEAVE=2|" "b4|PR_BLEND_INTERLEAVE=4|" \
  "cons2|PR_BLEND_INTERLEAVE=0|" "b2_2|PR_BLEND_INTERLEAVE=2|" "b4_2|PR_BLEND_INTERLEAVE=4|" "b8|PR_BLEND_INTERLEAVE=8|" || exit 1
bash tools/gpu.sh sweep r4d_eval eval "cons|PR_BLEND_INTERLEAVE=0|" "b2|PR_BLEND_INTERLEAVE=2|" "b4|PR_BLEND_INTERLEAVE=4|" || exit 1
bash tools/gpu.sh sweep r4d_cfg3 cfg3 "il|PR_BLEND_INTERLEAVE=1|" "b4|PR_BLEND_INTERLEAVE=4|" || exit 1
