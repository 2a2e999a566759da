# round 4 (re-entry): backward-only interleaved blocks on batch grids: blend / batch tests, cfg3 / cfg4 A/B
# (default = consecutive forward + interleaved backward, vs both interleaved, vs both consecutive), then the
# cfg2 records for the new source_sha (rocprof stats, PMC passes) and the default bench line
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"
timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_interleave.py tests/test_gpu_blend.py tests/test_gpu_cfg4_blend.py tests/test_gpu_fullsize.py tests/test_gpu_empty_blocks.py \
  tests/test_gpu_headline_parity.py tests/test_gpu_fused_finalize.py > gpurun_out/tests_r4h.log 2>&1
rc=$?; tail -n 2 gpurun_out/tests_r4h.log; [ $rc -ne 0 ] && exit $rc
for c in cfg3 cfg4; do
  bash tools/gpu.sh sweep r4h_$c $c "def|PR_X=0|" "il|PR_BLEND_INTERLEAVE=1|" "cons|PR_BLEND_INTERLEAVE=0|" || exit 1
done
bash tools/gpu.sh prof r4h --steps 200 --warmup 20 --no-cpu-baseline --no-dense || exit 1
bash tools/gpu.sh pmc pmc_r4h || exit 1
bash tools/gpu.sh bench r4h || exit 1
