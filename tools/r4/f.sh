# round 4: fence-free fused blend finalize (atomic partials), cross-product form A/B, launch floor
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/r4f"; mkdir -p "$OUT"; cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 100 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_fused_finalize.py tests/test_gpu_scalar_link.py > "$OUT/tests.log" 2>&1
rc=$?; tail -3 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -m pytest -q --timeout 100 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_shading.py tests/test_gpu_normals.py > "$OUT/x_fms.log" 2>&1
PR_NATIVE_LIB=$R/pertrenderer_amd/libpertrender_xplain.so timeout -k 10 200 python -u -m pytest -q --timeout 100 \
  --timeout-method thread -p no:cacheprovider tests/test_gpu_shading.py tests/test_gpu_normals.py > "$OUT/x_plain.log" 2>&1
tail -1 "$OUT/x_fms.log" "$OUT/x_plain.log"
timeout -k 10 120 python tools/launch_overhead.py > "$OUT/launch_overhead.json" 2>&1 || exit 1
bash tools/gpu.sh sweep r4f cfg2 "nosync|PR_BLEND_SYNC=0|" "sync|PR_BLEND_SYNC=1|" "nosync2|PR_BLEND_SYNC=0|" "sync2|PR_BLEND_SYNC=1|" || exit 1
