# round 4: znear / zfar once per pass in the blend kernels: tests, rocprof averages and bench lines vs the HEAD build
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_blend.py tests/test_gpu_empty_blocks.py tests/test_gpu_fused_finalize.py tests/test_gpu_headline_parity.py tests/test_gpu_variants.py tests/test_gpu_cfg4_blend.py tests/test_gpu_segments.py tests/test_gpu_pipeline_ref.py \
  tests/test_gpu_host_layer.py > gpurun_out/tests_r4z2.log 2>&1
rc=$?; tail -n 2 gpurun_out/tests_r4z2.log; [ $rc -ne 0 ] && exit $rc
for v in new base new2 base2; do
  lib=""; case $v in base*) lib="PR_NATIVE_LIB=$R/pertrenderer_amd/libpertrender_base.so";; esac
  (cd /tmp && export TMPDIR=/tmp && env $lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$R/gpurun_out/prof_r4z2_$v" -o p -- python "$R/bench.py" --steps 100 --warmup 10 --no-cpu-baseline --no-dense \
     > "$R/gpurun_out/bench_r4z2_$v.json" 2> "$R/gpurun_out/prof_r4z2_$v.err") || { echo "fail $v"; tail -3 "$R/gpurun_out/prof_r4z2_$v.err"; exit 1; }
  f=$(find "gpurun_out/prof_r4z2_$v" -name "*kernel_stats.csv" | head -n 1)
  echo "$v $f"
done
for v in new base new2 base2; do
  lib=""; case $v in base*) lib="PR_NATIVE_LIB=$R/pertrenderer_amd/libpertrender_base.so";; esac
  env $lib timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-dense > gpurun_out/bench_r4z2_plain_$v.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/bench_r4z2_plain_$v.json $v
done
