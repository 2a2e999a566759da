# round 4: batched loads in project_bwd_gather: tests, rocprof averages and bench lines vs the HEAD build
set -u
R="$GRAFT_REPO_ROOT"; cd "$R"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 250 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_rast.py tests/test_gpu_deterministic.py tests/test_gpu_headline_parity.py tests/test_gpu_pipeline_ref.py \
  tests/test_gpu_host_layer.py > gpurun_out/tests_r4x.log 2>&1
rc=$?; tail -n 2 gpurun_out/tests_r4x.log; [ $rc -ne 0 ] && exit $rc
for v in new base new2 base2; do
  lib=""; case $v in base*) lib="PR_NATIVE_LIB=$R/pertrenderer_amd/libpertrender_base.so";; esac
  (cd /tmp && export TMPDIR=/tmp && env $lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$R/gpurun_out/prof_r4x_$v" -o p -- python "$R/bench.py" --steps 100 --warmup 10 --no-cpu-baseline --no-dense \
     > "$R/gpurun_out/bench_r4x_$v.json" 2> "$R/gpurun_out/prof_r4x_$v.err") || { echo "fail $v"; tail -3 "$R/gpurun_out/prof_r4x_$v.err"; exit 1; }
  f=$(find "gpurun_out/prof_r4x_$v" -name "*kernel_stats.csv" | head -n 1)
  python - "$f" "$v" <<'PY'
import csv, sys
rows = {r["Name"]: r for r in csv.DictReader(open(sys.argv[1]))}
sel = {k.split("(")[0].split("::")[-1]: round(float(r["AverageNs"]) / 1000, 3) for k, r in rows.items()
       if any(n in k for n in ("project_bwd_gather", "rast_bwd_kernel", "rotate_bwd", "so3_exp_bwd"))}
print(sys.argv[2], sel)
PY
done
for v in new base new2 base2; do
  lib=""; case $v in base*) lib="PR_NATIVE_LIB=$R/pertrenderer_amd/libpertrender_base.so";; esac
  env $lib timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-dense > gpurun_out/bench_r4x_plain_$v.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/bench_r4x_plain_$v.json $v
done
