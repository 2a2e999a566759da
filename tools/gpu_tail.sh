# GPU check of the backward's masked-tail draw: blend/variant/full-size parity tests, then
# cfg2 + cfg4 bench lines and a cfg4 rocprofv3 kernel summary (run through gpurun).
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/tail"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_blend.py tests/test_gpu_variants.py tests/test_gpu_fullsize.py tests/test_public_api_parity.py \
  > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -3 "$OUT/tests.log"
timeout -k 10 200 python bench.py --no-cpu-baseline > "$OUT/cfg2.json" 2> "$OUT/cfg2.err" || { tail -20 "$OUT/cfg2.err"; exit 1; }
cat "$OUT/cfg2.json"
timeout -k 10 300 python bench.py --config cfg4 --steps 10 --warmup 3 --no-cpu-baseline --no-dense \
  > "$OUT/cfg4.json" 2> "$OUT/cfg4.err" || { tail -20 "$OUT/cfg4.err"; exit 1; }
cat "$OUT/cfg4.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_cfg4" -o p -- \
  python "$R/bench.py" --config cfg4 --steps 10 --warmup 3 --no-cpu-baseline --no-dense > /dev/null 2>&1 || exit 1
find "$OUT/prof_cfg4" -name "*kernel_stats.csv" -exec head -8 {} \;
