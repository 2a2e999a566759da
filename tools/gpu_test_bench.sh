# GPU tests, then bench (graph + eager) and a rocprofv3 kernel-trace summary
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
TAG="${1:-run}"
cd "$R"
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 180 -p no:cacheprovider > "$OUT/tests_$TAG.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 "$OUT/tests_$TAG.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python "$R/bench.py" > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench_$TAG.json"; tail -5 "$OUT/bench_$TAG.err"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python "$R/bench.py" --mode eager --no-cpu-baseline --no-dense > "$OUT/bench_eager_$TAG.json" 2>> "$OUT/bench_$TAG.err"
rc=$?; echo "bench eager rc=$rc"; cut -c1-400 "$OUT/bench_eager_$TAG.json"
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o prof -- \
  python "$R/bench.py" --no-cpu-baseline > "$OUT/bench_prof_$TAG.json" 2> "$OUT/prof_$TAG.err"
rc=$?; echo "rocprof rc=$rc"
exit $rc
