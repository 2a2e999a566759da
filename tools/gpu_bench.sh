# bench + rocprofv3 kernel-trace summary on one MI355X (run via gpurun)
set -u
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out"
mkdir -p "$OUT"
TAG="${1:-r1}"
timeout -k 10 600 python "$R/bench.py" > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench_$TAG.json"
if [ $rc -ne 0 ]; then tail -20 "$OUT/bench_$TAG.err"; exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o prof -- \
  python "$R/bench.py" --no-cpu-baseline > "$OUT/bench_prof_$TAG.json" 2> "$OUT/prof_$TAG.err"
rc=$?; echo "rocprof rc=$rc"
find "$OUT/prof_$TAG" -name "*stats*" | head
exit $rc
