# rocprofv3 kernel trace + stats of the graph bench (no cpu baseline / dense microbench)
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG="${1:-kt}"; shift || true
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$TAG" -o prof -- \
  python "$R/bench.py" --no-cpu-baseline --no-dense --steps 30 --warmup 5 "$@" > "$OUT/bench_prof_$TAG.json" 2> "$OUT/prof_$TAG.err"
rc=$?; echo "rocprof rc=$rc"; tail -2 "$OUT/prof_$TAG.err"
exit $rc
