# rocprofv3 kernel-trace + stats over tools/kprof.py (per-kernel durations, no counters)
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG="${1:-kt}"; shift || true
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$TAG" -o k -- \
   python "$R/tools/kprof.py" "$@" > "$OUT/$TAG.log" 2>&1
rc=$?; echo "ktrace rc=$rc"
python "$R/tools/kstats.py" "$OUT/$TAG" || true
exit $rc
