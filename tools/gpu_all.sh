# Full GPU test suite + smoke (run through gpurun); logs under gpurun_out/all/.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/all"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -15 "$OUT/tests.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
