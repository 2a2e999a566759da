# native vertex normals: full GPU suite, eval-renderer bench with and without them
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; cd "$R"
PR_NATIVE_NORMALS=1 timeout -k 10 600 python -u -m pytest tests -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests_nrm.log" 2>&1
rc=$?; grep -E "passed|failed|Error" "$OUT/tests_nrm.log" | tail -8; [ $rc -ne 0 ] && exit $rc
for flag in True False; do
  timeout -k 10 300 python -c "
import sys; sys.argv=['bench.py','--config','eval','--no-cpu-baseline','--no-dense']
import pertrenderer_amd.renderer.mesh as m; m.NATIVE_NORMALS=$flag
import runpy; runpy.run_path('bench.py', run_name='__main__')" > "$OUT/bench_eval_nrm_$flag.json" 2>> "$OUT/nrm.err" || exit 1
  python -c "import json;d=json.load(open('$OUT/bench_eval_nrm_$flag.json'));print('eval native normals=$flag',d['value'],d['ms_per_step'])"
done
