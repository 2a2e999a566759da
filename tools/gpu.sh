# One driver for the GPU-box runs (through gpurun):  bash tools/gpu.sh <command> [args]
#
#   tests [TAG]                     GPU test suite + smoke()
#   quick [TAG]                     smoke, GPU tests, one graph bench line
#   bench TAG [bench.py args]       one bench line -> gpurun_out/bench_TAG.json (+ kernel summary)
#   sweep TAG CONFIG SPEC...        bench kernel times per variant; SPEC = "name|ENV=V ...|libname"
#                                   (libname: a variant built with build_native --out, default the product)
#   rprof TAG [ENV=V ...]...        rast_fwd per-tile timeline (-DPR_RAST_PROFILE variant), one per env set
#   pmc TAG [kprof.py args]         PMC counter passes, each its own rocprofv3 run (kernel trace only)
#   pmcbench TAG [bench.py args]    PMC passes (as pmc) over one bench.py command
#   prof TAG [bench.py args]        rocprofv3 --kernel-trace --stats of one bench command
#   kvar TAG REGEX ENVS... -- ARGS  average times of the kernels matching REGEX, one rocprofv3 run of
#                                   bench.py ARGS per env set
#   final TAG                       round-end measurement: tests, smoke, bench lines (graph + CPU
#                                   baseline, eager, eager under HIP_LAUNCH_BLOCKING=1, eval, cfg3,
#                                   cfg4, eager eval), cfg5 (pose_opt 100 x 800), rocprof stats, PMC
#                                   passes and their summary
#   final2 TAG                      eager / HIP_LAUNCH_BLOCKING=1 rows of the eval renderer and cfg5
#                                   (20 problems), then the dense microbench records
#
# Every GPU step runs under its own timeout and the chain stops at the first failure.
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; cd "$R"
CMD="${1:-quick}"; shift || true

summ() {  # summary of a bench json
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'], d['ms_per_step'], d['config']['execution'], {k:(v['ms'],v.get('kernel_ms')) for k,v in d['kernels'].items()}, 'roofline', d['roofline']['kernel'], d['roofline']['frac'], 'dense', {k:v['frac'] for k,v in d.get('roofline_dense',{}).items()}, 'cpu', d.get('cpu_baseline',{}).get('value'))" "$1" "$2"
}

tests() {
  local tag="${1:-t}"
  timeout -k 10 1100 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/tests_$tag.log" 2>&1
  local rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" "$OUT/tests_$tag.log" | tail -15; [ $rc -ne 0 ] && return $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$tag.log" 2>&1 || { tail -5 "$OUT/smoke_$tag.log"; return 1; }
  tail -n 1 "$OUT/smoke_$tag.log"
}

bench() {
  local tag="$1"; shift
  timeout -k 10 600 python bench.py "$@" > "$OUT/bench_$tag.json" 2> "$OUT/bench_$tag.err" || { tail -5 "$OUT/bench_$tag.err"; return 1; }
  summ "$OUT/bench_$tag.json" "$tag"
}

sweep() {
  local tag="$1" cfg="$2"; shift 2
  for spec in "$@"; do
    IFS='|' read -r name envs lib <<< "$spec"
    local libpath=""; [ -n "$lib" ] && libpath="PR_NATIVE_LIB=$R/pertrenderer_amd/$lib.so"
    env $envs $libpath timeout -k 10 200 python bench.py --config "$cfg" --no-cpu-baseline --no-dense --steps 30 --warmup 5 \
      > "$OUT/sw_${tag}_$name.json" 2>> "$OUT/sw_$tag.err" || { echo "FAIL $name"; tail -3 "$OUT/sw_$tag.err"; return 1; }
    summ "$OUT/sw_${tag}_$name.json" "$name"
  done
}

rprof() {
  local tag="$1"; shift
  [ $# -eq 0 ] && set -- "PR_X=0"
  for envs in "$@"; do
    local f="$OUT/rprof_${tag}_${envs// /_}"
    env $envs PR_NATIVE_LIB=$R/pertrenderer_amd/libpertrender_prof.so timeout -k 10 120 python tools/rast_prof.py "$f.npy" > "$f.log" 2>&1 || { tail -5 "$f.log"; return 1; }
    python tools/rast_timeline.py "$f.npy"
  done
}

pmc() {
  local tag="$1"; shift
  (cd /tmp && export TMPDIR=/tmp
   local i=0
   for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" \
            "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
     i=$((i+1))
     timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/${tag}_p$i" -o p -- \
       python "$R/tools/kprof.py" "$@" > "$OUT/${tag}_p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -5 "$OUT/${tag}_p$i.log"; exit 1; }
   done) || return 1
  python tools/pmc_summary.py "$OUT"/${tag}_p* --traffic-out "$OUT/pmc_traffic_$tag.json" > "$OUT/pmc_summary_$tag.txt" 2>&1
  tail -20 "$OUT/pmc_summary_$tag.txt"
}

prof() {
  local tag="$1"; shift
  (cd /tmp && export TMPDIR=/tmp
   timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$tag" -o prof -- \
     python "$R/bench.py" "$@" > "$OUT/bench_prof_$tag.json" 2> "$OUT/prof_$tag.err") || { tail -5 "$OUT/prof_$tag.err"; return 1; }
  local f; f=$(find "$OUT/prof_$tag" -name "*kernel_stats.csv" | sort | sed -n 1p)
  python tools/rocprof_summary.py "$f" "$OUT/rocprof_kernels_$tag.json" "rocprofv3 --kernel-trace --stats -- python bench.py $*"
}

pmcbench() {  # PMC passes over a bench.py run: pmcbench TAG [bench.py args]
  local tag="$1"; shift
  (cd /tmp && export TMPDIR=/tmp
   local i=0
   for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" \
            "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
     i=$((i+1))
     timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/${tag}_p$i" -o p -- \
       python "$R/bench.py" "$@" > "$OUT/${tag}_p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -5 "$OUT/${tag}_p$i.log"; exit 1; }
     find "$OUT/${tag}_p$i" -name "*kernel_trace.csv" -delete
   done) || return 1
  python tools/pmc_summary.py "$OUT"/${tag}_p* > "$OUT/pmc_summary_$tag.txt" 2>&1
  tail -20 "$OUT/pmc_summary_$tag.txt"
}

dense() {  # SURVEY §8(d) dense-fragment blend microbench: rocprofv3 stats + PMC passes
  local tag="$1"
  (cd /tmp && export TMPDIR=/tmp
   timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/dense_$tag" -o prof -- \
     python "$R/tools/kprof.py" --dense --iters 40 > "$OUT/dense_$tag.log" 2>&1) || { tail -5 "$OUT/dense_$tag.log"; return 1; }
  local f; f=$(find "$OUT/dense_$tag" -name "*kernel_stats.csv" | sort | sed -n 1p)
  python tools/rocprof_summary.py "$f" "$OUT/rocprof_dense_$tag.json" \
    "rocprofv3 --kernel-trace --stats -- python tools/kprof.py --dense --iters 40" || return 1
  pmc "pmcdense_$tag" --dense
}

sel() {  # selected GPU test files: sel TAG FILE...
  local tag="$1"; shift
  timeout -k 10 900 python -u -m pytest "$@" -q -m gpu --timeout 240 --timeout-method thread -p no:cacheprovider \
    > "$OUT/tests_$tag.log" 2>&1
  local rc=$?; grep -E "^(FAILED|ERROR)|passed|failed" "$OUT/tests_$tag.log" | tail -15; return $rc
}

kvar() {  # kernel times per env variant: kvar TAG REGEX "ENV=V ..." ... -- bench.py args
  local tag="$1" pat="$2"; shift 2
  local vars=()
  while [ $# -gt 0 ] && [ "$1" != "--" ]; do vars+=("$1"); shift; done
  shift || true
  for envs in "${vars[@]}"; do
    local d="$OUT/kvar_${tag}_$(echo "$envs" | tr ' /' '__')"
    (cd /tmp && export TMPDIR=/tmp && export $envs
     timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o k -- \
       python "$R/bench.py" "$@" > "$d.json" 2> "$d.err") || { echo "FAIL $envs"; tail -5 "$d.err"; return 1; }
    local f; f=$(find "$d" -name "*kernel_stats.csv" | sort | sed -n 1p)
    find "$d" -name "*kernel_trace.csv" -delete
    python - "$f" "$pat" "$envs" "$d.json" <<'PY'
import csv, json, re, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if re.search(sys.argv[2], r["Name"])]
v = json.load(open(sys.argv[4]))["value"]
print(sys.argv[3], "value", v, {r["Name"].split("(")[0][-40:]: round(float(r["AverageNs"]) / 1e3, 2) for r in rows})
PY
  done
}

kernels() {  # per-step kernel list with the issuing call (tools/step_kernels.py)
  local tag="$1"; shift
  timeout -k 10 300 python tools/step_kernels.py --json "$OUT/step_kernels_$tag.json" "$@" > "$OUT/step_kernels_$tag.txt" 2>&1 \
    || { tail -5 "$OUT/step_kernels_$tag.txt"; return 1; }
  tail -1 "$OUT/step_kernels_$tag.txt"
}

case "$CMD" in
  dense) dense "${1:-d}" ;;
  sel) sel "$@" ;;
  kernels) kernels "$@" ;;
  kvar) kvar "$@" ;;
  pmcbench) pmcbench "$@" ;;
  tests) tests "${1:-t}" ;;
  quick) tests "${1:-q}" && bench "${1:-q}" --no-cpu-baseline ;;
  bench) bench "$@" ;;
  sweep) sweep "$@" ;;
  rprof) rprof "$@" ;;
  pmc) pmc "$@" ;;
  prof) prof "$@" ;;
  final)
    T="${1:-fin}"
    tests "$T" || exit 1
    bench "$T" || exit 1
    bench "eager_$T" --mode eager --no-cpu-baseline --no-dense || exit 1
    # eval.py's CUDA_LAUNCH_BLOCKING=1 (eval.py:4) is not honoured by the HIP runtime (the plain eager row
    # is what eval.py gets); HIP_LAUNCH_BLOCKING=1 is the host-synchronous launch mode it asks for
    HIP_LAUNCH_BLOCKING=1 bench "eager_blocking_$T" --mode eager --no-cpu-baseline --no-dense || exit 1
    timeout -k 10 60 python tools/launch_blocking_check.py > "$OUT/launch_blocking_$T.txt" 2>&1 &&
      CUDA_LAUNCH_BLOCKING=1 timeout -k 10 60 python tools/launch_blocking_check.py >> "$OUT/launch_blocking_$T.txt" 2>&1 &&
      HIP_LAUNCH_BLOCKING=1 timeout -k 10 60 python tools/launch_blocking_check.py >> "$OUT/launch_blocking_$T.txt" 2>&1 &&
      timeout -k 10 60 python tools/launch_blocking_check.py --eval-order >> "$OUT/launch_blocking_$T.txt" 2>&1 || exit 1
    for c in eval cfg3 cfg4; do bench "${c}_$T" --config $c --no-cpu-baseline || exit 1; done
    bench "eager_eval_$T" --config eval --mode eager --no-cpu-baseline --no-dense || exit 1
    # BASELINE cfg5: eval.py's pose benchmark, 100 problems x 800 iterations x {softras, gaussian}
    timeout -k 10 600 python -m pertrenderer_amd.pose_opt -np 100 -ni 800 --mode graph --out "$OUT/cfg5_$T" \
      > "$OUT/cfg5_$T.log" 2>&1 || { tail -5 "$OUT/cfg5_$T.log"; exit 1; }
    tail -3 "$OUT/cfg5_$T.log"
    prof "$T" --steps 200 --warmup 20 --no-cpu-baseline --no-dense || exit 1
    pmc "pmc_$T" || exit 1
    ;;
  final2)  # the eager / host-synchronous rows of eval.py's own mode + the dense records
    T="${1:-fin}"
    HIP_LAUNCH_BLOCKING=1 bench "eager_blocking_eval_$T" --config eval --mode eager --no-cpu-baseline --no-dense || exit 1
    # cfg5 at 20 of the 100 problems (the per-problem time is what compares): eager, then host-synchronous
    timeout -k 10 300 python -m pertrenderer_amd.pose_opt -np 20 -ni 800 --mode eager --out "$OUT/cfg5_eager_$T" \
      > "$OUT/cfg5_eager_$T.log" 2>&1 || { tail -5 "$OUT/cfg5_eager_$T.log"; exit 1; }
    tail -2 "$OUT/cfg5_eager_$T.log"
    HIP_LAUNCH_BLOCKING=1 timeout -k 10 400 python -m pertrenderer_amd.pose_opt -np 20 -ni 800 --mode eager \
      --out "$OUT/cfg5_eager_blocking_$T" > "$OUT/cfg5_eager_blocking_$T.log" 2>&1 || { tail -5 "$OUT/cfg5_eager_blocking_$T.log"; exit 1; }
    tail -2 "$OUT/cfg5_eager_blocking_$T.log"
    dense "$T" || exit 1
    ;;
  *) echo "unknown command $CMD"; exit 2 ;;
esac
