# round 4: rasterizer occupancy variants + one step's kernel timeline (through gpurun)
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/r4d"; mkdir -p "$OUT"; cd "$R"
bash tools/gpu.sh sweep r4d cfg2 "base|PR_X=0|" "wpe4|PR_X=0|libpertrender_wpe4" "wpe4q0|PR_X=0|libpertrender_wpe4q0" \
  "base2|PR_X=0|" "wpe4q0b|PR_X=0|libpertrender_wpe4q0" || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o tr -- \
   python "$R/bench.py" --steps 30 --warmup 5 --no-cpu-baseline --no-dense > "$OUT/trace_bench.json" 2> "$OUT/trace.err") || { tail -3 "$OUT/trace.err"; exit 1; }
f=$(find "$OUT/trace" -name "*kernel_trace.csv" | sed -n 1p)
python tools/step_timeline.py "$f" 10 > "$OUT/step_timeline.txt"; tail -30 "$OUT/step_timeline.txt"
