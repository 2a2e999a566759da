set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"
cd "$R"
for s in "16 8" "128 128"; do
  timeout -k 10 120 python tools/cfg5_step_prof.py --samples $s --iters 40 >> "$OUT/c5.log" 2>&1 || exit 1
done
timeout -k 10 120 python tools/cfg5_step_prof.py --noise softras --iters 40 >> "$OUT/c5.log" 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5prof_s16" -o p -- python "$R/tools/cfg5_step_prof.py" --samples 16 8 --iters 40 > /dev/null 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5prof_s128" -o p -- python "$R/tools/cfg5_step_prof.py" --samples 128 128 --iters 40 > /dev/null 2>&1 || exit 1
cat "$OUT/c5.log"
