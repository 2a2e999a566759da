# VALU picture of the blend kernels at cfg4: Philox/Box-Muller throughput microbenchmark and
# one SQ counter pass over the cfg4 workload (run through gpurun).
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out/valu"; mkdir -p "$OUT"
cd "$R"
timeout -k 10 120 tools/philox_bench || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
  --kernel-trace --output-format csv -d "$OUT/p1" -o p -- python "$R/tools/kprof.py" --config cfg4 --iters 3 > "$OUT/p1.log" 2>&1 || { tail -5 "$OUT/p1.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM \
  --kernel-trace --output-format csv -d "$OUT/p2" -o p -- python "$R/tools/kprof.py" --config cfg4 --iters 3 > "$OUT/p2.log" 2>&1 || { tail -5 "$OUT/p2.log"; exit 0; }
cd "$R" && python tools/pmc_summary.py "$OUT/p1" "$OUT/p2" 2>&1 | head -40
