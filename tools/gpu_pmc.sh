# PMC counter passes (each its own rocprofv3 run, kernel-trace only) over tools/kprof.py
set -u
R="$GRAFT_REPO_ROOT"; OUT="$R/gpurun_out"; mkdir -p "$OUT"; TAG="${1:-pmc}"; shift || true
EXTRA="$*"
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" \
         "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace --output-format csv -d "$OUT/${TAG}_p$i" -o p -- \
     python "$R/tools/kprof.py" $EXTRA > "$OUT/${TAG}_p$i.log" 2>&1
  rc=$?; echo "pass $i ($C) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/${TAG}_p$i.log"; exit $rc; fi
done
exit 0
