#!/bin/bash
# Memory-pipe counters of the DIN / DCN / DeepFM forward kernels (one --pmc pass per block group):
# TA busy / stalls, TCP stalls and L2 requests, L2 hit/miss.  bash tools/sessions/r04_ta.sh <tag>  (on the box)
set -o pipefail
T=${1:-ta}; O=gpurun_out/r04/$T; mkdir -p $O; export TMPDIR=/tmp
pass() {  # <name> <workload> <counters...>
  local n=$1 w=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d $O/$w/$n -o run --output-format csv -- python3 tools/kprof.py --workload $w --iters 20 > $O/${w}_$n.log 2>&1 || { echo "pass $n $w failed"; tail -3 $O/${w}_$n.log; return 1; }
}
for w in din dcn deepfm; do
  pass ta $w TA_TA_BUSY TA_DATA_STALLED_BY_TC_CYCLES || exit 1
  pass ta2 $w TA_ADDR_STALLED_BY_TC_CYCLES TA_TOTAL_WAVEFRONTS || exit 1
  pass tcp $w TCP_PENDING_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES TCP_TCC_READ_REQ || exit 1
  pass tcc $w TCC_HIT TCC_MISS || exit 1
  pass sq $w SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE || exit 1
  echo "$w done"
done
