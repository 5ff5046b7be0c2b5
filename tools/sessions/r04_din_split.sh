#!/bin/bash
# DIN kernel split by timing builds (RK_DIN_SKIP_A: phase B on zero rows; RK_DIN_SKIP_B: phase A
# only; RK_DIN_NO_GATHER: keys from 16 cache-resident rows) at the bench workload.
# Usage (on the box): bash tools/sessions/r04_din_split.sh <tag> [lib names...]
set -o pipefail
T=${1:-split}; shift; O=gpurun_out/r04; mkdir -p $O
P=implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd/rankops
for n in ${@:-librankops librankops_skipA librankops_skipB librankops_nogather}; do
  RANKOPS_LIB=$PWD/$P/$n.so timeout -k 10 120 python tools/din_phase_time.py >> $O/din_split_$T.log 2>&1 || { echo "$n failed"; tail -5 $O/din_split_$T.log; exit 1; }
done
grep -v amdgpu.ids $O/din_split_$T.log
