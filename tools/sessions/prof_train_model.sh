#!/bin/bash
# Kernel trace of one model's training step: bash tools/prof_train_model.sh <model> <outdir>
M=${1:-din}; O=${2:-gpurun_out/tr_$1}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o prof --output-format csv -- python3 tools/kprof_train.py --model $M --steps 10 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
grep '^{' $O/prof.log
