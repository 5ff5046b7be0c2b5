#!/bin/bash
# Full GPU test suite, then a training-step kernel trace of $2 (default bst): bash tools/gpu_full.sh <tag> [model]
set -o pipefail
T=${1:-full}; MODEL=${2:-bst}; O=gpurun_out/full_$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o prof --output-format csv -- python3 tools/kprof_train.py --model $MODEL --steps 10 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
grep '^{' $O/prof.log
