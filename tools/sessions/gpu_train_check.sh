#!/bin/bash
# GPU-box check for a training change: the train parity tests selected by $2 (pytest -k), then a
# kernel trace of the model's training step.  Usage: bash tools/gpu_train_check.sh <tag> <k-expr> <model>
set -o pipefail
T=${1:-chk}; K=${2:-bst}; MODEL=${3:-bst}; O=gpurun_out/tr_$T; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q -k "$K" --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { echo "train tests failed"; tail -30 $O/test.log; exit 1; }
tail -1 $O/test.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o prof --output-format csv -- python3 tools/kprof_train.py --model $MODEL --steps 10 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
grep '^{' $O/prof.log
