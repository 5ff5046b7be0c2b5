#!/bin/bash
# A/B of library builds on the training steps: bash tools/train_ab.sh <tag> <models> <lib>...
set -o pipefail
T=$1; M=$2; shift 2; O=gpurun_out/r03; mkdir -p $O
for L in "$@"; do
  N=$(basename $L .so)
  RANKOPS_LIB=$PWD/$L timeout -k 10 300 python tools/train_ratio.py $M 60 2 > $O/trab_${T}_$N.log 2>&1 || { echo "train $N failed"; tail -5 $O/trab_${T}_$N.log; exit 1; }
  echo "$N: $(grep ratio $O/trab_${T}_$N.log | tr '\n' '|')"
done
