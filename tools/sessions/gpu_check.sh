#!/bin/bash
# GPU-box check used between kernel changes: gpu tests, DIN phase split (timing build), headline bench.
# Usage (on the box): bash tools/gpu_check.sh <tag>
set -o pipefail
T=${1:-chk}; O=gpurun_out/r02; mkdir -p $O
PKG=$PWD/implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest_$T.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gputest_$T.log; exit 1; }
tail -1 $O/gputest_$T.log
if [ -f $PKG/rankops/librankops_phases.so ]; then
  RANKOPS_LIB=$PKG/rankops/librankops_phases.so timeout -k 10 200 python tools/din_phases.py > $O/din_phases_$T.log 2>&1 || { echo "phases failed"; exit 1; }
fi
timeout -k 10 200 python bench.py --no-extras --no-cpu --no-loader --no-sharded > $O/bench_head_$T.json 2>/dev/null || { echo "bench failed"; exit 1; }
echo done
