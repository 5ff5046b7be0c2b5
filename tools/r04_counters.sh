#!/bin/bash
# Round-4 counter collection on the GPU box: SQ passes (MFMA busy, waits) for the four timed
# forward kernels, PMC traffic for the headline kernel, and a per-kernel trace of each forward.
# Usage (on the box): bash tools/r04_counters.sh <tag> [workloads...]
set -o pipefail
T=${1:-base}; shift
WL=${@:-din dcn deepfm bst}
O=gpurun_out/r04/$T; mkdir -p $O
export TMPDIR=/tmp
for w in $WL; do
  bash tools/sq_pass.sh $O/sq_$w tools/kprof.py --workload $w --iters 20 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace_$w -o run --output-format csv -- \
    python3 tools/kprof.py --workload $w --iters 50 > $O/trace_$w.log 2>&1 || { echo "trace $w failed"; exit 1; }
  echo "$w done"
done
