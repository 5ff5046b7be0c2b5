#!/bin/bash
# Round-5 A/B: the DIN headline with the current library and with $ABLIB (default
# tools/bin/librankops_r4din.so: round 4's din_fused.hip)
# (round 4's din_fused.hip, everything else current), alternating; then SQ passes of the DIN and
# BST d16 kernels.  Usage (on the box): bash tools/sessions/r05_ab.sh <tag>
set -o pipefail
T=${1:-ab1}; O=gpurun_out/r05/$T; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2; do
  for L in cur var; do
    if [ $L = cur ]; then export RANKOPS_LIB=$PWD/implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd/rankops/librankops.so; else export RANKOPS_LIB=$PWD/${ABLIB:-tools/bin/librankops_r4din.so}; fi
    timeout -k 10 200 python bench.py --no-cpu --no-loader --no-train --no-sharded --no-extras > $O/din_${L}_$i.json 2> $O/din_${L}_$i.err || { echo "bench $L failed"; tail -5 $O/din_${L}_$i.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/din_${L}_$i.json').read().strip().splitlines()[-1]); print('$L', '$i', round(d['value']/1e6,2), 'M', d['roofline']['avg_launch_ms'])"
  done
done
unset RANKOPS_LIB
[ -n "$SQ" ] && { bash tools/sq_pass.sh $O/sq_bst_ref_blocks tools/kprof.py --workload bst_ref_blocks --iters 10 || exit 1; }
[ -n "$SQ" ] && { bash tools/sq_pass.sh $O/sq_din tools/kprof.py --workload din --iters 20 || exit 1; }
echo ab done
