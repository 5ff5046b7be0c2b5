#!/bin/bash
# Round-5 A/B of the BST d16 kernels: the bst_ref leg (whole one-launch forward and the blocks-only
# roofline launch) with the current library, a variant library, and the VALU kernels
# (RANKOPS_BST_MFMA=0).  Usage (on the box): bash tools/sessions/r05_ab_bst.sh <tag> <variant.so>
set -o pipefail
T=${1:-abb}; V=$2; O=gpurun_out/r05/$T; mkdir -p $O; export TMPDIR=/tmp
CUR=$PWD/implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd/rankops/librankops.so
run() {  # <name> <lib> [env]
  local n=$1 lib=$2; shift 2
  env RANKOPS_LIB=$lib "$@" timeout -k 10 200 python bench.py --no-cpu --no-loader --no-train --no-sharded --models bst_ref > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -5 $O/$n.err; return 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); m=d['models']['bst_ref']; print('$n', round(m['samples_per_s']/1e6,2), 'M step', m['ms_per_step'], 'blocks', m['roofline']['avg_launch_ms'], m['roofline']['kernel'])"
}
for i in 1 2; do
  run cur_$i $CUR || exit 1
  [ -n "$V" ] && { run var_$i $PWD/$V || exit 1; }
done
run valu $CUR RANKOPS_BST_MFMA=0 || exit 1
echo ab done
