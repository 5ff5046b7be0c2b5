#!/bin/bash
# Round-5: DIN headline and DCN / DeepFM legs for the current library and variant libraries, alternating.
# Usage (on the box): bash tools/sessions/r05_ab_multi.sh <tag> <variant.so>...
set -o pipefail
T=$1; shift; O=gpurun_out/r05/$T; mkdir -p $O; export TMPDIR=/tmp
CUR=$PWD/implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd/rankops/librankops.so
for i in 1 2; do
  for L in cur "$@"; do
    if [ $L = cur ]; then lib=$CUR; n=cur; else lib=$PWD/$L; n=$(basename $L .so); fi
    RANKOPS_LIB=$lib timeout -k 10 200 python bench.py --no-cpu --no-loader --no-train --no-sharded --models dcn,deepfm > $O/${n}_$i.json 2> $O/${n}_$i.err || { echo "bench $n failed"; tail -5 $O/${n}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/${n}_$i.json').read().strip().splitlines()[-1]); m=d['models']; print('$n', '$i', 'din', round(d['value']/1e6,2), d['roofline']['avg_launch_ms'], 'dcn', m['dcn']['roofline']['avg_launch_ms'], 'deepfm', m['deepfm']['roofline']['avg_launch_ms'])"
  done
done
echo ab done
