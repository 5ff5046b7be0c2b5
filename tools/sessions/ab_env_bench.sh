#!/bin/bash
# A/B of an environment switch on the bench's forward legs, twice interleaved:
# bash tools/sessions/ab_env_bench.sh <tag> <VAR> <value>...   (run on the box)
set -o pipefail
T=$1; V=$2; shift 2; O=gpurun_out/r04; export TMPDIR=/tmp; mkdir -p $O
for r in 1 2; do for v in "$@"; do
  env $V=$v timeout -k 10 300 python bench.py --no-cpu --no-loader --no-train --no-sharded --models dcn > $O/ab_${T}${r}_$v.json 2> $O/ab_${T}${r}_$v.err || { echo "bench failed"; tail -5 $O/ab_${T}${r}_$v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']/1e6,2), 'M kernel', d['roofline']['avg_launch_ms'])" $O/ab_${T}${r}_$v.json
done; done
