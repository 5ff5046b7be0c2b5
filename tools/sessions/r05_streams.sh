#!/bin/bash
# Round-5: the DIN headline with S batches in flight (bench.py --din-streams S), at the driver's
# --steps 20 --warmup 5 and at the default 50 / 10, alternating S, twice.
# Usage (on the box): bash tools/sessions/r05_streams.sh <tag>
set -o pipefail
T=${1:-st}; O=gpurun_out/r05/$T; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2; do
  for K in "20 5" "50 10"; do
    set -- $K
    for S in 1 2 3; do
      n=s${S}_k$1_$i
      timeout -k 10 200 python bench.py --no-cpu --no-loader --no-train --no-sharded --no-extras --steps $1 --warmup $2 --din-streams $S > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; tail -5 $O/$n.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', round(d['value']/1e6,2), 'M', d['ms_per_step'])"
    done
  done
done
echo streams done
