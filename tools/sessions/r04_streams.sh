#!/bin/bash
# DIN headline with 1 / 2 batches in flight, short (driver-like) and long windows.
set -o pipefail
O=gpurun_out/r04; mkdir -p $O
for S in 1 2 1 2; do
  timeout -k 10 200 python bench.py --no-cpu --no-loader --no-train --no-sharded --no-extras --din-streams $S --steps 20 --warmup 5 > $O/streams_$S.json 2> $O/streams_$S.err || { tail -5 $O/streams_$S.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/streams_$S.json').read().strip().splitlines()[-1]); print('S=$S steps 20', round(d['value']/1e6,2), d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
for S in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu --no-loader --no-train --no-sharded --no-extras --din-streams $S --steps 200 --warmup 20 > $O/streams_long_$S.json 2> $O/streams_long_$S.err || { tail -5 $O/streams_long_$S.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/streams_long_$S.json').read().strip().splitlines()[-1]); print('S=$S steps 200', round(d['value']/1e6,2), d['ms_per_step'])"
done
