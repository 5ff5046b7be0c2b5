#!/bin/bash
# Round-4 A/B: phase B's layer-0 chunks before the phase-A barrier (RANKOPS_DIN_PRE=1, default)
# against without (=0): DIN / streamed-tail tests, then the bench legs twice interleaved.
set -o pipefail
T=${1:-pre}; O=gpurun_out/r04; export TMPDIR=/tmp; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_din_plan.py tests/test_gpu_mlp_stream.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/test_$T.log 2>&1 || { echo "tests failed"; tail -30 $O/test_$T.log; exit 1; }
tail -1 $O/test_$T.log
for r in 1 2; do for v in 1 0; do
  RANKOPS_DIN_PRE=$v timeout -k 10 300 python bench.py --no-cpu --no-loader --no-train --no-sharded --models dcn > $O/ab_${T}${r}_pre$v.json 2> $O/ab_${T}${r}_pre$v.err || { echo "bench failed"; tail -5 $O/ab_${T}${r}_pre$v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']/1e6,2), 'M kernel', d['roofline']['avg_launch_ms'])" $O/ab_${T}${r}_pre$v.json
done; done
