#!/bin/bash
# Round-4 A/B: the DIN plan's epilogue image by LDS-DMA (RANKOPS_DIN_EPI_DMA=1, default) against
# resolving it per column at launch (=0): DIN tests, then the bench legs twice interleaved.
set -o pipefail
T=${1:-dma}; O=gpurun_out/r04; export TMPDIR=/tmp; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_din_plan.py tests/test_capi.py -x -q --timeout 120 --timeout-method thread > $O/test_$T.log 2>&1 || { echo "tests failed"; tail -30 $O/test_$T.log; exit 1; }
tail -1 $O/test_$T.log
for r in 1 2; do for v in 1 0; do
  RANKOPS_DIN_EPI_DMA=$v timeout -k 10 300 python bench.py --no-cpu --no-loader --no-train --no-sharded --models dcn > $O/ab_${T}${r}_dma$v.json 2> $O/ab_${T}${r}_dma$v.err || { echo "bench failed"; tail -5 $O/ab_${T}${r}_dma$v.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], round(d['value']/1e6,2), 'M kernel', d['roofline']['avg_launch_ms'])" $O/ab_${T}${r}_dma$v.json
done; done
