#!/bin/bash
# Round-4 GPU step for DIN kernel changes: DIN parity / plan / stream / fuzz tests, then the quick bench.
set -o pipefail
O=gpurun_out/r04; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_din_plan.py tests/test_gpu_mlp_stream.py tests/test_gpu_fuzz.py tests/test_gpu_golden.py tests/test_gpu_bst_small.py -x -q --timeout 150 --timeout-method thread -k "din or bst" > $O/test_din.log 2>&1 || { echo "din tests failed"; grep -E "Error|assert|FAILED" $O/test_din.log | head -30; tail -5 $O/test_din.log; exit 1; }
tail -1 $O/test_din.log
MODELS=${MODELS:-dcn,bst_ref,din_per_call} bash tools/sessions/r04_quick.sh
