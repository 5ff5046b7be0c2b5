#!/bin/bash
# Round-4 GPU step: stream/DCN tests, the quick bench of the given models, DCN and DIN phase splits.
set -o pipefail
O=gpurun_out/r04; mkdir -p $O; export TMPDIR=/tmp
P=implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd/rankops
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp_stream.py -x -q --timeout 150 --timeout-method thread > $O/test_stream_$1.log 2>&1 || { echo "tests failed"; grep -E "Error|assert|FAILED" $O/test_stream_$1.log | head -30; exit 1; }
tail -1 $O/test_stream_$1.log
MODELS=${MODELS:-dcn} bash tools/sessions/r04_quick.sh || exit 1
RANKOPS_LIB=$PWD/$P/librankops_phases.so timeout -k 10 120 python tools/dcn_phases.py > $O/dcn_phases_$1.log 2>&1 || exit 1
RANKOPS_LIB=$PWD/$P/librankops_phases.so timeout -k 10 120 python tools/din_phases.py > $O/din_phases_$1.log 2>&1 || exit 1
head -14 $O/dcn_phases_$1.log; tail -12 $O/din_phases_$1.log
