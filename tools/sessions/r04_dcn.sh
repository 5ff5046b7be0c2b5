#!/bin/bash
# Round-4 GPU step for MLP-tail / DCN / BST-16 changes: their tests, the quick bench, phase splits.
set -o pipefail
O=gpurun_out/r04; mkdir -p $O; export TMPDIR=/tmp
P=implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd/rankops
timeout -k 10 500 python -u -m pytest tests/test_gpu_mlp_stream.py tests/test_gpu_bst_small.py tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -k "dcn or bst or stream" > $O/test_dcn.log 2>&1 || { echo "tests failed"; grep -E "Error|assert|FAILED" $O/test_dcn.log | head -30; exit 1; }
tail -1 $O/test_dcn.log
MODELS=${MODELS:-dcn,deepfm,bst,bst_ref,din_per_call} bash tools/sessions/r04_quick.sh || exit 1
RANKOPS_LIB=$PWD/$P/librankops_phases.so timeout -k 10 120 python tools/dcn_phases.py > $O/dcn_phases_${1:-x}.log 2>&1 || exit 1
head -12 $O/dcn_phases_${1:-x}.log
