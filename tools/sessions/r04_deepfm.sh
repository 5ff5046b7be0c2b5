#!/bin/bash
# Round-4 GPU step for the one-launch DeepFM forward (and the staggered DCN side work): their tests,
# the quick bench, the DCN / DIN phase splits, rocprof of the DeepFM workload.
set -o pipefail
O=gpurun_out/r04; mkdir -p $O; export TMPDIR=/tmp
P=implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd/rankops
timeout -k 10 500 python -u -m pytest tests/test_gpu_deepfm_fused.py tests/test_gpu_fm_linear.py tests/test_gpu_mlp_stream.py tests/test_sharded_emulated.py -x -q --timeout 150 --timeout-method thread > $O/test_df_$1.log 2>&1 || { echo "tests failed"; grep -E "Error|assert|FAILED" $O/test_df_$1.log | head -30; tail -5 $O/test_df_$1.log; exit 1; }
tail -1 $O/test_df_$1.log
MODELS=${MODELS:-dcn,deepfm} bash tools/sessions/r04_quick.sh || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace_deepfm_$1 -o run --output-format csv -- python3 tools/kprof.py --workload deepfm --iters 30 > $O/trace_deepfm_$1.log 2>&1 || exit 1
find $O/trace_deepfm_$1 -name "*kernel_trace.csv" -delete
RANKOPS_LIB=$PWD/$P/librankops_phases.so timeout -k 10 120 python tools/dcn_phases.py > $O/dcn_phases_$1.log 2>&1 || exit 1
RANKOPS_LIB=$PWD/$P/librankops_phases.so timeout -k 10 120 python tools/din_phases.py > $O/din_phases_$1.log 2>&1 || exit 1
head -14 $O/dcn_phases_$1.log; tail -12 $O/din_phases_$1.log
RANKOPS_LIB=$PWD/$P/librankops_phases.so MODEL=deepfm timeout -k 10 120 python tools/dcn_phases.py > $O/deepfm_phases_$1.log 2>&1 || exit 1
head -14 $O/deepfm_phases_$1.log
if [ -n "$AB_BAL" ]; then bash tools/sessions/ab_env.sh bal RANKOPS_DIN_BALANCE 0 1 0 1 || exit 1; fi
