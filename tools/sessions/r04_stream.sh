#!/bin/bash
# Round-4 GPU step: streamed-MLP parity tests, A/B of RANKOPS_MLP_STREAM on the bench legs, SQ
# counters of the timed kernels with the stream on and off.  Usage (on the box): bash tools/sessions/r04_stream.sh <tag>
set -o pipefail
T=${1:-s1}; O=gpurun_out/r04; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp_stream.py -x -q --timeout 120 --timeout-method thread > $O/test_stream_$T.log 2>&1 || { echo "stream tests failed"; tail -40 $O/test_stream_$T.log; exit 1; }
tail -1 $O/test_stream_$T.log
bash tools/sessions/ab_env.sh ${T}a RANKOPS_MLP_STREAM 1 0 && bash tools/sessions/ab_env.sh ${T}b RANKOPS_MLP_STREAM 1 0 || exit 1
for s in 1 0; do
  RANKOPS_MLP_STREAM=$s bash tools/sessions/r04_counters.sh ${T}_stream$s din dcn || exit 1
done
