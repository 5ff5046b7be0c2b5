#!/bin/bash
# Round-4 A/B: layer hand-off by ready flags (default build) against the barrier hand-off
# (librankops_noflags.so, RK_STREAM_FLAGS=0): the streamed-tail / DIN / DCN / DeepFM tests, the
# bench legs twice interleaved, then the DIN phase split (timing builds, graph replays).
set -o pipefail
T=${1:-flags}; export ABDIR=gpurun_out/r04; export TMPDIR=/tmp; mkdir -p $ABDIR
P=implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd/rankops
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp_stream.py tests/test_gpu_din_plan.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > $ABDIR/test_$T.log 2>&1 || { echo "tests failed"; tail -30 $ABDIR/test_$T.log; exit 1; }
tail -1 $ABDIR/test_$T.log
bash tools/sessions/ab_bench.sh ${T} $P/librankops.so $P/librankops_noflags.so && bash tools/sessions/ab_bench.sh ${T}_2 $P/librankops.so $P/librankops_noflags.so || exit 1
bash tools/sessions/r04_din_split.sh $T || exit 1
