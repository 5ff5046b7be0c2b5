#!/bin/bash
# Round-4 A/B session: the streamed-MLP tests on the default library, then bench legs over the given
# library builds (twice, interleaved), then the DCN / DIN phase splits from the timing build.
# Usage (on the box): bash tools/sessions/r04_ab.sh <tag> <lib.so>...
set -o pipefail
T=$1; shift; export ABDIR=gpurun_out/r04; export TMPDIR=/tmp; mkdir -p $ABDIR
P=implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd/rankops
timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp_stream.py -x -q --timeout 120 --timeout-method thread > $ABDIR/test_stream_$T.log 2>&1 || { echo "stream tests failed"; tail -40 $ABDIR/test_stream_$T.log; exit 1; }
tail -1 $ABDIR/test_stream_$T.log
bash tools/sessions/ab_bench.sh ${T} "$@" && bash tools/sessions/ab_bench.sh ${T}_2 "$@" || exit 1
if [ -f $P/librankops_phases.so ]; then
  RANKOPS_LIB=$PWD/$P/librankops_phases.so timeout -k 10 120 python tools/dcn_phases.py > $ABDIR/dcn_phases_$T.log 2>&1 || exit 1
  RANKOPS_LIB=$PWD/$P/librankops_phases.so timeout -k 10 120 python tools/din_phases.py > $ABDIR/din_phases_$T.log 2>&1 || exit 1
  head -12 $ABDIR/dcn_phases_$T.log; tail -5 $ABDIR/din_phases_$T.log
fi
