#!/bin/bash
# Tests on one library variant, then the bench legs over several builds twice interleaved.
# bash tools/sessions/r04_libs_ab.sh <tag> <test-lib-name> <lib-name>...   (names under rankops/, no .so)
set -o pipefail
T=$1; TL=$2; shift 2; export ABDIR=gpurun_out/r04; export TMPDIR=/tmp; mkdir -p $ABDIR
P=implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd/rankops
RANKOPS_LIB=$PWD/$P/$TL.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mlp_stream.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_din_plan.py -x -q --timeout 120 --timeout-method thread > $ABDIR/test_$T.log 2>&1 || { echo "tests failed"; tail -30 $ABDIR/test_$T.log; exit 1; }
tail -1 $ABDIR/test_$T.log
L=""; for n in "$@"; do L="$L $P/$n.so"; done
bash tools/sessions/ab_bench.sh $T $L && bash tools/sessions/ab_bench.sh ${T}_2 $L
