#!/bin/bash
# GPU tests on the default library, then tools/sessions/ab_bench.sh over the given A/B libraries.
# Usage (on the box): bash tools/check_ab.sh <tag> <lib.so>...
set -o pipefail
T=$1; shift; O=gpurun_out/r03; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/test_$T.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/test_$T.log; exit 1; }
tail -1 $O/test_$T.log
bash tools/sessions/ab_bench.sh $T "$@" && bash tools/sessions/ab_bench.sh ${T}_2 "$@"
