#!/bin/bash
# Round-6 GPU session: the GPU suite, smoke, the bench under rocprofv3 (tools/bench_final.sh), then
# optional extra steps.  A test failure (pytest exit 1) does not stop the measurement; a timeout,
# crash or abort does.  Usage (on the box): bash tools/sessions/r06_session.sh <tag> [extra command]
set -o pipefail
T=${1:-s1}; shift; O=gpurun_out/r06/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/test.log 2>&1
rc=$?
tail -3 $O/test.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)" $O/test.log | head; [ $rc -eq 1 ] || exit $rc; fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
bash tools/bench_final.sh r06_$T || exit 1
if [ -n "$1" ]; then bash -c "$1" || exit 1; fi
echo session done
