#!/bin/bash
# Round-5 verification step: layout probe, the GPU tests touched this round, DCN row-tile timing and
# the gather probe.  Usage (on the box): bash tools/sessions/r05_check.sh <tag>
set -o pipefail
T=${1:-c1}; O=gpurun_out/r05/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 5 30 ./tools/bin/mfma4_probe > $O/mfma4_probe.log 2>&1 || { echo "probe failed"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_bst_small.py tests/test_gpu_din_plan.py tests/test_gpu_parity.py \
  tests/test_sharded_emulated.py tests/test_gpu_deepfm_fused.py tests/test_distributed.py -q --timeout 150 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -25 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc $rc"; exit $rc; fi
timeout -k 10 200 python -u tools/dcn_rt_time.py > $O/dcn_rt_time.log 2>&1 || { echo "dcn timing failed"; tail $O/dcn_rt_time.log; exit 1; }
cat $O/dcn_rt_time.log
timeout -k 10 120 ./tools/bin/gather_probe > $O/gather_probe.log 2>&1 || { echo "gather probe failed"; exit 1; }
grep -E "65536|copy" $O/gather_probe.log
echo check done
