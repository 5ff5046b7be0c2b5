#!/bin/bash
# Round-6 gather calibration on the GPU box: the probe's timings, the available TCC counters, then
# one --pmc pass per counter over the calibration kernels (known bytes) and the gather variants.
# Usage (on the box): bash tools/sessions/r06_gather.sh <tag>
set -o pipefail
T=${1:-g1}; O=gpurun_out/r06/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 180 tools/bin/gather_probe2 > $O/probe.log 2>&1 || { echo "probe failed"; tail $O/probe.log; exit 1; }
cat $O/probe.log
timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || echo "list-avail rc $?"
grep -o "TCC_EA0_RD[A-Z0-9_]*\|TCC_EA0_WR[A-Z0-9_]*\|TCC_BUBBLE[A-Z0-9_]*\|TCC_REQ[A-Z0-9_]*" $O/avail.txt | sort -u > $O/tcc_counters.txt || true
cat $O/tcc_counters.txt
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c -d $O/pmc_$c -o run --output-format csv -- tools/bin/gather_probe2 "${2:-}" > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -3 $O/pmc_$c.log; exit 1; }
done
# request counts by size where the part exposes them (best effort: a name it lacks fails fast)
for c in TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B; do
  grep -qx "$c" $O/tcc_counters.txt || continue
  timeout -s KILL 90 rocprofv3 --pmc ${c}_sum -d $O/pmc_$c -o run --output-format csv -- tools/bin/gather_probe2 "${2:-}" > $O/pmc_$c.log 2>&1 || { echo "pmc $c rc $?"; tail -3 $O/pmc_$c.log; }
done
echo gather session done
