#!/bin/bash
# Kernel traces of every benchmark workload (one rocprofv3 run each) into $1 (default gpurun_out/kprof).
OUT=${1:-gpurun_out/kprof}
mkdir -p "$OUT"
ROOT=$(pwd)
export TMPDIR=/tmp
for w in ${WORKLOADS:-din dcn deepfm bst}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT" -o "$w" --output-format csv -- \
    python3 "$ROOT/tools/kprof.py" --workload "$w" --iters 40 > "$ROOT/$OUT/$w.log" 2>&1 || { echo "prof $w failed"; exit 1; }
done
echo prof_all ok
