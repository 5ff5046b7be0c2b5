#!/bin/bash
# PMC traffic passes for one workload/kernel: tools/pmc.sh <workload> <kernel-substring> [outdir]
W=$1; K=$2; OUT=${3:-gpurun_out/pmc_$1}
ROOT=$(pwd); export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$ROOT/$OUT/fetch" -o run --output-format csv -- \
  python3 "$ROOT/tools/kprof.py" --workload "$W" --iters 20 > "$ROOT/$OUT/fetch.log" 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$ROOT/$OUT/write" -o run --output-format csv -- \
  python3 "$ROOT/tools/kprof.py" --workload "$W" --iters 20 > "$ROOT/$OUT/write.log" 2>&1 || { echo "write pass failed"; exit 1; }
python3 "$ROOT/tools/pmc_traffic.py" "$ROOT/$OUT" "$W" "$K"
