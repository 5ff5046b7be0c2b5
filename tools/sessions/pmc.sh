#!/bin/bash
# PMC traffic passes for one workload/kernel: [BATCH=n] tools/pmc.sh <workload> <kernel-substring> [outdir]
# (key in profiles/traffic.json: "<workload>:<kernel>", or "<workload>@<BATCH>:<kernel>" with BATCH set)
W=$1; K=$2; OUT=${3:-gpurun_out/pmc_$1${BATCH:+_$BATCH}}
ROOT=$(pwd); export TMPDIR=/tmp
BARG=${BATCH:+--batch $BATCH}
mkdir -p "$OUT"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$ROOT/$OUT/fetch" -o run --output-format csv -- \
  python3 "$ROOT/tools/kprof.py" --workload "$W" --iters 20 $BARG > "$ROOT/$OUT/fetch.log" 2>&1 || { echo "fetch pass failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$ROOT/$OUT/write" -o run --output-format csv -- \
  python3 "$ROOT/tools/kprof.py" --workload "$W" --iters 20 $BARG > "$ROOT/$OUT/write.log" 2>&1 || { echo "write pass failed"; exit 1; }
python3 "$ROOT/tools/pmc_traffic.py" "$ROOT/$OUT" "$W${BATCH:+@$BATCH}" "$K"
