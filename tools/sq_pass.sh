#!/bin/bash
# One SQ-counter pass over a python driver: tools/sq_pass.sh <outdir> <driver.py> [args...]
OUT=$1; shift; ROOT=$(pwd); export TMPDIR=/tmp; mkdir -p "$OUT"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$ROOT/$OUT/a" -o run --output-format csv -- python3 "$@" > "$ROOT/$OUT/a.log" 2>&1 || { echo "pass a failed"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS SQ_WAVES -d "$ROOT/$OUT/b" -o run --output-format csv -- python3 "$@" > "$ROOT/$OUT/b.log" 2>&1 || { echo "pass b failed"; exit 1; }
echo sq ok
