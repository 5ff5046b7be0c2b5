#!/bin/bash
# Round-6 counter session on the GPU box: per workload two SQ passes (MFMA busy, waits, LDS) and a
# kernel trace of the forward; FETCH_SIZE / WRITE_SIZE passes for the headline kernel and the
# standalone gather (both layouts); then tools/pmc_counters.py digests it into <session>/counters.json.
# Usage (on the box): bash tools/sessions/r06_counters.sh <tag> [workloads...]
set -o pipefail
T=${1:-base}; shift
WL=${@:-din dcn deepfm bst bst_ref bst_ref_blocks afm deepcrossing}
O=gpurun_out/r06/$T; mkdir -p $O
export TMPDIR=/tmp
for w in $WL; do
  bash tools/sq_pass.sh $O/sq_$w tools/kprof.py --workload $w --iters 20 || exit 1
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace_$w -o run --output-format csv -- \
    python3 tools/kprof.py --workload $w --iters 50 > $O/trace_$w.log 2>&1 || { echo "trace $w failed"; exit 1; }
  find $O/trace_$w -name "*kernel_trace.csv" -delete
  echo "$w done"
done
pmc() {  # <name> <kprof args...>
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_$n/fetch -o run --output-format csv -- python3 tools/kprof.py "$@" > $O/pmc_$n.log 2>&1 || return 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_$n/write -o run --output-format csv -- python3 tools/kprof.py "$@" >> $O/pmc_$n.log 2>&1 || return 1
}
if [ -z "$NO_PMC" ]; then
  pmc din --workload din --iters 20 || { echo "pmc din failed"; exit 1; }
  pmc deepfm_gather --workload deepfm_gather --iters 3 || { echo "pmc gather failed"; exit 1; }
  pmc deepfm_gather65536 --workload deepfm_gather --iters 3 --batch 65536 || { echo "pmc gather 65536 failed"; exit 1; }
  pmc deepfm_gather_tables65536 --workload deepfm_gather_tables --iters 3 --batch 65536 || { echo "pmc gather tables failed"; exit 1; }
  pmc deepfm_gather_tables --workload deepfm_gather_tables --iters 3 || { echo "pmc gather tables 4096 failed"; exit 1; }
fi
python3 tools/pmc_counters.py $O din:din_forward_kernel dcn:dcn_fused_kernel deepfm:deepfm_fused_kernel \
  bst:bst_block_kernel bst:mlp_stream_kernel bst_ref:bst_mfma_fwd_kernel bst_ref_blocks:bst_mfma_kernel afm:afm_tiles_kernel deepcrossing:dc_forward_kernel \
  deepfm_gather:fm_gather_kernel deepfm_gather65536:fm_gather_fmaj_kernel deepfm_gather_tables65536:fm_gather_fmaj_kernel \
  deepfm_gather_tables:fm_gather_kernel \
  > $O/digest.log 2>&1 || { echo "digest failed"; tail $O/digest.log; exit 1; }
cat $O/digest.log | cut -c1-300
