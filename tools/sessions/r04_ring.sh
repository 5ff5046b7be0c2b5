set -o pipefail
export ABDIR=gpurun_out/r04
P=implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd/rankops
bash tools/sessions/ab_bench.sh ring $P/librankops.so $P/librankops_r12.so $P/librankops_r16.so && bash tools/sessions/ab_bench.sh ring2 $P/librankops.so $P/librankops_r12.so $P/librankops_r16.so || exit 1
RANKOPS_LIB=$PWD/$P/librankops_phases.so timeout -k 10 120 python tools/dcn_phases.py > gpurun_out/r04/dcn_phases_stream.log 2>&1 || exit 1
RANKOPS_LIB=$PWD/$P/librankops_phases.so timeout -k 10 120 python tools/din_phases.py > gpurun_out/r04/din_phases_stream.log 2>&1 || exit 1
cat gpurun_out/r04/dcn_phases_stream.log gpurun_out/r04/din_phases_stream.log
