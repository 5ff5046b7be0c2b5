#!/bin/bash
# A/B: the streamed tail with split accumulators on single-tile layers (librankops_split.so) against the default.
set -o pipefail
export ABDIR=gpurun_out/r04
P=implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd/rankops
bash tools/sessions/ab_bench.sh split $P/librankops.so $P/librankops_split.so && bash tools/sessions/ab_bench.sh split2 $P/librankops.so $P/librankops_split.so
