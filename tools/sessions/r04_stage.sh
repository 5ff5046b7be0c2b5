#!/bin/bash
# DIN / DCN phase marks (timing builds): the default carve against one without the epilogue image.
set -o pipefail
T=${1:-stage}; O=gpurun_out/r04; mkdir -p $O; export TMPDIR=/tmp
P=$PWD/implementation-of-rank-algorithm-for-mainstream-recommender-systems_amd/rankops
RANKOPS_LIB=$P/librankops_phases.so timeout -k 10 120 python tools/din_phases.py > $O/din_phases_$T.log 2>&1 || { echo din phases failed; tail $O/din_phases_$T.log; exit 1; }
RANKOPS_LIB=$P/librankops_phases_noepi.so timeout -k 10 120 python tools/din_phases.py > $O/din_phases_${T}_noepi.log 2>&1 || { echo noepi failed; exit 1; }
RANKOPS_LIB=$P/librankops_phases.so timeout -k 10 120 python tools/dcn_phases.py > $O/dcn_phases_$T.log 2>&1 || { echo dcn phases failed; exit 1; }
head -12 $O/din_phases_$T.log; echo ---; head -12 $O/din_phases_${T}_noepi.log; echo ---; head -8 $O/dcn_phases_$T.log
