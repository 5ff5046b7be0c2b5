#!/bin/bash
# Round-end measurement: the full bench line, then the bench command under rocprofv3 kernel-trace stats.
set -o pipefail
T=${1:-final}; O=gpurun_out/bench_$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --details $O/bench_details.json > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
tail -c 400 $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 bench.py --no-cpu --no-loader --details $O/bench_under_rocprof_details.json > $O/bench_under_rocprof.json 2> $O/prof.err || { echo "rocprof bench failed"; tail -5 $O/prof.err; exit 1; }
echo done
