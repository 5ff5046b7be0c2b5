#!/bin/bash
# GPU-box quick check between kernel changes: the GPU test suite, then the bench's forward legs
# (no CPU baseline, loader, training or sharded legs).  Usage (on the box): bash tools/quick_bench.sh <tag>
set -o pipefail
T=${1:-chk}; O=gpurun_out/r03; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest_$T.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/gputest_$T.log; exit 1; }
tail -1 $O/gputest_$T.log
timeout -k 10 300 python bench.py --no-cpu --no-loader --no-train --no-sharded --models dcn,deepfm,bst > $O/bench_$T.json 2> $O/bench_$T.err || { echo "bench failed"; tail -20 $O/bench_$T.err; exit 1; }
python - $O/bench_$T.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("headline", d["value"], "ms", d["ms_per_step"], "frac", d["roofline"]["frac"], "kernel ms", d["roofline"]["avg_launch_ms"])
for k, v in d.get("models", {}).items():
    print(k, v.get("samples_per_s"), v.get("ms_per_step"))
PY
