#!/bin/bash
# Round-5 GPU step: sharded DeepFM tests (cross-batch pipeline, emulated P = 2/4/8) and the sharded
# leg with its modelled 1->8 curve (pipelined column).  Usage (on the box): bash tools/sessions/r05_sharded.sh <tag>
set -o pipefail
T=${1:-sh1}; O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_sharded_emulated.py tests/test_distributed.py -x -q --timeout 200 --timeout-method thread > $O/test_sharded_$T.log 2>&1 || { echo "sharded tests failed"; tail -60 $O/test_sharded_$T.log; exit 1; }
tail -1 $O/test_sharded_$T.log
timeout -k 10 400 python bench.py --no-cpu --no-loader --no-train --models "" > $O/bench_sharded_$T.json 2> $O/bench_sharded_$T.err || { echo "bench failed"; tail -20 $O/bench_sharded_$T.err; exit 1; }
python - $O/bench_sharded_$T.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("headline", d["value"], d["roofline"]["avg_launch_ms"])
c = d.get("sharded_deepfm", {})
print("P1", c.get("ms_per_step"))
for p, e in c.get("model_curve", {}).get("curve", {}).items():
    if p != "1":
        print(p, json.dumps({k: e[k] for k in ("pipelined_compute_ms", "wire_ms", "ms_per_step", "speedup_vs_p1", "pipelined_bound")}))
PY
