#!/bin/bash
# Round-5 quick GPU step: bench.py with a chosen model list, no CPU / loader / train legs; prints the
# headline, the chosen legs' rooflines and the sharded model curve.
# Usage (on the box): bash tools/sessions/r05_quick.sh <tag> <models> [extra bench args]
set -o pipefail
T=${1:-q1}; M=${2:-dcn}; shift 2; O=gpurun_out/r05; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python bench.py --no-cpu --no-loader --no-train --models "$M" "$@" > $O/bench_$T.json 2> $O/bench_$T.err || { echo "bench failed"; tail -20 $O/bench_$T.err; exit 1; }
python - $O/bench_$T.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("headline", d["value"], d["roofline"]["avg_launch_ms"], d["roofline"]["frac"])
for k, v in d.get("models", {}).items():
    r = v.get("roofline", {})
    print(k, v.get("samples_per_s"), v.get("ms_per_step"), json.dumps({a: b for a, b in r.items() if a.startswith("batch_") or a in ("avg_launch_ms", "frac")})[:600])
c = d.get("sharded_deepfm", {})
print("sharded", c.get("ms_per_step"), c.get("error"))
for p, e in c.get("model_curve", {}).get("curve", {}).items():
    if p != "1":
        print(p, json.dumps({k: e[k] for k in ("pipelined_compute_ms", "wire_ms", "ms_per_step", "speedup_vs_p1", "pipelined_bound")}))
PY
