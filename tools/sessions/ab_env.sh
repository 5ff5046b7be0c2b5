#!/bin/bash
# A/B of one environment switch on the bench's forward legs (one library build): for each value,
# the headline + DCN / DeepFM / BST legs with VAR=value.  Usage (on the box):
#   bash tools/sessions/ab_env.sh <tag> <VAR> <value>...
set -o pipefail
T=$1; V=$2; shift 2; O=gpurun_out/r04; mkdir -p $O
for X in "$@"; do
  env $V=$X timeout -k 10 300 python bench.py --no-cpu --no-loader --no-train --no-sharded --models dcn,deepfm,bst > $O/ab_${T}_$X.json 2> $O/ab_${T}_$X.err || { echo "bench $V=$X failed"; tail -5 $O/ab_${T}_$X.err; exit 1; }
  python - $O/ab_${T}_$X.json "$V=$X" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
m = d.get("models", {})
print(sys.argv[2], "din", round(d["value"] / 1e6, 2), "M  kernel", d["roofline"]["avg_launch_ms"], "| " + " ".join(
    f"{k} {round(v['samples_per_s'] / 1e6, 2)}M {v['ms_per_step']}ms" for k, v in m.items()))
PY
done
