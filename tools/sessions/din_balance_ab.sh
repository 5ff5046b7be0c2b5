#!/bin/bash
# A/B of DIN's balanced sample assignment (RANKOPS_DIN_BALANCE=0 keeps contiguous 16-sample
# blocks) on the headline leg, alternated 3x.  Usage (on the box): bash tools/din_balance_ab.sh <tag>
set -o pipefail
T=$1; O=gpurun_out/r03; mkdir -p $O
for i in 1 2 3; do
  for B in 0 1; do
    RANKOPS_DIN_BALANCE=$B timeout -k 10 200 python bench.py --no-cpu --no-loader --no-train --no-sharded --models din_zipf > $O/bal_${T}_${B}_$i.json 2> $O/bal_${T}_${B}_$i.err || { echo "bench bal=$B failed"; tail -5 $O/bal_${T}_${B}_$i.err; exit 1; }
    python - $O/bal_${T}_${B}_$i.json $B <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
m = d.get("models", {})
print("balance", sys.argv[2], "din", round(d["value"] / 1e6, 2), "M  kernel", d["roofline"]["avg_launch_ms"], "| " + " ".join(
    f"{k} {round(v['samples_per_s'] / 1e6, 2)}M {v['ms_per_step']}ms" for k, v in m.items()))
PY
  done
done
