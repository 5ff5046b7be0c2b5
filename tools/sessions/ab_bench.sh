#!/bin/bash
# A/B of library builds on the headline legs: for each .so given, the bench's forward legs with
# RANKOPS_LIB pointing at it.  Usage (on the box): bash tools/sessions/ab_bench.sh <tag> <lib.so>...
set -o pipefail
T=$1; shift; O=${ABDIR:-gpurun_out/r03}; mkdir -p $O
for L in "$@"; do
  N=$(basename $L .so)
  RANKOPS_LIB=$PWD/$L timeout -k 10 300 python bench.py --no-cpu --no-loader --no-train --no-sharded --models dcn,deepfm,bst > $O/ab_${T}_$N.json 2> $O/ab_${T}_$N.err || { echo "bench $N failed"; tail -5 $O/ab_${T}_$N.err; exit 1; }
  python - $O/ab_${T}_$N.json $N <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
m = d.get("models", {})
print(sys.argv[2], "din", round(d["value"] / 1e6, 2), "M  kernel", d["roofline"]["avg_launch_ms"], "| " + " ".join(
    f"{k} {round(v['samples_per_s'] / 1e6, 2)}M {v['ms_per_step']}ms" for k, v in m.items()))
PY
done
