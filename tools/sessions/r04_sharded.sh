#!/bin/bash
# Round-4 GPU step: sharded DeepFM tests (fused front end, int32 wire) and the sharded leg with its
# modelled 1->8 curve.  Usage (on the box): bash tools/sessions/r04_sharded.sh <tag>
set -o pipefail
T=${1:-sh1}; O=gpurun_out/r04; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_sharded_emulated.py tests/test_gpu_fm_linear.py -x -q --timeout 150 --timeout-method thread > $O/test_sharded_$T.log 2>&1 || { echo "sharded tests failed"; tail -40 $O/test_sharded_$T.log; exit 1; }
tail -1 $O/test_sharded_$T.log
timeout -k 10 400 python bench.py --no-cpu --no-loader --no-train --models "" > $O/bench_sharded_$T.json 2> $O/bench_sharded_$T.err || { echo "bench failed"; tail -20 $O/bench_sharded_$T.err; exit 1; }
python - $O/bench_sharded_$T.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(json.dumps(d.get("sharded_deepfm"), indent=1)[:3000])
PY
