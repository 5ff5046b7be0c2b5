#!/bin/bash
# DeepFM 32-row workgroups (RT = 2): the DeepFM / sharded tests, then the bench's DeepFM and
# sharded legs (with the modelled curve) with the default row tiles and forced to 1, twice interleaved.
set -o pipefail
T=$1; O=gpurun_out/r04; export TMPDIR=/tmp; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_deepfm_fused.py tests/test_sharded_emulated.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > $O/test_$T.log 2>&1 || { echo "tests failed"; tail -30 $O/test_$T.log; exit 1; }
tail -1 $O/test_$T.log
for k in 1 2; do
  for rt in def 1; do
    if [ $rt = def ]; then unset RANKOPS_DEEPFM_ROW_TILES; else export RANKOPS_DEEPFM_ROW_TILES=$rt; fi
    timeout -k 10 300 python bench.py --no-cpu --no-loader --no-train --models deepfm > $O/ab_${T}${k}_$rt.json 2> $O/ab_${T}${k}_$rt.err || { echo "bench failed"; tail -5 $O/ab_${T}${k}_$rt.err; exit 1; }
    python - $O/ab_${T}${k}_$rt.json $rt <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
m = d.get("models", {}); s = d.get("sharded_deepfm", {})
c = s.get("model_curve", {})
print(sys.argv[2], "din", round(d["value"] / 1e6, 2), "deepfm", m.get("deepfm", {}).get("ms_per_step"), "sharded P=1",
      s.get("ms_per_step"), "curve", json.dumps(c)[:400])
PY
  done
done
