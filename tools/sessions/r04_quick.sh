set -o pipefail
O=gpurun_out/r04; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu --no-loader --no-train --no-sharded --models ${MODELS:-dcn,deepfm,bst,bst_ref,din_per_call,dcn_per_call} > $O/bench_q1.json 2> $O/bench_q1.err || { tail -20 $O/bench_q1.err; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/trace_bst_ref -o run --output-format csv -- python3 tools/kprof.py --workload bst_ref --iters 30 > $O/trace_bst_ref.log 2>&1 || exit 1
find $O/trace_bst_ref -name "*kernel_trace.csv" -delete
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r04/bench_q1.json").read().strip().splitlines()[-1])
print("headline", d["value"], json.dumps(d["roofline"])[:900])
for k, v in d["models"].items():
    print(k, v.get("samples_per_s"), v.get("ms_per_step"), json.dumps(v.get("roofline"))[:600], json.dumps(v.get("mfma_busy"))[:300])
PY
