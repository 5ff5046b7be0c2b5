set -o pipefail
mkdir -p gpurun_out/r03
for i in 1 2; do
for B in 0 1; do
RANKOPS_DIN_BALANCE=$B timeout -k 10 120 python bench.py --no-extras --no-cpu --no-loader > gpurun_out/r03/bal_${B}_$i.json 2>/dev/null || exit 1
python -c "import json,sys; d=json.loads(open('gpurun_out/r03/bal_${B}_$i.json').read().strip().splitlines()[-1]); print('balance=$B', d['value'], d['roofline']['avg_launch_ms'])"
done; done
