set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/bsttr
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bsttr -o bst --output-format csv -- python3 tools/kprof_train.py --model bst --steps 10 > gpurun_out/bsttr/log.txt 2>&1
