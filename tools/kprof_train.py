"""Training-step kernel timing driver for rocprofv3: runs bench.bench_train for one model
(eager + hipGraph legs) so the kernel trace holds only that model's training kernels.

    rocprofv3 --kernel-trace --stats -d out -o bst_train --output-format csv -- \
        python3 tools/kprof_train.py --model bst --steps 20
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="bst")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=None)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    import rankops
    rankops.load_library()
    batch = args.batch or (2048 if args.model == "bst" else 4096)
    res = bench.bench_train(batch, args.steps, 3, args.model)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
