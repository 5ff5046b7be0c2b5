"""Per-workload kernel timing driver for rocprofv3: replays one benchmark workload's forward
graph N times so the kernel trace holds only that model's kernels.

    rocprofv3 --kernel-trace --stats -d out -o dcn --output-format csv -- \
        python3 tools/kprof.py --workload dcn --iters 50
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="din")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--eager", action="store_true")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    import rankops
    rankops.load_library()
    batch = args.batch or (2048 if args.workload == "bst" else 4096)
    # rk_fm_gather alone (bench.py gather_roofline): packed [V, 36] tables, or (_tables) the
    # line-aligned [V, 32] second-order rows with the first-order weights in their own [V, 1] table
    gather = args.workload in ("deepfm_gather", "deepfm_gather_tables")
    blocks = args.workload == "bst_ref_blocks"  # the d-16 blocks + pooling launch alone (bench roofline)
    model, inp, fn, cfg, name = bench.workload("deepfm" if gather else "bst_ref" if blocks else args.workload,
                                               batch, 0)
    if blocks:
        bl = model.blocks_kernel_launcher(inp["seq_feedid"], inp["seq_length"])
        fn = lambda: [bl() for _ in range(20)]  # noqa: E731
    if gather:
        launch = model.gather_launcher(inp["category"], packed=args.workload == "deepfm_gather")
        fn = lambda: [launch() for _ in range(20)]  # noqa: E731
    torch.cuda.synchronize()
    if args.eager:
        with torch.no_grad():
            for _ in range(args.iters):
                fn()
    else:
        g, _ = bench.graph_of(fn)
        for _ in range(args.iters):
            g.replay()
    torch.cuda.synchronize()
    print(f"{args.workload}: {args.iters} forwards of batch {batch} done")


if __name__ == "__main__":
    main()
