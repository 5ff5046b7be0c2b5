"""DIN's balanced assignment ranked over the whole batch (NIT 4 / 8) or per 1,024-sample universe
(RANKOPS_DIN_UNI=1, NIT 1): two prepared plans of the bench workload built under each setting
(the switch is read when the plan is made), timed interleaved (bench.kernel_avg_ms), outputs compared.

    python3 tools/din_uni_ab.py --batches 4096,65536
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
    ap.add_argument("--batches", default="4096")
    ap.add_argument("--rounds", type=int, default=4)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    import rankops
    rankops.load_library()
    for B in [int(b) for b in args.batches.split(",")]:
        model, inp, fn, cfg, name = bench.workload("din", B, 0)
        runs = {}
        for lab, val in (("batch", "0"), ("universe", "1")):
            os.environ["RANKOPS_DIN_UNI"] = val
            runs[lab] = model.prepare(inp["dense"], inp["category"], inp["sequence"], inp["target"])
        os.environ.pop("RANKOPS_DIN_UNI", None)
        outs = {}
        for lab, run in runs.items():
            with torch.no_grad():
                o = run()
            torch.cuda.synchronize()
            outs[lab] = [t.clone() if isinstance(t, torch.Tensor) else t for t in o]
        for a_, b_ in zip(outs["batch"], outs["universe"]):
            if isinstance(a_, torch.Tensor):
                print(f"B {B}: max |diff| {float((a_ - b_).abs().max()):.3g}  equal {torch.equal(a_, b_)}")
        times = {lab: [] for lab in runs}
        for _ in range(args.rounds):
            for lab, run in runs.items():
                times[lab].append(bench.kernel_avg_ms(run))
        for lab, ts in times.items():
            print(f"din B {B} {lab:9s}: {1e3 * min(ts):7.2f} us min, {1e3 * sum(ts) / len(ts):7.2f} us mean")
        del runs, model, inp
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
