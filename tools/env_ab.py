"""A/B of a library switch read per call (an environment variable) on one bench workload: the
prepared forward timed as 50 back-to-back launches with HIP events on the stream it launches on
(bench.kernel_avg_ms; a prepared launch binds the current stream at prepare() time),
interleaved over the settings for several rounds, with the outputs compared against the first
setting's (max abs difference).

    python3 tools/env_ab.py --workload afm --var RANKOPS_AFM_S --values 0,2,4 --batches 4096,65536
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import bench  # noqa: E402


def prepared(model, name, inp):
    if name == "afm":
        return model.prepare(inp["dense_input"], inp["category_input"])
    if name == "deepcrossing":
        return model.prepare(inp["dense"], inp["category"])
    if name in ("dcn",):
        return model.prepare(inp["dense"], inp["category"])
    if name == "din":
        return model.prepare(inp["dense"], inp["category"], inp["sequence"], inp["target"])
    if name == "bst_ref":
        return model.prepare(inp["dense"], inp["category"], inp["seq_feedid"], inp["seq_length"])
    if name == "deepfm":
        return model.prepare(inp["category"])
    if name == "fwfm":
        return model.prepare(inp["x"])
    raise ValueError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="afm")
    ap.add_argument("--var", required=True)
    ap.add_argument("--values", required=True)
    ap.add_argument("--batches", default="4096")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    import rankops
    rankops.load_library()
    values = args.values.split(",")
    for B in [int(b) for b in args.batches.split(",")]:
        model, inp, fn, cfg, name = bench.workload(args.workload, B, 0)
        run = prepared(model, args.workload, inp)
        ref = None
        times = {v: [] for v in values}
        for rnd in range(args.rounds):
            for v in values:
                os.environ[args.var] = v
                with torch.no_grad():
                    out = [o.clone() for o in run()]
                torch.cuda.synchronize()
                if ref is None:
                    ref = out
                diff = max(float((a - b).abs().max()) for a, b in zip(out, ref))
                ms = bench.kernel_avg_ms(run)
                times[v].append(ms)
                if rnd == 0:
                    print(f"{args.workload} B {B} {args.var}={v}: max |diff| vs {values[0]} = {diff:.3g}", flush=True)
        for v in values:
            ts = times[v]
            print(f"{args.workload} B {B} {args.var}={v}: {1e3 * min(ts):8.2f} us min, {1e3 * sum(ts) / len(ts):8.2f} "
                  f"us mean over {len(ts)} rounds  -> {B / (min(ts) * 1e-3) / 1e6:.1f} M samples/s", flush=True)
        os.environ.pop(args.var, None)
        del model, inp, run
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
