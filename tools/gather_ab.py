"""rk_fm_gather at DeepFM configs[1]'s tables (30 x 1e6 x 32 + first-order), timed per launch as
bench.gather_roofline does (graph_kernel_avg_ms), for environment settings read per call by the
library, interleaved over several rounds; outputs checked equal to the first setting's.

    python3 tools/gather_ab.py --batch 65536 --settings "base:;v1:RANKOPS_FM_FMAJ_VARIANT=1;sm:RANKOPS_FM_FMAJ_MIN=0"
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
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--settings", required=True)
    ap.add_argument("--packed", action="store_true")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    import helpers as H
    import rankops
    rankops.load_library()
    model, inp, fn, cfg, name = bench.workload("deepfm", 4096, 0)
    cat = H.to_device(H.make_inputs("deepfm", cfg, args.batch, seed=1234), "cuda")["category"]
    launch = model.gather_launcher(cat, packed=args.packed)
    settings = []
    for item in args.settings.split(";"):
        label, _, env = item.partition(":")
        settings.append((label, dict(kv.split("=", 1) for kv in env.split(",") if kv)))
    keys = {k for _, e in settings for k in e}
    plan = model._gather_plan([c for c in model.second_order_embeddings], cat, packed=args.packed)
    times = {lab: [] for lab, _ in settings}
    ref = None
    for rnd in range(args.rounds):
        for lab, env in settings:
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update(env)
            model._launch(plan)
            torch.cuda.synchronize()
            out = [plan[5].clone(), plan[6].clone(), plan[7].clone()]
            if ref is None:
                ref = out
            elif rnd == 0:
                same = torch.equal(out[0], ref[0])
                d = max(float((a - b).abs().max()) for a, b in zip(out[1:], ref[1:]))
                print(f"{lab}: deep_in equal {same}, fm max |diff| {d:.3g}", flush=True)
            times[lab].append(bench.graph_kernel_avg_ms(launch))
    for lab, _ in settings:
        ts = times[lab]
        ms = min(ts)
        print(f"B {args.batch} {'packed' if args.packed else 'tables'} {lab:10s}: {1e3 * ms:8.2f} us min "
              f"({1e3 * sum(ts) / len(ts):8.2f} mean)  frac {bench.DEEPFM_GATHER_BYTES * args.batch / (ms * 1e-3) / 8e12:.4f}",
              flush=True)


if __name__ == "__main__":
    main()
