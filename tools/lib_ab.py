"""A/B of library builds (RANKOPS_LIB) on one kernel launcher: each build timed in its own child
process (bench.kernel_avg_ms over back-to-back launches, HIP events on the launch stream), the
builds interleaved over several rounds; each child also prints a checksum of the launch's output.

    python3 tools/lib_ab.py --libs base:,ring3:tools/bin/ab/librankops_ring3.so --what bst_blocks
"""
import argparse
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(what, batch):
    sys.path.insert(0, REPO)
    import torch
    import bench
    torch.cuda.set_device(0)
    import rankops
    rankops.load_library()
    if what == "bst_blocks":
        model, inp, fn, cfg, name = bench.workload("bst", batch, 0)
        launch = model.blocks_kernel_launcher(inp["seq_feedid"], inp["seq_length"])
        launch()
        torch.cuda.synchronize()
        ts = [bench.kernel_avg_ms(launch, 20) for _ in range(3)]
        print(f"RESULT {min(ts) * 1e3:.2f} {sum(ts) / len(ts) * 1e3:.2f}", flush=True)
    elif what in ("afm", "deepcrossing"):
        sys.path.insert(0, os.path.join(REPO, "tools"))
        from env_ab import prepared
        model, inp, fn, cfg, name = bench.workload(what, batch, 0)
        run = prepared(model, what, inp)
        with torch.no_grad():
            out = run()
        torch.cuda.synchronize()
        ts = [bench.kernel_avg_ms(run) for _ in range(3)]
        print(f"RESULT {min(ts) * 1e3:.2f} {sum(ts) / len(ts) * 1e3:.2f} {float(out[0].double().sum()):.9e}",
              flush=True)
    else:
        raise ValueError(what)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="")
    ap.add_argument("--what", default="bst_blocks")
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--child", action="store_true")
    args = ap.parse_args()
    if args.child:
        child(args.what, args.batch)
        return
    libs = [item.partition(":")[::2] for item in args.libs.split(",")]
    res = {lab: [] for lab, _ in libs}
    for rnd in range(args.rounds):
        for lab, path in libs:
            env = dict(os.environ)
            if path:
                env["RANKOPS_LIB"] = os.path.join(REPO, path)
            else:
                env.pop("RANKOPS_LIB", None)
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--what", args.what,
                                  "--batch", str(args.batch)], env=env, capture_output=True, text=True, timeout=300)
            line = [l for l in out.stdout.splitlines() if l.startswith("RESULT")]
            if out.returncode != 0 or not line:
                print(f"{lab}: child failed rc={out.returncode}\n{out.stderr[-2000:]}", flush=True)
                sys.exit(1)
            mn, mean = map(float, line[0].split()[1:3])
            res[lab].append(mn)
            extra = " ".join(line[0].split()[3:])
            print(f"round {rnd} {lab:8s}: {mn:8.2f} us min {mean:8.2f} us mean {extra}", flush=True)
    for lab, ts in res.items():
        print(f"{args.what} B {args.batch} {lab:8s}: best {min(ts):8.2f} us, mean of mins {sum(ts) / len(ts):8.2f} us")


if __name__ == "__main__":
    main()
