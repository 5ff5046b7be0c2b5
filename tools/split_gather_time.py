"""rk_shard_gather_rows_split at configs[4]'s P = 8 shape (rank 0: 4 fields of 1e8 / 30 rows, D 32,
8 sources x 8,192 samples): device time per launch from 20 launches captured in one hipGraph
(bench.graph_kernel_avg_ms) for the grouped form and the flattened one (RANKOPS_SHARD_SPLIT_FLAT=1,
read once per process, hence one child process per form), and the two outputs compared by checksum.
Extra forms: SPLIT_VARIANTS="name=path/to/lib.so,..." (grouped form of another build, via RANKOPS_LIB).
Usage: python tools/split_gather_time.py [P] [B_l] [F]"""
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(P, B, F):
    sys.path.insert(0, ROOT)
    import torch
    import bench
    import rankops
    from rankops import ops
    from rankops._lib import Segment
    torch.cuda.set_device(0)
    rankops.load_library()
    lib = ops._lib.load()
    V, D = 100_000_000 // 30, 32
    g = torch.Generator(device="cuda").manual_seed(5)
    second = [torch.randn(V, D, device="cuda", generator=g) for _ in range(F)]
    first = [torch.randn(V, 1, device="cuda", generator=g) for _ in range(F)]
    idx = torch.randint(0, V, (P, B, F), device="cuda", dtype=torch.int32, generator=g)
    blk = B * F * D + (B + 3) // 4 * 4
    out = torch.empty(P * blk, device="cuda")
    ops._lib.ensure_device(out.device)
    s2 = ops._seg_array([Segment(t.data_ptr(), None, 0, t.stride(0), V, D, 0) for t in second])
    s1 = ops._seg_array([Segment(t.data_ptr(), None, 0, t.stride(0), V, 1, 0) for t in first])

    def fn():
        ops.check(lib.rk_shard_gather_rows_split(s2, s1, F, D, idx.data_ptr(), P, B, 0, B, out.data_ptr(),
                                                 ops._lib.stream_of(out)), "rk_shard_gather_rows_split")

    fn()
    torch.cuda.synchronize()
    digest = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()
    us = bench.graph_kernel_avg_ms(fn) * 1e3
    byts = P * B * F * (4 + 2 * 4 * D + 4) + P * B * 4  # index + row read/write + first-order read, + partial write
    print(json.dumps({"us": us, "digest": digest, "GBps": byts / us / 1e3}))


def main():
    P, B, F = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (8, 8192, 4)))
    res = {}
    forms = [("grouped", "0", None), ("grouped_no_nts", "0", None), ("flat", "1", None)]
    for v in filter(None, os.environ.get("SPLIT_VARIANTS", "").split(",")):
        name, lib = v.split("=")
        forms.append((name, "0", os.path.join(ROOT, lib)))
    for form, flat, lib in forms:
        env = dict(os.environ, RANKOPS_SHARD_SPLIT_FLAT=flat)
        if form == "grouped_no_nts":  # round 6: the grouped form with ordinary send-buffer stores
            env["RANKOPS_SHARD_NTS"] = "0"
        if lib:
            env["RANKOPS_LIB"] = lib
        out = subprocess.run([sys.executable, __file__, "--child", str(P), str(B), str(F)], env=env,
                             capture_output=True, text=True, timeout=300)
        if out.returncode:
            print(out.stderr[-2000:])
            sys.exit(out.returncode)
        res[form] = json.loads(out.stdout.strip().splitlines()[-1])
        print(form, res[form], flush=True)
    print("identical", all(r["digest"] == res["grouped"]["digest"] for r in res.values()),
          "speedup over flat", {k: round(res["flat"]["us"] / r["us"], 3) for k, r in res.items()})


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(*(int(a) for a in sys.argv[2:5]))
    else:
        main()
