"""One rank of tests/test_gpu_process_group.py: ShardedDeepFM (BASELINE configs[4]'s field shape)
over a REAL torch.distributed process group — gloo with the tensors on cuda:0, since RCCL refuses
two ranks on one GPU (profiles/r05/rccl_pair.log) — with every device step the real HIP one.

Run as a child process by the test (env: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT, RK_OUT):
  1. run_steps with the local batch split in chunks (async row all-to-alls waited in order);
  2. ShardedDeepFM.pipeline (the cross-batch exchange pipeline), eager, 5 batches + flush;
  3. the captured pipeline bench.py drives (pack / gather / forward as hipGraphs per slot), 5 steps
     + flush over its three bound batches.
Every batch's outputs are compared on this rank with oracle.reference_forward.deepfm_forward
(deepfm.py:121-151) over the global batch; the verdict goes to RK_OUT as JSON."""
import json
import os
import sys
import traceback

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import helpers as H  # noqa: E402
from oracle import reference_forward as ref  # noqa: E402
from rankops import sharded  # noqa: E402

FIELDS30 = {f"field_{i:02d}": 300 + 37 * i for i in range(30)}
CFG30 = {"dim": 32, "fields": FIELDS30, "hidden": [512, 256, 128]}
NAMES = ("prob", "total_logit", "fm1", "fm2", "deep_logit")


def check(got, expect, lo, hi, what):
    for n, g, e in zip(NAMES, got, expect):
        torch.testing.assert_close(g.detach().cpu(), e[lo:hi], atol=1e-4, rtol=1e-4,
                                   msg=lambda m: f"{what} {n}: {m}")


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    out_path = os.environ["RK_OUT"]
    res = {"rank": rank, "ok": False}
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo")
        import rankops
        rankops.load_library()
        B_l = int(os.environ.get("RK_BATCH", "520"))
        full = H.build("deepfm", CFG30, seed=42).cuda()
        sh = sharded.ShardedDeepFM.from_deepfm(full, rank=rank, world_size=world)
        assert sh.exchange_fn is None and sh.world == world  # the real all_to_all_single
        assert sh.split_wire(), "configs[4]'s shape takes the split wire format"
        params = H.cpu_params(full)

        def batch(seed):
            cat = H.make_inputs("deepfm", CFG30, B_l * world, seed=seed)["category"]
            with torch.no_grad():
                exp = ref.deepfm_forward(params, cat, list(FIELDS30), len(CFG30["hidden"]))
            mine = {f: v[rank * B_l:(rank + 1) * B_l].contiguous().cuda() for f, v in cat.items()}
            return mine, exp

        lo, hi = rank * B_l, (rank + 1) * B_l
        # 1. run_steps, chunked: per chunk gather -> async row exchange, waited in order
        sh.min_chunk = 128
        mine, exp = batch(11)
        with torch.no_grad():
            got = sh.run_steps(mine, chunks=3)
        torch.cuda.synchronize()
        check(got, exp, lo, hi, "run_steps chunks=3")
        res["run_steps"] = "ok"

        # 2. the cross-batch pipeline, eager: batch i's outputs come back at push(i + 2) / flush()
        data = [batch(700 + i) for i in range(5)]
        pipe = sh.pipeline(B_l)
        outs = []
        with torch.no_grad():
            for i, (m, _) in enumerate(data):
                o = pipe.push(m)
                assert (o is None) == (i < 2)
                if o is not None:
                    outs.append(o)
            outs.extend(pipe.flush())
        torch.cuda.synchronize()
        assert len(outs) == len(data)
        for i, (o, (_, e)) in enumerate(zip(outs, data)):
            check(o, e, lo, hi, f"pipeline batch {i}")
        res["pipeline"] = "ok"

        # 3. the captured pipeline (bench.py's step): three slots bound to three batches
        data3 = [batch(900 + i) for i in range(3)]
        with torch.no_grad():
            cp = sh.pipeline(B_l, capture=[m for m, _ in data3])
            outs = []
            for i in range(5):
                o = cp.step()
                if o is not None:  # slot outputs are overwritten three steps later: copy now
                    torch.cuda.synchronize()
                    outs.append(tuple(x.cpu() for x in o))
            for o in cp.flush():
                torch.cuda.synchronize()
                outs.append(tuple(x.cpu() for x in o))
        assert len(outs) == 5
        for i, o in enumerate(outs):
            check(o, data3[i % 3][1], lo, hi, f"captured step batch {i}")
        res["captured"] = "ok"
        res["error_flags"] = int(rankops.error_flags())
        assert res["error_flags"] == 0
        res["ok"] = True
    except Exception as exc:  # reported to the parent test
        res["error"] = traceback.format_exc()[-3000:] + repr(exc)
    finally:
        with open(out_path, "w") as f:
            json.dump(res, f)
        if dist.is_initialized():
            dist.destroy_process_group()


if __name__ == "__main__":
    main()
