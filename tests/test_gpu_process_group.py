"""the sharded DeepFM pipeline through a REAL torch.distributed process group with
the real HIP device steps.  Two ranks, both on cuda:0, gloo backend with device tensors (RCCL
refuses two ranks on one GPU); each rank is a child process running tests/dist_pg_worker.py, which
checks run_steps (chunked), ShardedDeepFM.pipeline (eager, 5 batches) and the captured pipeline
bench.py drives (5 steps) against the oracle.  This is the one pre-8-GPU check of work.wait()
stream ordering together with the real gathers and forwards (reference: deepfm.py:121-151)."""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run_ranks(world, tmp_path, timeout=180, batch=520):
    port = _free_port()
    procs, outs = [], []
    for r in range(world):
        out = str(tmp_path / f"rank{r}.json")
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), RK_OUT=out, RK_BATCH=str(batch))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.join(HERE, "dist_pg_worker.py")], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
        outs.append(out)
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=timeout)[0].decode(errors="replace")[-2000:])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    res = []
    for r, out in enumerate(outs):
        if not os.path.exists(out):
            res.append({"rank": r, "ok": False, "error": "no result", "log": logs[r] if r < len(logs) else ""})
        else:
            with open(out) as f:
                res.append(json.load(f))
    return res, [p.returncode for p in procs]


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_pipeline_real_process_group(world, tmp_path):
    res, rcs = _run_ranks(world, tmp_path)
    bad = [r for r in res if not r.get("ok")]
    assert not bad, json.dumps(bad, indent=1)[:6000]
    assert rcs == [0] * world
    for r in res:
        assert r["run_steps"] == r["pipeline"] == r["captured"] == "ok"
