"""Multi-process tests of the table-sharded DeepFM exchange (rankops.sharded) on CPU with the
gloo backend, world sizes 2 and 3: the real all_to_all_single index/row exchanges run; the
two device steps (local table gather, FM + deep tail) are replaced by CPU stand-ins defined
here, so the routing/layout logic is checked end to end against the single-process oracle.
The device steps themselves are covered at P = 1 by the GPU test at the bottom."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

import helpers as H
from oracle import reference_forward as ref
from rankops import sharded

FIELDS = {f"f{i:02d}": 40 + 3 * i for i in range(7)}
CFG = {"dim": 8, "fields": FIELDS, "hidden": [16, 8]}


class CpuStepsSharded(sharded.ShardedDeepFM):
    """Device steps done with torch CPU ops (test stand-ins for rk_concat_gather / rk_fm_gather /
    rk_mlp_forward); the exchange steps are inherited unchanged."""

    def gather_rows(self, recv_idx, B_src, b0, bc):
        sel = recv_idx.view(self.world, B_src, len(self.local_fields))[:, b0:b0 + bc].reshape(-1)
        return self.gather_local(sel, self.world * bc)

    def gather_local(self, recv_idx, rows_total):
        D, RS, Fm = self.embedding_dim, sharded.row_stride(self.embedding_dim), len(self.local_fields)
        out = torch.full((rows_total, Fm * RS), float("nan"))
        idx = recv_idx.view(rows_total, Fm) if Fm else None
        for j, f in enumerate(self.local_fields):
            out[:, j * RS:j * RS + D] = self.second_order_embeddings[f].weight[idx[:, j]]
            out[:, j * RS + D] = self.first_order_embeddings[f].weight[idx[:, j], 0]
        return out

    def fm_and_tail(self, recv_rows, B_l):
        D, RS = self.embedding_dim, sharded.row_stride(self.embedding_dim)
        off, e2, e1 = 0, {}, {}
        for r in range(self.world):
            fr = self.fields_of[r]
            blk = recv_rows[off:off + B_l * len(fr) * RS].view(B_l, len(fr), RS)
            for j, f in enumerate(fr):
                e2[f], e1[f] = blk[:, j, :D], blk[:, j, D:D + 1]
            off += B_l * len(fr) * RS
        fm1 = torch.sum(torch.cat([e1[f] for f in self.fields], 1), 1, keepdim=True)
        s = torch.stack([e2[f] for f in self.fields], 1)
        fm2 = 0.5 * torch.sum(s.sum(1) ** 2 - (s ** 2).sum(1), 1, keepdim=True)
        h = torch.cat([e2[f] for f in self.fields], 1)
        p = self.state_dict()
        for lin, bn in ref.deepfm_layout(len(self._tail)):
            h = F.linear(h, p[f"deep_layers.{lin}.weight"], p[f"deep_layers.{lin}.bias"])
            h = F.batch_norm(h, p[f"deep_layers.{bn}.running_mean"], p[f"deep_layers.{bn}.running_var"],
                             p[f"deep_layers.{bn}.weight"], p[f"deep_layers.{bn}.bias"], False, 0.0, 1e-5)
            h = torch.relu(h)
        deep = F.linear(h, p["deep_output_layer.weight"], p["deep_output_layer.bias"])
        total = F.linear(torch.cat([fm1, fm2, deep], 1), p["final_layer.weight"], p["final_layer.bias"])
        return torch.sigmoid(total), total, fm1, fm2, deep


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, B, q, chunks=1):
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        full = H.build("deepfm", CFG, seed=42)
        inp = H.make_inputs("deepfm", CFG, B * world, seed=77)
        with torch.no_grad():
            expect = ref.deepfm_forward(H.cpu_params(full), inp["category"], list(FIELDS), len(CFG["hidden"]))
        sh = CpuStepsSharded(dict((f, e.num_embeddings) for f, e in full.second_order_embeddings.items()),
                             CFG["dim"], CFG["hidden"], rank=rank, world_size=world)
        sd = {k: v for k, v in full.state_dict().items()
              if not k.startswith(("first_order", "second_order")) or k.split(".")[1] in sh.local_fields}
        sh.load_state_dict(sd, strict=True)
        sh.eval()
        sh.min_chunk = 4  # pipeline the exchange even at this small batch
        mine = {f: v[rank * B:(rank + 1) * B].contiguous() for f, v in inp["category"].items()}
        assert len(sh.chunk_bounds(B, chunks)) == chunks
        with torch.no_grad():
            got = sh.run_steps(mine, chunks=chunks)
        for g, e in zip(got, expect):
            torch.testing.assert_close(g, e[rank * B:(rank + 1) * B], atol=1e-5, rtol=1e-5)
        # every rank only holds its own fields' tables
        assert set(sh.second_order_embeddings) == {f for i, f in enumerate(FIELDS) if i % world == rank}
        q.put((rank, "ok"))
    except Exception as exc:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc() + repr(exc)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _pipe_worker(rank, world, port, B, q, nbatch):
    """ShardedDeepFM.pipeline (the cross-batch exchange pipeline) over `nbatch` consecutive local
    batches: push() returns batch i - 2's outputs, flush() the last two; all against the oracle."""
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        full = H.build("deepfm", CFG, seed=42)
        sh = CpuStepsSharded(dict((f, e.num_embeddings) for f, e in full.second_order_embeddings.items()),
                             CFG["dim"], CFG["hidden"], rank=rank, world_size=world)
        sd = {k: v for k, v in full.state_dict().items()
              if not k.startswith(("first_order", "second_order")) or k.split(".")[1] in sh.local_fields}
        sh.load_state_dict(sd, strict=True)
        sh.eval()
        batches, expects = [], []
        for i in range(nbatch):
            inp = H.make_inputs("deepfm", CFG, B * world, seed=900 + i)
            with torch.no_grad():
                expects.append(ref.deepfm_forward(H.cpu_params(full), inp["category"], list(FIELDS),
                                                  len(CFG["hidden"])))
            batches.append({f: v[rank * B:(rank + 1) * B].contiguous() for f, v in inp["category"].items()})
        pipe = sh.pipeline(B)
        got = []
        with torch.no_grad():
            for i, cat in enumerate(batches):
                out = pipe.push(cat)
                assert (out is None) == (i < 2)
                if out is not None:
                    got.append(out)
            got.extend(pipe.flush())
        assert len(got) == nbatch
        for g, e in zip(got, expects):
            for x, y in zip(g, e):
                torch.testing.assert_close(x, y[rank * B:(rank + 1) * B], atol=1e-5, rtol=1e-5)
        q.put((rank, "ok"))
    except Exception as exc:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc() + repr(exc)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _spawn(target, world, B, extra):
    """Runs target(rank, world, port, B, queue, extra) on `world` spawned processes; the failures."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, B, q, extra)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    return [r for r in results if r[1] != "ok"]


@pytest.mark.parametrize("world,nbatch", [(2, 2), (2, 5), (3, 1), (3, 4)])
def test_sharded_deepfm_cross_batch_pipeline_gloo(world, nbatch):
    """The cross-batch pipeline at world 2 / 3 with real gloo all-to-alls, 1-5 batches (fill, steady
    state and drain): every batch's outputs equal the single-process oracle's."""
    bad = _spawn(_pipe_worker, world, 16, nbatch)
    assert not bad, bad


@pytest.mark.parametrize("world,chunks", [(2, 1), (3, 1), (2, 3), (3, 4)])
def test_sharded_deepfm_exchange_gloo(world, chunks):
    """Exchange routing at world 2 / 3, unpipelined and with the batch split into 3-4 chunks whose
    all-to-alls run asynchronously (async_op work objects waited in pipeline order)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 24, q, chunks)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    bad = [r for r in results if r[1] != "ok"]
    assert not bad, bad


def test_field_ownership_balanced():
    own = sharded.field_owner(30, 8)
    counts = [own.count(r) for r in range(8)]
    assert counts == [4, 4, 4, 4, 4, 4, 3, 3]
    assert sharded.row_stride(32) == 36 and sharded.row_stride(8) == 12


@pytest.mark.gpu
def test_sharded_single_rank_equals_deepfm_on_gpu():
    """P = 1: the sharded module (device gather into exchange rows + FM over dense segments)
    reproduces DeepFM.forward on the same weights."""
    cfg = {"dim": 32, "fields": {f"f{i:02d}": 500 + i for i in range(30)}}
    full = H.build("deepfm", cfg).cuda()
    sh = sharded.ShardedDeepFM.from_deepfm(full, rank=0, world_size=1)
    inp = H.to_device(H.make_inputs("deepfm", cfg, 333), "cuda")
    with torch.no_grad():
        a = full(inp["category"])
        b = sh(inp["category"])
    for x, y in zip(a, b):
        torch.testing.assert_close(x, y, atol=1e-5, rtol=1e-5)


def test_front_ok_without_hidden_layers():
    """with hidden_units=[] the fused front end is off (no IndexError on the empty tail)."""
    sh = sharded.ShardedDeepFM({"a": 10, "b": 12}, 8, [], rank=0, world_size=1)
    assert sh._front_ok(64) is False
