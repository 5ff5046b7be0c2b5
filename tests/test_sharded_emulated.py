"""The P > 1 table-sharded DeepFM (rankops.sharded, BASELINE configs[4]) with P shards in one
process on one device: every device step is the real one — pack_indices, gather_rows / gather_local
(rk_concat_gather over the packed tables), fm_and_tail (rk_fm_gather over the received rows'
dense segments + the fused tail) and run_steps' chunk pipeline — and only the RCCL transport is
replaced by the in-process all-to-all emulator (tests/a2a_emulator.py).  Outputs are compared
with the oracle (oracle.reference_forward.deepfm_forward: deepfm.py:121-151) at configs[4]'s field
shape: 30 fields, emb_dim 32, 512-256-128, field f on rank f % P (4/4/4/4/4/4/3/3 at P = 8).

The CPU test runs the same emulator under the CPU stand-ins of test_distributed.py, so the
emulator itself is checked against the gloo all_to_all_single routing there."""
import pytest
import torch

import helpers as H
from a2a_emulator import InProcessAllToAll, run_ranks
from oracle import reference_forward as ref
from rankops import sharded

FIELDS30 = {f"field_{i:02d}": 300 + 37 * i for i in range(30)}
CFG30 = {"dim": 32, "fields": FIELDS30, "hidden": [512, 256, 128]}


def _shards(full, world, cls=sharded.ShardedDeepFM, device=None):
    rows = {f: e.num_embeddings for f, e in full.second_order_embeddings.items()}
    hidden = [l.out_features for l in full.deep_layers if isinstance(l, torch.nn.Linear)]
    emu = InProcessAllToAll(world)
    shards = []
    for r in range(world):
        if cls is sharded.ShardedDeepFM:
            sh = cls.from_deepfm(full, rank=r, world_size=world)
        else:
            sh = cls(rows, full.embedding_dim, hidden, rank=r, world_size=world)
            sd = {k: v for k, v in full.state_dict().items()
                  if not k.startswith(("first_order", "second_order")) or k.split(".")[1] in sh.local_fields}
            sh.load_state_dict(sd, strict=True)
            sh.eval()
        sh.exchange_fn = emu.bind(r)
        shards.append(sh)
    return shards, emu


def _oracle(full, cfg, cat):
    with torch.no_grad():
        return ref.deepfm_forward(H.cpu_params(full), {f: v.cpu() for f, v in cat.items()}, list(cfg["fields"]),
                                  len(cfg["hidden"]))


def _check(got, expect, lo, hi, tol):
    names = ("prob", "total_logit", "fm1", "fm2", "deep_logit")
    for n, g, e in zip(names, got, expect):
        torch.testing.assert_close(g.cpu(), e[lo:hi], atol=tol, rtol=tol, msg=lambda m: f"{n}: {m}")


@pytest.mark.parametrize("world,chunks", [(2, 1), (3, 4), (8, 3)])
def test_emulator_routes_like_gloo_cpu(world, chunks):
    """CPU: the emulator under the CPU stand-in device steps reproduces the oracle (the gloo
    routing test's counterpart), so a GPU failure below is a device-step failure."""
    from test_distributed import CFG, CpuStepsSharded
    full = H.build("deepfm", CFG, seed=42)
    B = 24
    inp = H.make_inputs("deepfm", CFG, B * world, seed=77)
    expect = _oracle(full, CFG, inp["category"])
    shards, emu = _shards(full, world, cls=CpuStepsSharded)

    def rank_fn(r):
        sh = shards[r]
        sh.min_chunk = 4
        mine = {f: v[r * B:(r + 1) * B].contiguous() for f, v in inp["category"].items()}
        with torch.no_grad():
            return sh.run_steps(mine, chunks=chunks)

    outs = run_ranks(world, rank_fn, on_error=emu.abort)
    for r, got in enumerate(outs):
        _check(got, expect, r * B, (r + 1) * B, 1e-5)
    assert emu.calls == 1 + chunks  # one index exchange, then one row exchange per chunk


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("chunks", [1, 4])
def test_sharded_pipeline_emulated_on_gpu(world, chunks):
    full = H.build("deepfm", CFG30, seed=42).cuda()
    B_l = 520
    inp = H.to_device(H.make_inputs("deepfm", CFG30, B_l * world, seed=4000 + world), "cuda")
    expect = _oracle(full, CFG30, inp["category"])
    shards, emu = _shards(full, world)
    counts = [len(sh.local_fields) for sh in shards]
    assert counts == [sum(1 for f in range(30) if f % world == r) for r in range(world)]
    if world == 8:
        assert counts == [4, 4, 4, 4, 4, 4, 3, 3]

    def rank_fn(r):
        sh = shards[r]
        sh.min_chunk = 64
        mine = {f: v[r * B_l:(r + 1) * B_l] for f, v in inp["category"].items()}
        assert len(sh.chunk_bounds(B_l, chunks)) == chunks
        with torch.no_grad():
            out = sh(mine) if chunks == sh.pipeline_chunks else sh.run_steps(
                {f: v.contiguous() for f, v in mine.items()}, chunks=chunks)
        torch.cuda.synchronize()
        return tuple(o.cpu() for o in out)

    outs = run_ranks(world, rank_fn, on_error=emu.abort)
    torch.cuda.synchronize()
    for r, got in enumerate(outs):
        _check(got, expect, r * B_l, (r + 1) * B_l, 1e-4)
    import rankops
    assert rankops.error_flags() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 8])
def test_sharded_step_functions_emulated_on_gpu(world):
    """The four steps one by one (index exchange, local gather, row exchange, FM + tail) with the
    packed wire rows: received indices equal the owner's fields of every source, gathered rows
    equal the packed table rows (second order, then the first-order weight at column D), and the
    FM + tail equals the oracle."""
    full = H.build("deepfm", CFG30, seed=42).cuda()
    B_l = 96
    inp = H.to_device(H.make_inputs("deepfm", CFG30, B_l * world, seed=11), "cuda")
    expect = _oracle(full, CFG30, inp["category"])
    shards, emu = _shards(full, world)
    for sh in shards:
        sh.wire = "packed"
    D, RS = 32, sharded.row_stride(32)

    def rank_fn(r):
        sh = shards[r]
        mine = {f: v[r * B_l:(r + 1) * B_l] for f, v in inp["category"].items()}
        with torch.no_grad():
            recv_idx = sh.exchange_indices(mine, B_l)
            rows = sh.gather_local(recv_idx, world * B_l)
            recv_rows = sh.exchange_rows(rows, B_l)
            out = sh.fm_and_tail(recv_rows, B_l)
        torch.cuda.synchronize()
        return recv_idx.cpu(), rows.cpu(), tuple(o.cpu() for o in out)

    outs = run_ranks(world, rank_fn, on_error=emu.abort)
    names = list(FIELDS30)
    for r, (recv_idx, rows, got) in enumerate(outs):
        mine = shards[r].local_fields
        ri = recv_idx.view(world * B_l, len(mine))
        assert ri.dtype == torch.int32  # int32 on the wire (every table < 2^31 rows)
        want_idx = torch.stack([inp["category"][f].cpu() for f in mine], 1)  # sources in order = global rows
        assert torch.equal(ri.long(), want_idx)
        rv = rows.view(world * B_l, len(mine), RS)
        for j, f in enumerate(mine):
            w2 = full.second_order_embeddings[f].weight.detach().cpu()
            w1 = full.first_order_embeddings[f].weight.detach().cpu()
            assert torch.equal(rv[:, j, :D], w2[want_idx[:, j]])
            assert torch.equal(rv[:, j, D], w1[want_idx[:, j], 0])
        _check(got, expect, r * B_l, (r + 1) * B_l, 1e-4)
        assert names.index(mine[0]) == r
    import rankops
    assert rankops.error_flags() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 8])
def test_captured_pipeline_emulated_on_gpu(world):
    """bench.py's world > 1 step (ShardedDeepFM.capture_pipeline: per chunk three hipGraph
    segments with the exchanges between them) driven through the emulator, replayed twice."""
    full = H.build("deepfm", CFG30, seed=42).cuda()
    B_l = 1024
    inp = H.to_device(H.make_inputs("deepfm", CFG30, B_l * world, seed=21), "cuda")
    expect = _oracle(full, CFG30, inp["category"])
    shards, emu = _shards(full, world)
    pipes = []
    for r, sh in enumerate(shards):  # capture is local (no collective): serially, here
        sh.min_chunk = 256
        mine = {f: v[r * B_l:(r + 1) * B_l].contiguous() for f, v in inp["category"].items()}
        pipes.append((sh.capture_pipeline(mine), mine))
    assert len(pipes[0][0].segs) == 4

    def rank_fn(r):
        for _ in range(2):
            pipes[r][0].step()
        torch.cuda.synchronize()
        return tuple(o.cpu() for o in pipes[r][0].result())

    outs = run_ranks(world, rank_fn, on_error=emu.abort)
    for r, got in enumerate(outs):
        _check(got, expect, r * B_l, (r + 1) * B_l, 1e-4)
    assert emu.calls == 2 * (1 + 4)
    import rankops
    assert rankops.error_flags() == 0  # the capture's warm-up gathers read valid (zeroed) indices


@pytest.mark.gpu
@pytest.mark.parametrize("world", [1, 2, 8])
@pytest.mark.parametrize("mode", ["whole", "front", "unfused"])
def test_fused_front_and_unfused_path_match_oracle(world, mode):
    """fm_and_tail / local_fm_and_tail through rk_deepfm_forward (whole: the received rows read in
    place as dense blocks of packed rows; P = 1 from the packed tables), through rk_fm_linear_packed
    + the tail (front) and through the three-launch rk_fm_gather path (unfused), against the oracle;
    ragged local batch."""
    full = H.build("deepfm", CFG30, seed=42).cuda()
    B_l = 333
    inp = H.to_device(H.make_inputs("deepfm", CFG30, B_l * world, seed=600 + world), "cuda")
    expect = _oracle(full, CFG30, inp["category"])
    shards, emu = _shards(full, world)

    def rank_fn(r):
        sh = shards[r]
        sh.fused_whole = mode == "whole"
        sh.fused_front = mode != "unfused"
        mine = {f: v[r * B_l:(r + 1) * B_l].contiguous() for f, v in inp["category"].items()}
        with torch.no_grad():
            out = sh.run_steps(mine, chunks=1)
        torch.cuda.synchronize()
        return tuple(o.cpu() for o in out)

    outs = run_ranks(world, rank_fn, on_error=emu.abort)
    for r, got in enumerate(outs):
        _check(got, expect, r * B_l, (r + 1) * B_l, 1e-4)
    import rankops
    assert rankops.error_flags() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 8])
def test_shard_pack_and_gather_kernels(world):
    """rk_shard_pack_indices equals the torch stack/cat/cast permute; rk_shard_gather_rows equals
    the packed-table rows at the received indices for a chunk [b0, b0 + bc) of every source, and an
    out-of-range index gives a zero row and raises RK_FLAG_INDEX_OOB."""
    import rankops
    full = H.build("deepfm", CFG30, seed=42).cuda()
    shards, _ = _shards(full, world)
    sh = shards[0]
    B = 777
    g = torch.Generator().manual_seed(world)
    cat = {f: torch.randint(0, n, (B,), generator=g).cuda() for f, n in FIELDS30.items()}
    sh.wire = "packed"  # the packed-row gather here; the split one in test_split_wire_gather_rows
    got = sh.pack_indices(cat)
    want = torch.cat([torch.stack([cat[f] for f in fr], 1).reshape(-1) for fr in sh.fields_of if fr]).to(torch.int32)
    assert got.dtype == torch.int32 and torch.equal(got, want)
    F_me = len(sh.local_fields)
    recv = torch.stack([torch.randint(0, FIELDS30[f], (world, B), generator=g) for f in sh.local_fields], 2)
    recv[1, 5, 0] = sh.packed_table(sh.local_fields[0]).shape[0]  # one past the table's last row: OOB
    recv_d = recv.reshape(-1).to(torch.int32).cuda()
    rankops.error_flags(reset=True)
    RS = sharded.row_stride(32)
    for b0, bc in ((0, B), (100, 333), (776, 1)):
        rows = sh.gather_rows(recv_d, B, b0, bc).view(world, bc, F_me, RS).cpu()
        for j, f in enumerate(sh.local_fields):
            tab = sh.packed_table(f).cpu()
            idx = recv[:, b0:b0 + bc, j]
            ok = idx < tab.shape[0]
            exp = tab[idx.clamp(max=tab.shape[0] - 1)] * ok[..., None]
            assert torch.equal(rows[:, :, j, :], exp[:, :, :RS])
    assert rankops.error_flags(reset=True) & 1
    # ids outside [0, 2^31) go out as -1: never narrowed into a valid row
    bad = dict(cat)
    f0 = sh.fields[0]
    bad[f0] = cat[f0].clone()
    bad[f0][3] = 2 ** 32 + 5
    bad[f0][4] = -2 ** 32 + 1
    got = sh.pack_indices(bad).cpu()
    pos = [q for q, f in enumerate([f for fr in sh.fields_of for f in fr]) if f == f0][0]
    o = sh.owner[0]
    start = sum(len(sh.fields_of[r]) for r in range(o))
    j = sh.fields_of[o].index(f0)
    Fr = len(sh.fields_of[o])
    assert got[B * start + 3 * Fr + j] == -1 and got[B * start + 4 * Fr + j] == -1
    assert pos >= 0


def _pipe_run(shards, emu, batches, B_l, capture=False):
    """Each emulated rank drives ShardedDeepFM.pipeline over `batches` (per batch: the global
    category dict); returns per rank the list of per-batch outputs (CPU)."""
    world = len(shards)
    mines = [[{f: v[r * B_l:(r + 1) * B_l].contiguous() for f, v in cat.items()} for cat in batches]
             for r in range(world)]
    pipes = []
    if capture:  # capture is process-global: serially, here (no collective inside the graphs)
        with torch.no_grad():
            pipes = [shards[r].pipeline(B_l, capture=mines[r][:3]) for r in range(world)]

    def rank_fn(r):
        sh = shards[r]
        mine = mines[r]
        outs = []
        with torch.no_grad():
            if capture:
                pipe = pipes[r]
                for i in range(len(batches)):
                    o = pipe.step()
                    if o is not None:
                        torch.cuda.synchronize()
                        outs.append(tuple(x.cpu() for x in o))
                for o in pipe.flush():
                    torch.cuda.synchronize()
                    outs.append(tuple(x.cpu() for x in o))
            else:
                pipe = sh.pipeline(B_l)
                for cat in mine:
                    o = pipe.push(cat)
                    if o is not None:
                        outs.append(o)
                outs.extend(pipe.flush())
                if outs and outs[0][0].is_cuda:
                    torch.cuda.synchronize()
                outs = [tuple(x.cpu() for x in o) for o in outs]
        return outs

    return run_ranks(world, rank_fn, on_error=emu.abort)


@pytest.mark.parametrize("world,nbatch", [(2, 4), (8, 3)])
def test_emulator_cross_batch_pipeline_cpu(world, nbatch):
    """CPU: the cross-batch pipeline through the emulator under the CPU stand-in device steps."""
    from test_distributed import CFG, CpuStepsSharded
    full = H.build("deepfm", CFG, seed=42)
    B = 12
    batches = [H.make_inputs("deepfm", CFG, B * world, seed=300 + i)["category"] for i in range(nbatch)]
    shards, emu = _shards(full, world, cls=CpuStepsSharded)
    outs = _pipe_run(shards, emu, batches, B)
    for i, cat in enumerate(batches):
        expect = _oracle(full, CFG, cat)
        for r in range(world):
            _check(outs[r][i], expect, r * B, (r + 1) * B, 1e-5)
    assert emu.calls == 2 * nbatch  # one index and one row exchange per batch


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
def test_cross_batch_pipeline_emulated_on_gpu(world):
    """ShardedDeepFM.pipeline (eager) at P = 2 / 4 / 8 on one GPU: 5 batches through the three-stage
    pipeline (index exchange, gather + row exchange on the side stream, the one-launch forward on the
    compute stream), each against the oracle; ragged local batch."""
    full = H.build("deepfm", CFG30, seed=42).cuda()
    B_l = 520
    batches = [H.to_device(H.make_inputs("deepfm", CFG30, B_l * world, seed=7000 + 31 * i + world), "cuda")["category"]
               for i in range(5)]
    shards, emu = _shards(full, world)
    outs = _pipe_run(shards, emu, batches, B_l)
    for i, cat in enumerate(batches):
        expect = _oracle(full, CFG30, cat)
        for r in range(world):
            _check(outs[r][i], expect, r * B_l, (r + 1) * B_l, 1e-4)
    assert emu.calls == 2 * len(batches)
    import rankops
    assert rankops.error_flags() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 8])
def test_captured_cross_batch_pipeline_emulated_on_gpu(world):
    """bench.py's P > 1 step: the pipeline with pack / gather / forward captured per slot, 5 steps +
    flush over the three bound batches (slot i % 3), each batch's outputs against the oracle."""
    full = H.build("deepfm", CFG30, seed=42).cuda()
    B_l = 1000
    batches = [H.to_device(H.make_inputs("deepfm", CFG30, B_l * world, seed=8100 + i), "cuda")["category"]
               for i in range(3)]
    shards, emu = _shards(full, world)
    order = [batches[i % 3] for i in range(5)]
    outs = _pipe_run(shards, emu, order, B_l, capture=True)
    for i, cat in enumerate(order):
        expect = _oracle(full, CFG30, cat)
        for r in range(world):
            _check(outs[r][i], expect, r * B_l, (r + 1) * B_l, 1e-4)
    import rankops
    assert rankops.error_flags() == 0


@pytest.mark.gpu
def test_cross_batch_pipeline_full_local_batch_p8():
    """P = 8 at configs[4]'s local batch (8,192 samples: the forward's 32-row workgroups, one per CU)
    over 30 x 200k-row tables: pipelined outputs bit-equal to the unpipelined run_steps (chunks=1),
    and the first 300 samples of every rank against the oracle."""
    cfg = {"dim": 32, "fields": {f"field_{i:02d}": 200_000 + i for i in range(30)}, "hidden": [512, 256, 128]}
    full = H.build("deepfm", cfg, seed=42).cuda()
    world, B_l = 8, 8192
    batches = [H.to_device(H.make_inputs("deepfm", cfg, B_l * world, seed=9100 + i), "cuda")["category"]
               for i in range(2)]
    shards, emu = _shards(full, world)
    outs = _pipe_run(shards, emu, batches, B_l)

    def plain(r):
        with torch.no_grad():
            o = shards[r].run_steps({f: v[r * B_l:(r + 1) * B_l].contiguous() for f, v in batches[1].items()}, chunks=1)
        torch.cuda.synchronize()
        return tuple(x.cpu() for x in o)

    ref_outs = run_ranks(world, plain, on_error=emu.abort)
    for r in range(world):
        for a, b in zip(outs[r][1], ref_outs[r]):
            assert torch.equal(a, b)
    for i, cat in enumerate(batches):
        sub = {f: torch.cat([v[r * B_l:r * B_l + 300] for r in range(world)]) for f, v in cat.items()}
        expect = _oracle(full, cfg, sub)
        for r in range(world):
            got = tuple(x[:300] for x in outs[r][i])
            _check(got, expect, r * 300, (r + 1) * 300, 1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3, 8])
def test_split_wire_gather_rows(world):
    """rk_shard_gather_rows_split: per source block, the [bc][F_me][D] second-order rows straight from
    the nn.Embedding weights, then per sample the owner's first-order weights summed in field order;
    an out-of-range index gives a zero row, adds 0 and raises RK_FLAG_INDEX_OOB."""
    import rankops
    full = H.build("deepfm", CFG30, seed=42).cuda()
    shards, _ = _shards(full, world)
    sh = shards[0]
    assert sh.split_wire()
    B, D = 515, 32
    g = torch.Generator().manual_seed(world)
    F_me = len(sh.local_fields)
    recv = torch.stack([torch.randint(0, FIELDS30[f], (world, B), generator=g) for f in sh.local_fields], 2)
    recv[1, 5, 0] = full.second_order_embeddings[sh.local_fields[0]].num_embeddings  # one past the last row: OOB
    recv_d = recv.reshape(-1).to(torch.int32).cuda()
    rankops.error_flags(reset=True)
    for b0, bc in ((0, B), (100, 333), (514, 1)):
        out = sh.gather_rows(recv_d, B, b0, bc).cpu()
        blk = bc * F_me * D + (bc + 3) // 4 * 4
        assert out.numel() == world * blk
        for s_ in range(world):
            rows = out[s_ * blk:s_ * blk + bc * F_me * D].view(bc, F_me, D)
            part = out[s_ * blk + bc * F_me * D:s_ * blk + bc * F_me * D + bc]
            want_p = torch.zeros(bc)
            for j, f in enumerate(sh.local_fields):
                w2 = full.second_order_embeddings[f].weight.detach().cpu()
                w1 = full.first_order_embeddings[f].weight.detach().cpu()[:, 0]
                idx = recv[s_, b0:b0 + bc, j]
                ok = idx < w2.shape[0]
                cl = idx.clamp(max=w2.shape[0] - 1)
                assert torch.equal(rows[:, j, :], w2[cl] * ok[:, None])
                want_p = want_p + torch.where(ok, w1[cl], torch.zeros(()))
            torch.testing.assert_close(part, want_p, atol=1e-6, rtol=1e-6)
    assert rankops.error_flags(reset=True) & 1


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 8])
def test_split_and_packed_wire_agree(world):
    """The split wire format (default) and the packed one give the same forward (within fp32
    rounding: fm1 is summed per owner first), both against the oracle."""
    full = H.build("deepfm", CFG30, seed=42).cuda()
    B_l = 300
    inp = H.to_device(H.make_inputs("deepfm", CFG30, B_l * world, seed=77 + world), "cuda")
    expect = _oracle(full, CFG30, inp["category"])
    outs = {}
    for wire in ("split", "packed"):
        shards, emu = _shards(full, world)

        def rank_fn(r, shards=shards, wire=wire):
            sh = shards[r]
            sh.wire = wire
            assert sh.split_wire() == (wire == "split")
            mine = {f: v[r * B_l:(r + 1) * B_l].contiguous() for f, v in inp["category"].items()}
            with torch.no_grad():
                out = sh.run_steps(mine, chunks=1)
            torch.cuda.synchronize()
            return tuple(o.cpu() for o in out)

        outs[wire] = run_ranks(world, rank_fn, on_error=emu.abort)
    for r in range(world):
        _check(outs["split"][r], expect, r * B_l, (r + 1) * B_l, 1e-4)
        _check(outs["packed"][r], expect, r * B_l, (r + 1) * B_l, 1e-4)
        for a, b in zip(outs["split"][r], outs["packed"][r]):
            torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-5)


FIELDS15 = {f"field_{i:02d}": 200 + 11 * i for i in range(15)}
CFG15 = {"dim": 64, "fields": FIELDS15, "hidden": [512, 256, 128]}


@pytest.mark.parametrize("world", [8, 15, 16, 20])
def test_split_wire_splits_agree_across_ranks(world):
    """every rank's row all-to-all splits pair up (rank r's receive split from s equals
    s's send split to r), including owners with no fields when world > fields (15 fields at D = 64,
    the split format's shape), whose blocks are empty."""
    shards = [sharded.ShardedDeepFM(FIELDS15, 64, [512, 256, 128], rank=r, world_size=world) for r in range(world)]
    for B in (1, 7, 300):
        splits = [sh.row_splits(B) for sh in shards]
        for r in range(world):
            assert shards[r].split_wire()
            for s in range(world):
                assert splits[r][0][s] == splits[s][1][r], (world, B, r, s)
            if not shards[r].local_fields:
                assert sum(splits[r][1]) == 0


@pytest.mark.gpu
def test_split_wire_world_above_fields_on_gpu():
    """15 fields at D = 64 on 16 emulated ranks (one owns nothing): run_steps and the cross-batch
    pipeline with the split wire format against the oracle."""
    full = H.build("deepfm", CFG15, seed=42).cuda()
    world, B_l = 16, 40
    shards, emu = _shards(full, world)
    assert all(sh.split_wire() for sh in shards) and not shards[15].local_fields
    batches = [H.to_device(H.make_inputs("deepfm", CFG15, B_l * world, seed=5100 + i), "cuda")["category"]
               for i in range(3)]

    def rank_fn(r):
        mine = {f: v[r * B_l:(r + 1) * B_l].contiguous() for f, v in batches[0].items()}
        with torch.no_grad():
            out = shards[r].run_steps(mine, chunks=1)
        torch.cuda.synchronize()
        return tuple(o.cpu() for o in out)

    outs = run_ranks(world, rank_fn, on_error=emu.abort)
    expect = _oracle(full, CFG15, batches[0])
    for r in range(world):
        _check(outs[r], expect, r * B_l, (r + 1) * B_l, 1e-4)
    piped = _pipe_run(shards, emu, batches, B_l)
    for i, cat in enumerate(batches):
        expect = _oracle(full, CFG15, cat)
        for r in range(world):
            _check(piped[r][i], expect, r * B_l, (r + 1) * B_l, 1e-4)
