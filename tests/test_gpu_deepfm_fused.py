"""GPU parity of the one-launch DeepFM eval forward (rk_deepfm_forward, csrc/deepfm_fused.hip:
packed-table gather, FM sums, the three deep layers on one weight stream and the head per 16-row
tile; deepfm.py:121-151) — through rankops.DeepFM at configs[1]'s shape (30 fields x 32, hidden
[512, 256, 128]) against the CPU oracle and against the two-launch path (rk_fm_linear_packed +
rk_mlp_forward), and directly: out-of-range indices, dense blocks of packed rows (the ShardedDeepFM
receive layout), hipGraph replay, the shapes without a compiled plan, and the 32-row workgroups of
large batches (RT = 2, layer 0 in place) bit-identical to the 16-row ones.
Tolerance as every forward test: atol = rtol = 1e-4 (fp32)."""
import pytest
import torch

import helpers as H
import rankops
from rankops import deepfm as deepfm_mod
from rankops import ops

ATOL = RTOL = 1e-4
FIELDS30 = {f"field_{i:02d}": 1000 + 37 * i for i in range(30)}


def _launch_names(model):
    entry = next(iter(model.__dict__["_eager"]._d.values()))
    return [name for name, _ in entry[0]]


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 15, 17, 4096, 4100])
def test_deepfm_one_launch_against_oracle_and_two_launch(B, monkeypatch):
    cfg = {"dim": 32, "fields": FIELDS30}
    model = H.build("deepfm", cfg)
    H.randomize_eval_stats(model, 5)
    p = H.cpu_params(model)
    inp = H.make_inputs("deepfm", cfg, B)
    with torch.no_grad():
        ref = H.as_tuple(H.call_oracle("deepfm", cfg, p, inp))
    model = model.cuda().eval()
    d = H.to_device(inp, "cuda")
    rankops.error_flags(reset=True)
    with torch.no_grad():
        out = tuple(o.clone() for o in H.as_tuple(model(d["category"])))
    torch.cuda.synchronize()
    assert rankops.error_flags(reset=True) == 0
    assert _launch_names(model) == ["rk_deepfm_forward"]
    for i, (o, r) in enumerate(zip(out, ref)):
        torch.testing.assert_close(o.cpu(), r, atol=ATOL, rtol=RTOL, msg=lambda m: f"output {i}: {m}")
    monkeypatch.setattr(deepfm_mod, "FUSED_WHOLE", False)
    model.__dict__.pop("_eager")
    with torch.no_grad():
        two = H.as_tuple(model(d["category"]))
    assert _launch_names(model)[0] == "rk_fm_linear_packed" or B < 2048
    for o, q in zip(out, two):
        torch.testing.assert_close(o, q, atol=1e-5, rtol=1e-5)


@pytest.mark.gpu
def test_deepfm_one_launch_repeat_calls_and_graph_replay():
    """Cached eager launches with fresh outputs, and the forward captured in a hipGraph, replay to
    the same values bit for bit."""
    cfg = {"dim": 32, "fields": FIELDS30}
    model = H.build("deepfm", cfg).cuda().eval()
    d = H.to_device(H.make_inputs("deepfm", cfg, 1000, seed=3), "cuda")
    with torch.no_grad():
        a = tuple(o.clone() for o in model(d["category"]))
        b = tuple(o.clone() for o in model(d["category"]))
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            model(d["category"])
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            c = model(d["category"])
        g.replay()
    torch.cuda.synchronize()
    for x, y, z in zip(a, b, c):
        assert torch.equal(x, y) and torch.equal(x, z)


def _direct_case(M, seed=11, oob=False, vocab=3000):
    """Packed tables, indices, and the model pieces of a configs[1]-shaped DeepFM."""
    g = torch.Generator().manual_seed(seed)
    F, D = 30, 32
    tables = [torch.randn(vocab + 1, 36, generator=g).cuda() for _ in range(F)]
    idx = [torch.randint(0, vocab + 1, (M,), generator=g).cuda() for _ in range(F)]
    if oob:
        idx[7][M // 2] = vocab + 9
        idx[29][0] = -1
    widths, k = [512, 256, 128], F * D
    ws, keep, mls = [], [], []
    for n in widths:
        w = (torch.randn(n, k, generator=g) * (1.0 / k ** 0.5)).cuda()
        bias = (0.1 * torch.randn(n, generator=g)).cuda()
        sc = (1 + 0.1 * torch.randn(n, generator=g)).cuda()
        sh = (0.1 * torch.randn(n, generator=g)).cuda()
        pk = ops.pack_mlp_weight(w)
        mls.append(ops.make_mlp_layer(w, pk, bias=bias, pre_scale=sc, pre_shift=sh, act="relu"))
        ws.append((w, bias, sc, sh))
        keep += [pk, w, bias, sc, sh]
        k = n
    hw = (0.1 * torch.randn(1, 128, generator=g)).cuda()
    hb = torch.tensor([0.02]).cuda()
    fw = torch.tensor([[0.3, -0.2, 0.9]]).cuda()
    fb = torch.tensor([0.05]).cuda()
    return tables, idx, mls, ws, (hw, hb, fw, fb), keep


def _reference(tables, idx, ws, head):
    rows = []
    for t, i in zip(tables, idx):
        ok = (i >= 0) & (i < t.shape[0])
        r = t.double()[torch.where(ok, i, 0)]
        rows.append(torch.where(ok[:, None], r, torch.zeros_like(r)))
    emb = torch.stack([r[:, :32] for r in rows], 1)
    fm1 = torch.stack([r[:, 32] for r in rows], 1).sum(1, keepdim=True)
    s = emb.sum(1)
    fm2 = 0.5 * (s * s - (emb * emb).sum(1)).sum(1, keepdim=True)
    h = emb.reshape(emb.shape[0], -1)
    for w, b, sc, sh in ws:
        h = torch.relu((h @ w.double().T + b.double()) * sc.double() + sh.double())
    hw, hb, fw, fb = (x.double() for x in head)
    deep = h @ hw.T + hb
    total = torch.cat([fm1, fm2, deep], 1) @ fw.T + fb
    return torch.sigmoid(total), total, fm1, fm2, deep


def _run_direct(segs, M, mls, head):
    hw, hb, fw, fb = head
    outs = [torch.full((M, 1), float("nan"), device="cuda") for _ in range(5)]
    prob, total, fm1, fm2, deep = outs
    ep = ops.make_epilogue(head_w=hw, head_b=hb, final_w=fw, final_b=fb, head_logit=total, head_prob=prob,
                           head_aux=deep)
    ops.deepfm_forward(segs, 32, M, mls, ep, fm1, fm2)
    torch.cuda.synchronize()
    return outs


@pytest.mark.gpu
@pytest.mark.parametrize("oob", [False, True])
def test_deepfm_forward_direct(oob):
    """Out-of-range indices (past the table, negative) read a zero row and raise RK_FLAG_INDEX_OOB,
    as rk_fm_linear_packed; every output against a float64 restatement."""
    M = 777
    tables, idx, mls, ws, head, keep = _direct_case(M, oob=oob)
    segs = [ops.packed_segment(t, i, 32, f * 32) for f, (t, i) in enumerate(zip(tables, idx))]
    rankops.error_flags(reset=True)
    outs = _run_direct(segs, M, mls, head)
    assert bool(rankops.error_flags(reset=True) & 1) == oob
    for i, (o, r) in enumerate(zip(outs, _reference(tables, idx, ws, head))):
        torch.testing.assert_close(o, r.float(), atol=ATOL, rtol=RTOL, msg=lambda m: f"output {i}: {m}")


@pytest.mark.gpu
def test_deepfm_forward_dense_blocks_equal_indexed():
    """Fields without an index array read row b of a dense block of packed rows (what ShardedDeepFM
    receives); the result equals the indexed gather of the same rows bit for bit."""
    M = 300
    tables, idx, mls, ws, head, keep = _direct_case(M, seed=5)
    segs = [ops.packed_segment(t, i, 32, f * 32) for f, (t, i) in enumerate(zip(tables, idx))]
    a = _run_direct(segs, M, mls, head)
    blocks = [t[i].contiguous() for t, i in zip(tables, idx)]
    dsegs = []
    for f, blk in enumerate(blocks):
        s = ops.packed_segment(blk, idx[f], 32, f * 32)
        s.idx, s.idx_stride = None, 0
        dsegs.append(s)
    b = _run_direct(dsegs, M, mls, head)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.gpu
def test_deepfm_forward_rejects_shapes_without_a_plan():
    M = 64
    tables, idx, mls, ws, head, keep = _direct_case(M, seed=2)
    segs = [ops.packed_segment(t, i, 32, f * 32) for f, (t, i) in enumerate(zip(tables, idx))]
    with pytest.raises(rankops._lib.RankOpsError):  # 28 fields: K0 896, not the layer's 960
        _run_direct(segs[:28], M, mls, head)
    with pytest.raises(rankops._lib.RankOpsError):  # two deep layers
        _run_direct(segs, M, mls[:2], head)


@pytest.mark.gpu
def test_deepfm_prepare_equals_forward():
    """DeepFM.prepare: the bound one-launch forward recomputes from the inputs' current contents."""
    cfg = {"dim": 32, "fields": FIELDS30}
    model = H.build("deepfm", cfg).cuda().eval()
    d = H.to_device(H.make_inputs("deepfm", cfg, 2000, seed=4), "cuda")
    run = model.prepare(d["category"])
    with torch.no_grad():
        a = tuple(o.clone() for o in run())
        ref = model(d["category"])
    for x, y in zip(a, ref):
        assert torch.equal(x, y)
    e = H.to_device(H.make_inputs("deepfm", cfg, 2000, seed=5), "cuda")
    for k in d["category"]:
        d["category"][k].copy_(e["category"][k])
    with torch.no_grad():
        b = run()
        ref = model(e["category"])
    for x, y in zip(b, ref):
        assert torch.equal(x, y)


@pytest.mark.gpu
@pytest.mark.parametrize("M,oob,dense", [(1, False, False), (33, True, False), (1000, False, True),
                                         (8200, True, False), (16384, False, False)])
def test_deepfm_forward_32_row_tiles_bit_identical(M, oob, dense, monkeypatch):
    """RANKOPS_DEEPFM_ROW_TILES=2 (32 rows per workgroup: each weight float4 feeds both 16-row tiles,
    layer 0 written over its input in LDS) against =1: every output equal bit for bit, ragged last
    workgroups included (rows past the batch), with out-of-range indices and with dense blocks; and
    against the float64 restatement.  The default picks 2 once the batch gives every CU a 32-row
    workgroup (16384 here), 1 below."""
    tables, idx, mls, ws, head, keep = _direct_case(M, seed=13, oob=oob)
    if dense:
        segs, blocks = [], [t[i].contiguous() for t, i in zip(tables, idx)]  # (kept alive: segments hold raw pointers)
        for f, (blk, i) in enumerate(zip(blocks, idx)):
            s = ops.packed_segment(blk, i, 32, f * 32)
            s.idx, s.idx_stride = None, 0
            segs.append(s)
    else:
        segs = [ops.packed_segment(t, i, 32, f * 32) for f, (t, i) in enumerate(zip(tables, idx))]
    got = {}
    for rt in ("1", "2", None):
        if rt is None:
            monkeypatch.delenv("RANKOPS_DEEPFM_ROW_TILES", raising=False)
        else:
            monkeypatch.setenv("RANKOPS_DEEPFM_ROW_TILES", rt)
        rankops.error_flags(reset=True)
        got[rt] = _run_direct(segs, M, mls, head)
        assert bool(rankops.error_flags(reset=True) & 1) == oob
    for a, b, c in zip(got["1"], got["2"], got[None]):
        assert torch.equal(a, b) and torch.equal(a, c)
    for i, (o, r) in enumerate(zip(got["2"], _reference(tables, idx, ws, head))):
        torch.testing.assert_close(o, r.float(), atol=ATOL, rtol=RTOL, msg=lambda m: f"output {i}: {m}")


@pytest.mark.gpu
def test_prepared_run_survives_cache_rebuilds():
    """DeepFM.prepare()'s run() binds raw pointers to the packed FM tables and the folded
    BatchNorm affines.  A later .eval() (generation bump) plus a normal forward rebuilds both caches;
    run() must still read live images and reproduce its first outputs bit for bit."""
    cfg = {"dim": 32, "fields": FIELDS30}
    model = H.build("deepfm", cfg)
    H.randomize_eval_stats(model, 9)
    model = model.cuda().eval()
    d = H.to_device(H.make_inputs("deepfm", cfg, 700, seed=3), "cuda")
    run = model.prepare(d["category"])
    with torch.no_grad():
        first = tuple(o.clone() for o in run())
    model.eval()  # bumps the generation: the next forward repacks tables and refolds BatchNorm
    with torch.no_grad():
        model(d["category"])
        scratch = [torch.randn(1 << 20, device="cuda") for _ in range(64)]  # reuse freed blocks
        again = run()
    torch.cuda.synchronize()
    for a, b in zip(first, again):
        assert torch.equal(a, b)
    del scratch
