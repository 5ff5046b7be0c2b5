"""GPU: the prepared DIN forward (DIN.prepare -> rk_din_forward_plan / rk_din_plan_launch) equals
the eager forward bit for bit and follows new input contents like a captured graph; the packed
attention image path (rk_din_pack_attention) equals the in-kernel split and the oracle."""
import pytest
import torch

import helpers as H
from rankops import ops

ATOL = RTOL = 1e-4


def _cfg(**kw):
    cfg = {"T": 50, "dim": 32, "interaction_weights": "frozen"}
    cfg.update(kw)
    return cfg


@pytest.mark.gpu
def test_batches_in_flight_on_streams_equal_single_stream():
    """DinPlan.launch_on: several prepared forwards (own inputs, outputs and l2 workspaces) issued
    round-robin on their own HIP streams, as bench.py --din-streams N runs them, give each batch's
    single-stream outputs bit for bit (l2 included: each plan has its own hand-off counter)."""
    cfg = _cfg()
    model = H.build("din", cfg).cuda().eval()
    inps = [H.to_device(H.make_inputs("din", cfg, 1000, seed=500 + i), "cuda") for i in range(3)]
    with torch.no_grad():
        runs = [model.prepare(x["dense"], x["category"], x["sequence"], x["target"]) for x in inps]
        live = [r() for r in runs]  # the plan's own output tensors, rewritten by every launch
        ref = [tuple(x.clone() if isinstance(x, torch.Tensor) else x for x in o) for o in live]
        for o in live:  # poison them: the stream launches below must rewrite every element
            for x in o:
                if isinstance(x, torch.Tensor):
                    x.fill_(float("nan"))
        torch.cuda.synchronize()
        streams = [torch.cuda.Stream() for _ in runs]
        for st in streams:
            st.wait_stream(torch.cuda.current_stream())
        for k in range(12):
            i = k % len(runs)
            runs[i].plan.launch_on(streams[i].cuda_stream)
        for st in streams:
            torch.cuda.current_stream().wait_stream(st)
        torch.cuda.synchronize()
        for got, want in zip(live, ref):
            for g, w in zip(got, want):
                if isinstance(w, torch.Tensor):
                    assert torch.equal(g, w)


@pytest.mark.gpu
@pytest.mark.parametrize("softmax", [False, True])
def test_prepared_equals_eager_and_follows_inputs(softmax):
    cfg = _cfg(softmax=softmax)
    model = H.build("din", cfg).cuda().eval()
    inp = H.to_device(H.make_inputs("din", cfg, 300), "cuda")
    with torch.no_grad():
        eager = H.as_tuple(H.call_model(model, "din", inp))
        run = model.prepare(inp["dense"], inp["category"], inp["sequence"], inp["target"])
        out = run()
        torch.cuda.synchronize()
        for e, o in zip(eager, out):
            assert torch.equal(e, o)
        # new batch contents in the same input buffers: the plan recomputes from them
        new = H.to_device(H.make_inputs("din", cfg, 300, seed=4242), "cuda")
        inp["sequence"]["his_read_comment_7d_seq"].copy_(new["sequence"]["his_read_comment_7d_seq"])
        inp["sequence"]["his_read_comment_7d_seq_length"].copy_(new["sequence"]["his_read_comment_7d_seq_length"])
        inp["target"]["feedid"].copy_(new["target"]["feedid"])
        out2 = tuple(x.clone() if isinstance(x, torch.Tensor) else x for x in run())
        eager2 = H.as_tuple(H.call_model(model, "din", inp))
        torch.cuda.synchronize()
        for e, o in zip(eager2, out2):
            assert torch.equal(e, o)
        assert not torch.equal(out2[0], eager[0])


@pytest.mark.gpu
def test_prepared_matches_oracle_with_edge_lengths():
    cfg = _cfg()
    model = H.build("din", cfg)
    inp = H.make_inputs("din", cfg, 128)
    L = inp["sequence"]["his_read_comment_7d_seq_length"]
    L[:6] = torch.tensor([0, 1, 31, 32, 33, 50])
    p = H.cpu_params(model)
    model = model.cuda().eval()
    d = H.to_device(inp, "cuda")
    torch.manual_seed(5)  # the frozen H2 draw happens on the first forward, as the oracle's per-call draw
    with torch.no_grad():
        out = model.prepare(d["dense"], d["category"], d["sequence"], d["target"])()
        torch.manual_seed(5)
        ref = H.as_tuple(H.call_oracle("din", cfg, p, inp))
    for o, r in zip(out, ref):
        if isinstance(r, torch.Tensor):
            torch.testing.assert_close(o.cpu(), r, atol=ATOL, rtol=RTOL)


@pytest.mark.gpu
@pytest.mark.parametrize("H_", [8, 16, 32])
def test_attention_image_layout(H_):
    """rk_din_pack_attention writes WK = W1b - W1c, WQK = W1d, WQ = W1a + W1c (rows padded to H+4),
    W2 (rows padded to 68), b1, b2, w3 — the layout din_forward_kernel stages."""
    g = torch.Generator().manual_seed(H_)
    w1 = torch.randn(64, 4 * H_, generator=g)
    b1, w2, b2 = torch.randn(64, generator=g), torch.randn(32, 64, generator=g), torch.randn(32, generator=g)
    w3, b3 = torch.randn(1, 32, generator=g), torch.randn(1, generator=g)
    img = ops.din_pack_attention(tuple(t.cuda() for t in (w1, b1, w2, b2, w3, b3)), H_).cpu()
    L = H_ + 4
    wa, wb, wc, wd = w1[:, :H_], w1[:, H_:2 * H_], w1[:, 2 * H_:3 * H_], w1[:, 3 * H_:]
    blk = 64 * L
    for i, want in enumerate((wb - wc, wd, wa + wc)):
        got = img[i * blk:(i + 1) * blk].view(64, L)
        assert torch.equal(got[:, :H_], want) and not got[:, H_:].any()
    o = 3 * blk
    got = img[o:o + 32 * 68].view(32, 68)
    assert torch.equal(got[:, :64], w2) and not got[:, 64:].any()
    o += 32 * 68
    assert torch.equal(img[o:o + 64], b1) and torch.equal(img[o + 64:o + 96], b2)
    assert torch.equal(img[o + 96:o + 128], w3[0])


@pytest.mark.gpu
def test_l2_hand_off_stable_over_repeated_launches():
    """The l2 mean is finished by the last workgroup to publish its partial (an sc1 store + agent
    counter hand-off, din_fused.hip): back-to-back launches with no host sync between them must
    give the same l2 bit for bit, equal to the eager forward's, for 4096 rows (256 workgroups)."""
    cfg = _cfg()
    model = H.build("din", cfg).cuda().eval()
    inp = H.to_device(H.make_inputs("din", cfg, 4096), "cuda")
    with torch.no_grad():
        eager = H.as_tuple(H.call_model(model, "din", inp))
        run = model.prepare(inp["dense"], inp["category"], inp["sequence"], inp["target"])
        got = torch.empty(200, device="cuda")
        for i in range(200):
            out = run()
            got[i:i + 1].copy_(out[2].reshape(1))
        torch.cuda.synchronize()
    assert torch.equal(got, eager[2].reshape(1).expand(200))


@pytest.mark.gpu
@pytest.mark.parametrize("softmax", [False, True])
@pytest.mark.parametrize("batch,T", [(17, 50), (1000, 50), (1025, 50), (4096, 50), (5000, 50), (8192, 50), (3000, 160),
                                     (8192, 256), (10000, 50), (33 * 1024 + 5, 64)])
def test_balanced_assignment_matches_contiguous_blocks(monkeypatch, softmax, batch, T):
    """Batches of 17..33,797 rows rank the samples by attention tile count inside the kernel and
    deal them round-robin to the workgroups (din_fused.hip, balanced assignment: the default for
    T > 32, forced here with RANKOPS_DIN_BALANCE=1), per 1,024-sample universe (the default, round
    6) or over the whole batch (RANKOPS_DIN_UNI=0, batches up to 8,192; beyond, contiguous blocks);
    every output row must equal the contiguous-block launch (RANKOPS_DIN_BALANCE=0) bit for bit —
    zero, short and full-length histories mixed, all tile classes present, a partial last universe
    — and the l2 mean within fp32 rounding."""
    cfg = _cfg(softmax=softmax, T=T)
    model = H.build("din", cfg).cuda().eval()
    inp = H.make_inputs("din", cfg, batch, seed=batch)
    L = inp["sequence"]["his_read_comment_7d_seq_length"]
    L[: min(batch, 9)] = torch.tensor([0, 1, 31, 32, 33, T, 0, T + 14, -3])[: min(batch, 9)]
    d = H.to_device(inp, "cuda")
    outs = {}
    with torch.no_grad():
        for mode, bal, uni in (("universe", "1", "1"), ("whole", "1", "0"), ("contiguous", "0", "1")):
            monkeypatch.setenv("RANKOPS_DIN_BALANCE", bal)
            monkeypatch.setenv("RANKOPS_DIN_UNI", uni)
            outs[mode] = H.as_tuple(H.call_model(model, "din", d))
    torch.cuda.synchronize()
    ctg = outs["contiguous"]
    for mode in ("universe", "whole"):
        bal = outs[mode]
        assert torch.equal(bal[0], ctg[0]) and torch.equal(bal[1], ctg[1]), mode
        torch.testing.assert_close(bal[2], ctg[2], rtol=1e-6, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("dim", [8, 16, 32])
@pytest.mark.parametrize("softmax", [False, True])
@pytest.mark.parametrize("balance", ["0", "1"])
def test_pre_barrier_layer0_chunks_bit_identical(monkeypatch, dim, softmax, balance):
    """Phase B's first layer-0 K-chunks (the dense, category and query columns) accumulated by each
    wave before the barrier that closes phase A (din_fused.hip PreChunks; RANKOPS_DIN_PRE=0 turns
    them off): the same chunks in the same order into the same accumulators, so every output is
    bit-identical to the launch without them — contiguous and balanced launches (the balanced one
    waits on the rows-ready count), zero / short / full histories, a partial last workgroup."""
    cfg = _cfg(softmax=softmax, dim=dim)
    model = H.build("din", cfg).cuda().eval()
    batch = 4096 + 37
    inp = H.make_inputs("din", cfg, batch, seed=77 + dim)
    L = inp["sequence"]["his_read_comment_7d_seq_length"]
    L[:6] = torch.tensor([0, 1, 16, 17, 50, 0])
    d = H.to_device(inp, "cuda")
    monkeypatch.setenv("RANKOPS_DIN_BALANCE", balance)
    with torch.no_grad():
        monkeypatch.setenv("RANKOPS_DIN_PRE", "1")
        pre = H.as_tuple(H.call_model(model, "din", d))
        monkeypatch.setenv("RANKOPS_DIN_PRE", "0")
        ref = H.as_tuple(H.call_model(model, "din", d))
    torch.cuda.synchronize()
    assert torch.equal(pre[0], ref[0]) and torch.equal(pre[1], ref[1])
    torch.testing.assert_close(pre[2], ref[2], rtol=1e-6, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("dim", [16, 32])
@pytest.mark.parametrize("batch", [4096, 4133])
@pytest.mark.parametrize("balance", ["0", "1"])
def test_plan_epilogue_image_by_lds_dma_bit_identical(monkeypatch, dim, batch, balance):
    """A prepared plan binds phase B's epilogue parameters packed once (rk_mlp_pack_epilogue,
    rk_din_plan_set_epilogue_image); balanced launches copy them into LDS by LDS-DMA after phase A
    instead of resolving each column at launch (balanced and contiguous launches).  Same values, same
    arithmetic: the plan's outputs
    equal the plan without the image (RANKOPS_DIN_EPI_DMA=0) and the eager forward bit for bit,
    and match the oracle."""
    cfg = _cfg(dim=dim, T=50)
    model = H.build("din", cfg)
    p = H.cpu_params(model)
    model = model.cuda().eval()
    inp = H.make_inputs("din", cfg, batch, seed=5 + batch)
    d = H.to_device(inp, "cuda")
    monkeypatch.setenv("RANKOPS_DIN_BALANCE", balance)
    args = (d["dense"], d["category"], d["sequence"], d["target"])
    torch.manual_seed(5)  # the frozen H2 draw happens on the first forward, as the oracle's per-call draw
    with torch.no_grad():
        monkeypatch.setenv("RANKOPS_DIN_EPI_DMA", "1")
        run = model.prepare(*args)
        assert run.plan._epi is not None  # the image is bound
        dma_all = [t.clone() for t in H.as_tuple(run())]
        dma = dma_all[:2]
        monkeypatch.setenv("RANKOPS_DIN_EPI_DMA", "0")
        run0 = model.prepare(*args)
        assert run0.plan._epi is None
        res = [t.clone() for t in H.as_tuple(run0())[:2]]
        model.__dict__.pop("_eager", None)
        eager = [t.clone() for t in H.as_tuple(H.call_model(model, "din", d))[:2]]  # rk_din_forward_ex, no image
        monkeypatch.setenv("RANKOPS_DIN_EPI_DMA", "1")
        model.__dict__.pop("_eager", None)
        eager_dma = H.as_tuple(H.call_model(model, "din", d))  # the cached eager entry packs its image
        entry = next(iter(model._eager._d.values()))
        assert entry[-1][-1] is not None
    torch.cuda.synchronize()
    for a, b, c, e in zip(dma, res, eager, eager_dma):
        assert torch.equal(a, b) and torch.equal(a, c) and torch.equal(a, e)
    torch.manual_seed(5)
    with torch.no_grad():
        ref = H.as_tuple(H.call_oracle("din", cfg, p, inp))
    # prob, logit and the l2 term of the prepared LDS-DMA launch against the oracle
    assert len(dma_all) == len(ref) == 3
    for i, (g, r) in enumerate(zip(dma_all, ref)):
        torch.testing.assert_close(g.cpu().reshape(r.shape), r, atol=ATOL, rtol=RTOL, msg=lambda m: f"output {i}: {m}")


@pytest.mark.gpu
def test_unsupported_fused_shape_falls_back_to_unfused(monkeypatch):
    """When rk_din_forward refuses a configuration (RK_ERR_UNSUPPORTED, e.g. an LDS carve past 160
    KiB), the forward takes the unfused launches for that shape from then on: simulated
    by refusing every fused launch; the outputs still match the oracle."""
    import rankops
    from rankops import common
    cfg = _cfg(T=80)
    model = H.build("din", cfg)
    inp = H.make_inputs("din", cfg, 300)
    p = H.cpu_params(model)
    model = model.cuda().eval()
    d = H.to_device(inp, "cuda")

    def refuse(*a, **k):
        err = rankops._lib.RankOpsError("rk_din_forward failed (code 4): simulated")
        err.code = rankops._lib.RK_ERR_UNSUPPORTED
        raise err
    monkeypatch.setattr(ops, "din_forward", refuse)
    monkeypatch.setattr(common, "EAGER_CACHE", False)
    torch.manual_seed(5)
    with torch.no_grad():
        out = H.as_tuple(model(d["dense"], d["category"], d["sequence"], d["target"]))
        assert model.__dict__.get("_unfusable")  # the shape is marked: no second fused attempt
        again = H.as_tuple(model(d["dense"], d["category"], d["sequence"], d["target"]))
        torch.manual_seed(5)
        ref = H.as_tuple(H.call_oracle("din", cfg, p, inp))
    for o, a, r in zip(out, again, ref):
        if isinstance(r, torch.Tensor):
            torch.testing.assert_close(o.cpu(), r, atol=ATOL, rtol=RTOL)
            assert torch.equal(o, a)
