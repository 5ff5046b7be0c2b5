"""GPU parity: every rankops model (HIP path, through the C ABI) against the CPU oracle on
the same seeded inputs and weights.  Tolerance (north star): logits and probabilities within
atol 1e-4 + rtol 1e-4 in fp32; indices are used bit-exactly (same rows gathered)."""
import pytest
import torch

import helpers as H
import rankops

ATOL = 1e-4
RTOL = 1e-4

FIELDS30 = {f"field_{i:02d}": 1000 + 37 * i for i in range(30)}

CASES = [
    ("dcn", {}),
    ("dcn", {"cross": 3}),
    ("dcn", {"cross": 0}),
    ("dcn", {"hidden": [64, 300]}),  # last hidden width > 256: head runs as its own GEMM
    ("deepfm", {}),
    ("deepfm", {"dim": 32, "fields": FIELDS30}),
    ("deepfm", {"batch_norm": False}),
    ("din", {"T": 50}),
    ("din", {"T": 50, "softmax": True}),
    ("din", {"T": 50, "dim": 32}),
    ("din", {"T": 50, "dim": 32, "softmax": True}),
    ("din", {"T": 7, "activation": "prelu", "batch_norm": False, "l2": 0.0}),
    ("din", {"T": 77}),  # more than two 32-position tiles
    ("afm", {}),
    ("afm", {"dim": 32, "att": 64}),
    ("afm", {"dim": 16, "att": 200}),  # > 128 units: the VALU kernel (as dim 32)
    ("afm", {"dim": 4, "att": 100}),    # the MFMA kernel with a partial unit tile
    ("afm", {"dim": 16, "att": 128}),
    ("deepcrossing", {}),
    ("deepcrossing", {"units": 3, "internal": 64}),
    ("bst", {"T": 50}),
    ("bst", {"T": 50, "pooling": "mean"}),
    ("bst", {"T": 64, "dim": 128, "max_len": 64, "heads": 4}),
    ("bst", {"T": 20, "blocks": 2, "batch_norm": False}),
    ("bst", {"T": 1}),
    ("bst", {"T": 20, "blocks": 0}),  # no transformer block: pooling straight over the history rows
    ("bst", {"T": 33, "blocks": 0, "pooling": "mean"}),
    # rk_bst_forward_blocks envelope (d_model 128, 4 heads, T <= 64)
    ("bst", {"T": 50, "dim": 128, "pooling": "mean"}),
    ("bst", {"T": 37, "dim": 128, "blocks": 2, "max_len": 40}),
    ("bst", {"T": 64, "dim": 128, "blocks": 3, "max_len": 64}),
    ("bst", {"T": 1, "dim": 128}),
]


def _ids(case):
    name, cfg = case
    return name + ("-" + "-".join(f"{k}{v}" for k, v in cfg.items() if k != "fields") if cfg else "")


def _compare(out, ref, what):
    out, ref = H.as_tuple(out), H.as_tuple(ref)
    assert len(out) == len(ref), what
    for i, (o, r) in enumerate(zip(out, ref)):
        if not isinstance(r, torch.Tensor):
            assert o == r, f"{what}[{i}]"
            continue
        assert o.device.type == "cuda", f"{what}[{i}] not produced on the GPU"
        assert tuple(o.shape) == tuple(r.shape), f"{what}[{i}] shape {tuple(o.shape)} vs {tuple(r.shape)}"
        torch.testing.assert_close(o.detach().cpu(), r, atol=ATOL, rtol=RTOL, equal_nan=True,
                                   msg=lambda m: f"{what}[{i}]: {m}")


def run_pair(name, cfg, B, seed=123, inputs=None, model=None):
    model = model if model is not None else H.build(name, cfg)
    p = H.cpu_params(model)
    inp = inputs if inputs is not None else H.make_inputs(name, cfg, B)
    torch.manual_seed(seed)
    with torch.no_grad():
        ref = H.call_oracle(name, cfg, p, inp)
    model = model.cuda()
    torch.manual_seed(seed)
    with torch.no_grad():
        out = H.call_model(model, name, H.to_device(inp, "cuda"))
    torch.cuda.synchronize()
    return out, ref


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=_ids)
def test_model_parity(case):
    name, cfg = case
    out, ref = run_pair(name, cfg, B=300)
    _compare(out, ref, _ids(case))
    assert rankops.error_flags() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["dcn", "deepcrossing", "din"])
def test_frozen_interaction_weights(name):
    """'frozen' draws the H2 weights once with the reference's calls; the first forward equals
    the reference's first call and later forwards reuse the same weights."""
    cfg = {"interaction_weights": "frozen", "T": 20}
    model = H.build(name, cfg).cuda()
    inp = H.to_device(H.make_inputs(name, cfg, 128), "cuda")
    torch.manual_seed(5)
    with torch.no_grad():
        a = H.call_model(model, name, inp)
        torch.manual_seed(99)
        b = H.call_model(model, name, inp)
    for x, y in zip(H.as_tuple(a), H.as_tuple(b)):
        assert torch.equal(x, y)
    p = H.cpu_params(model)
    torch.manual_seed(5)
    ref = H.call_oracle(name, cfg, p, H.to_device(inp, "cpu"))
    _compare(a, ref, f"{name}-frozen")


@pytest.mark.gpu
def test_wechat_scale_tables():
    """Full wechat vocabulary sizes at batch 4096: DCN and DIN."""
    for name, cfg in (("dcn", {"vocab": H.WECHAT_VOCAB}), ("din", {"vocab": H.WECHAT_VOCAB, "T": 50, "dim": 32})):
        out, ref = run_pair(name, cfg, B=4096)
        _compare(out, ref, name + "-wechat")


@pytest.mark.gpu
@pytest.mark.parametrize("softmax", [False, True])
def test_din_edge_lengths(softmax):
    """Length 0 (softmax -> uniform weights over T, din.py:74-77; plain -> zeros), T=1, len=T."""
    cfg = {"T": 9, "softmax": softmax}
    inp = H.make_inputs("din", cfg, 64)
    lens = inp["sequence"]["his_read_comment_7d_seq_length"]
    lens[:8] = 0
    lens[8:16] = 9
    lens[16:24] = 1
    out, ref = run_pair("din", cfg, B=64, inputs=inp)
    _compare(out, ref, f"din-edge-softmax{softmax}")
    cfg1 = {"T": 1, "softmax": softmax}
    out, ref = run_pair("din", cfg1, B=32)
    _compare(out, ref, "din-T1")


@pytest.mark.gpu
def test_bst_empty_sequence_is_nan_like_reference():
    """A length-0 row is all -inf in the reference softmax -> NaN output (bst.py:80-82)."""
    cfg = {"T": 12}
    inp = H.make_inputs("bst", cfg, 32)
    inp["seq_length"][:4] = 0
    out, ref = run_pair("bst", cfg, B=32, inputs=inp)
    assert torch.isnan(ref[1][:4]).all()
    _compare(out, ref, "bst-empty")


@pytest.mark.gpu
def test_out_of_range_index_is_flagged():
    cfg = {}
    model = H.build("dcn", {"interaction_weights": "frozen"}).cuda()
    inp = H.to_device(H.make_inputs("dcn", cfg, 64), "cuda")
    rankops.error_flags(reset=True)
    with torch.no_grad():
        H.call_model(model, "dcn", inp)
    assert rankops.error_flags() == 0
    inp["category"]["userid"][3] = model.vocab_sizes["userid"] + 5
    with torch.no_grad():
        H.call_model(model, "dcn", inp)
    assert rankops.error_flags(reset=True) & 1
    assert rankops.error_flags() == 0


@pytest.mark.gpu
def test_graph_capture_replay_matches_eager():
    """The forward has no host sync or allocation outside the caching allocator, so it captures
    into a hipGraph; replay must equal the eager result."""
    for name, cfg in (("deepfm", {"dim": 32, "fields": FIELDS30}), ("din", {"T": 50, "dim": 32,
                      "interaction_weights": "frozen"}), ("bst", {"T": 64, "dim": 128, "max_len": 64})):
        model = H.build(name, cfg).cuda()
        inp = H.to_device(H.make_inputs(name, cfg, 512), "cuda")
        with torch.no_grad():
            eager = H.as_tuple(H.call_model(model, name, inp))
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    H.call_model(model, name, inp)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                static = H.as_tuple(H.call_model(model, name, inp))
            g.replay()
            torch.cuda.synchronize()
        for e, r in zip(eager, static):
            if isinstance(e, torch.Tensor):
                assert torch.equal(e, r), name


@pytest.mark.gpu
def test_cpu_inputs_raise():
    model = H.build("dcn", {}).cuda()
    inp = H.make_inputs("dcn", {}, 8)
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        H.call_model(model, "dcn", inp)


@pytest.mark.gpu
def test_training_mode_raises():
    """A train-mode forward without autograd (no backward to attach) is refused instead of
    silently running eval semantics; with autograd every model trains (tests/test_gpu_train.py)."""
    model = H.build("bst", {"T": 20}).cuda().train()
    inp = H.to_device(H.make_inputs("bst", {"T": 20}, 8), "cuda")
    with torch.no_grad(), pytest.raises(NotImplementedError):
        H.call_model(model, "bst", inp)


@pytest.mark.gpu
def test_standalone_reference_functions():
    """cross_layer, residual_unit and din_attention_gather (din_attention with the history as
    table + index) as module-level functions (dcn.py:25, deepcrossing.py:25, din.py:42) draw per
    call like the reference."""
    from oracle import reference_forward as ref
    g = torch.Generator().manual_seed(3)
    x0 = torch.randn(40, 50, generator=g)
    xl = torch.randn(40, 50, generator=g)
    torch.manual_seed(11)
    w, b = ref.draw_cross(50, 1)[0]
    expect = ref.dcn_cross_layer(x0, xl, w, b)
    torch.manual_seed(11)
    got = rankops.cross_layer(x0.cuda(), xl.cuda(), 0)
    torch.testing.assert_close(got.cpu(), expect, atol=ATOL, rtol=RTOL)

    torch.manual_seed(12)
    expect = ref.residual_unit(x0, *ref.draw_residual(50, 32))
    torch.manual_seed(12)
    got = rankops.residual_unit(x0.cuda(), 32, 0)
    torch.testing.assert_close(got.cpu(), expect, atol=ATOL, rtol=RTOL)

    table = torch.randn(90, 16, generator=g)
    seq = torch.randint(0, 90, (40, 13), generator=g)
    lens = torch.randint(0, 14, (40,), generator=g)
    q = torch.randn(40, 16, generator=g)
    for sm in (False, True):
        torch.manual_seed(13)
        expect = ref.din_attention(q, table[seq], lens, sm)
        torch.manual_seed(13)
        got = rankops.din_attention_gather(q.cuda(), table.cuda(), seq.cuda(), lens.cuda(), sm)
        torch.testing.assert_close(got.cpu(), expect, atol=ATOL, rtol=RTOL)


@pytest.mark.gpu
@pytest.mark.parametrize("case", [("dcn", {}), ("deepfm", {"dim": 32, "fields": FIELDS30}), ("din", {"T": 20}),
                                  ("bst", {"T": 20}), ("deepcrossing", {"units": 2})], ids=_ids)
def test_unfused_tail_path(case, monkeypatch):
    """The per-layer rk_linear path (used when a tail does not fit rk_mlp_forward) stays exact."""
    monkeypatch.setattr(rankops.common, "FUSED_MLP", False)
    name, cfg = case
    out, ref = run_pair(name, cfg, B=200)
    _compare(out, ref, "unfused-" + _ids(case))


@pytest.mark.gpu
@pytest.mark.parametrize("case", [("din", {"T": 50, "dim": 32}), ("din", {"T": 50, "dim": 32, "softmax": True}),
                                  ("din", {"T": 9, "activation": "prelu"})], ids=_ids)
def test_din_split_path_vs_reference_formulation(case, monkeypatch):
    """rk_din_forward (algebraically split att-MLP layer 1) and the reference-formulation
    rk_din_attention + rk_mlp_forward path agree with the oracle and with each other."""
    name, cfg = case
    fused, ref = run_pair(name, cfg, B=257)
    _compare(fused, ref, "fused-" + _ids(case))
    monkeypatch.setattr(rankops.common, "FUSED_DIN", False)
    plain, ref2 = run_pair(name, cfg, B=257)
    _compare(plain, ref2, "plain-" + _ids(case))
    for a, b in zip(H.as_tuple(fused), H.as_tuple(plain)):
        if isinstance(a, torch.Tensor):
            torch.testing.assert_close(a, b, atol=ATOL, rtol=RTOL)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [{"T": 64, "dim": 128, "max_len": 64}, {"T": 29, "dim": 128, "blocks": 2},
                                 {"T": 50, "dim": 128, "pooling": "mean"}], ids=str)
def test_bst_fused_blocks_vs_per_layer_path(cfg, monkeypatch):
    """rk_bst_forward_blocks (whole block in LDS) and the per-layer rk_linear/rk_bst_attention
    path agree with the oracle and with each other; length-0 rows stay NaN in both."""
    inp = H.make_inputs("bst", cfg, 300)
    inp["seq_length"][:3] = 0
    inp["seq_length"][3:6] = cfg["T"]
    inp["seq_length"][6:9] = 1
    model = H.build("bst", cfg)
    fused, ref = run_pair("bst", cfg, B=300, inputs=inp, model=model)
    assert model._fused_blocks(cfg["T"]) is not None
    _compare(fused, ref, "fused-bst")
    assert torch.isnan(fused[1][:3].cpu()).all()
    monkeypatch.setattr(rankops.common, "FUSED_BST", False)
    plain, _ = run_pair("bst", cfg, B=300, inputs=inp, model=model)
    for a, b in zip(fused, plain):
        torch.testing.assert_close(a, b, atol=ATOL, rtol=RTOL, equal_nan=True)
    assert rankops.error_flags() == 0


@pytest.mark.gpu
def test_bst_fused_blocks_oob_sequence_index_is_flagged():
    cfg = {"T": 16, "dim": 128}
    model = H.build("bst", cfg).cuda()
    inp = H.to_device(H.make_inputs("bst", cfg, 32), "cuda")
    rankops.error_flags(reset=True)
    inp["seq_feedid"][5, 2] = model.vocab_sizes["feedid"] + 3
    with torch.no_grad():
        H.call_model(model, "bst", inp)
    assert rankops.error_flags(reset=True) & 1


@pytest.mark.gpu
@pytest.mark.parametrize("tiled", [True, False])
def test_deepfm_wide_first_layer_tiled(tiled, monkeypatch):
    """DeepFM configs[1] shape (30 fields x 32: a 960-wide first layer) at batch >= 2048 runs its
    first layer tiled (the fused rk_fm_linear_packed front end) or in the fused tail; both match
    the oracle."""
    monkeypatch.setattr(rankops.common, "TILED_FIRST_MIN_K", 512 if tiled else 0)
    if tiled:  # 33 x 4 tiles at batch 2100: let them count as filling the GPU
        monkeypatch.setattr(rankops.common, "_num_cus", lambda device: 64)
    cfg = {"dim": 32, "fields": FIELDS30}
    out, ref = run_pair("deepfm", cfg, B=2100)
    _compare(out, ref, f"deepfm-wide-tiled{tiled}")


@pytest.mark.gpu
def test_linear_tiled_direct():
    """rk_linear_tiled against torch fp32 on ragged shapes (M not a multiple of 64, n not a
    multiple of 128, K not a multiple of 256), with BatchNorm affine + LeakyReLU."""
    g = torch.Generator().manual_seed(4)
    for M, K, n in ((333, 960, 512), (64, 70, 50), (1000, 300, 200)):
        x = torch.randn(M, K, generator=g).cuda()
        w = (0.05 * torch.randn(n, K, generator=g)).cuda()
        b = torch.randn(n, generator=g).cuda()
        sc = (1 + 0.1 * torch.randn(n, generator=g)).cuda()
        sh = (0.1 * torch.randn(n, generator=g)).cuda()
        packed = rankops.ops.pack_mlp_weight(w)
        layer = rankops.ops.make_mlp_layer(w, packed, bias=b, pre_scale=sc, pre_shift=sh, act="leaky", slope=0.01)
        y = torch.empty(M, n, device="cuda")
        rankops.ops.linear_tiled(x, layer, y)
        z = (x.double() @ w.double().T + b.double()) * sc.double() + sh.double()
        ref = torch.where(z > 0, z, 0.01 * z).float()
        torch.testing.assert_close(y, ref, atol=1e-4, rtol=1e-4)


@pytest.mark.gpu
def test_afm_prepare_equals_forward():
    """AFM.prepare: the bound one-launch forward equals the module's forward bit for bit and
    recomputes from the inputs' current contents."""
    cfg = {"vocab": H.WECHAT_VOCAB, "dim": 8, "att": 128}
    model = H.build("afm", cfg).cuda().eval()
    d = H.to_device(H.make_inputs("afm", cfg, 3000, seed=21), "cuda")
    run = model.prepare(d["dense_input"], d["category_input"])
    with torch.no_grad():
        a = tuple(o.clone() for o in run())
        ref = H.as_tuple(H.call_model(model, "afm", d))
    for x, y in zip(a, ref):
        assert torch.equal(x, y)
    e = H.to_device(H.make_inputs("afm", cfg, 3000, seed=22), "cuda")
    d["dense_input"].copy_(e["dense_input"])
    for k in d["category_input"]:
        d["category_input"][k].copy_(e["category_input"][k])
    with torch.no_grad():
        b = run()
        ref = H.as_tuple(H.call_model(model, "afm", e))
    for x, y in zip(b, ref):
        assert torch.equal(x, y)


@pytest.mark.gpu
def test_deepcrossing_prepare_equals_forward():
    """DeepCrossingModel.prepare: the bound gather + residual-MLP launches equal the module's forward
    bit for bit and recompute from the inputs' current contents."""
    cfg = {"vocab": H.WECHAT_VOCAB, "internal": 128, "units": 1, "interaction_weights": "frozen"}
    model = H.build("deepcrossing", cfg).cuda().eval()
    d = H.to_device(H.make_inputs("deepcrossing", cfg, 3000, seed=23), "cuda")
    run = model.prepare(d["dense"], d["category"])
    with torch.no_grad():
        a = tuple(o.clone() for o in run())
        ref = H.as_tuple(H.call_model(model, "deepcrossing", d))
    for x, y in zip(a, ref):
        assert torch.equal(x, y)
    e = H.to_device(H.make_inputs("deepcrossing", cfg, 3000, seed=24), "cuda")
    d["dense"].copy_(e["dense"])
    for k in d["category"]:
        d["category"][k].copy_(e["category"][k])
    with torch.no_grad():
        b = run()
        ref = H.as_tuple(H.call_model(model, "deepcrossing", e))
    for x, y in zip(b, ref):
        assert torch.equal(x, y)


@pytest.mark.gpu
def test_deepcrossing_fused_gather_equals_two_launches(monkeypatch):
    """rk_mlp_forward_gather (the row gather inside the residual MLP's launch) against
    rk_concat_gather + rk_mlp_forward: bit-identical outputs (same staged values, same tail), and an
    out-of-range index reads a zero row and raises RK_FLAG_INDEX_OOB in both."""
    cfg = {"vocab": H.WECHAT_VOCAB, "internal": 64, "units": 2, "interaction_weights": "frozen"}
    model = H.build("deepcrossing", cfg).cuda().eval()
    d = H.to_device(H.make_inputs("deepcrossing", cfg, 1037, seed=25), "cuda")
    name = next(iter(d["category"]))
    d["category"][name][7] = model.embeddings[name].num_embeddings  # one past the table
    outs = {}
    for fused in (True, False):
        monkeypatch.setattr(rankops.common, "FUSED_GATHER_MLP", fused)
        rankops.error_flags(reset=True)
        with torch.no_grad():
            outs[fused] = tuple(o.clone() for o in H.as_tuple(H.call_model(model, "deepcrossing", d)))
        assert rankops.error_flags(reset=True) & 1
    for a, b in zip(outs[True], outs[False]):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("internal,units,B", [(128, 1, 4097), (64, 2, 1037), (100, 1, 33), (128, 2, 16)])
def test_deepcrossing_register_kernel_equals_ring_kernel(internal, units, B, monkeypatch):
    """dc_forward_kernel (round 6: every weight fragment in registers from entry) against
    mlp_gather_kernel (RANKOPS_DC_KERNEL=0: the streamed ring) on the same inputs: bit-identical
    (same MFMA order, epilogue and head), out-of-range index flagged in both, and the oracle."""
    cfg = {"vocab": H.WECHAT_VOCAB, "internal": internal, "units": units, "interaction_weights": "frozen"}
    model = H.build("deepcrossing", cfg)
    p = H.cpu_params(model)
    inp = H.make_inputs("deepcrossing", cfg, B, seed=41)
    name = next(iter(inp["category"]))
    inp["category"][name][B // 2] = model.embeddings[name].num_embeddings  # one past the table
    model = model.cuda().eval()
    d = H.to_device(inp, "cuda")
    torch.manual_seed(0)
    outs = {}
    for k in ("1", "0"):
        monkeypatch.setenv("RANKOPS_DC_KERNEL", k)
        rankops.error_flags(reset=True)
        with torch.no_grad():
            outs[k] = tuple(o.clone() for o in H.as_tuple(H.call_model(model, "deepcrossing", d)))
        torch.cuda.synchronize()
        assert rankops.error_flags(reset=True) & 1
    for a, b in zip(outs["1"], outs["0"]):
        assert torch.equal(a, b)
    emb = p[f"embeddings.{name}.weight"]
    p[f"embeddings.{name}.weight"] = torch.cat([emb, torch.zeros(1, emb.shape[1])], 0)
    torch.manual_seed(0)  # the oracle draws the residual units as the frozen model did at its first forward
    with torch.no_grad():
        ref = H.as_tuple(H.call_oracle("deepcrossing", cfg, p, inp))
    for o, r in zip(outs["1"], ref):
        torch.testing.assert_close(o.cpu(), r, atol=1e-4, rtol=1e-4)


@pytest.mark.gpu
def test_fwfm_prepare_equals_forward():
    """FwFM.prepare: the bound launch equals the module's forward bit for bit, and recomputes from
    the indices' current contents."""
    cfg = {"vocab": H.WECHAT_VOCAB, "dim": 8}
    model = H.build("fwfm", cfg).cuda().eval()
    d = H.to_device(H.make_inputs("fwfm", cfg, 3000, seed=26), "cuda")
    run = model.prepare(d["x"])
    with torch.no_grad():
        prob, logit = (o.clone() for o in run())
        ref_p, ref_l = model(d["x"], return_logit=True)
    assert torch.equal(prob, ref_p) and torch.equal(logit, ref_l)
    e = H.to_device(H.make_inputs("fwfm", cfg, 3000, seed=27), "cuda")
    for k in d["x"]:
        d["x"][k].copy_(e["x"][k])
    with torch.no_grad():
        prob, logit = run()
        ref_p, ref_l = model(e["x"], return_logit=True)
    assert torch.equal(prob, ref_p) and torch.equal(logit, ref_l)
