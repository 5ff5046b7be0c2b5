"""GPU: the streamed fused-MLP tail (csrc/mlp_stream.h, round 4) against the generic mlp_rows path
(RANKOPS_MLP_STREAM=0) — bit for bit, since the accumulation order and the epilogue arithmetic are
the same — and against a float64 restatement of the layer stack.

Covered: every compiled plan (K0 chunks 4/8/12/16 over [512, 256, 128], and [256, 128] over K0 512),
every activation (none, ReLU, LeakyReLU, PReLU with one or per-channel alpha, Dice), with and without
bias and pre-/post-BatchNorm affines, ragged batches (1, 15, 17, 1000), 32-row workgroups
(RANKOPS_MLP_ROWS, the default at large batches) bit-identical to 16-row ones, and the model forwards that
run it: DCN (dcn_fused_kernel), DIN (phase B of din_forward_kernel, contiguous and balanced
assignment, softmax and PReLU variants), DeepFM (tail after the tiled first layer), BST (DNN tail).
Reference rows: dcn.py:144-152,175-180; din.py:272-285,312-316; deepfm.py:100-112,143-151;
bst.py:203-214,245-247."""
import os

import pytest
import torch

import helpers as H
from rankops import ops
from rankops._lib import Epilogue  # noqa: F401

ATOL = RTOL = 1e-4


class _stream_env:
    """Sets RANKOPS_MLP_STREAM (read by the C library at every launch / plan preparation)."""

    def __init__(self, on: bool):
        self.on = on

    def __enter__(self):
        self.old = os.environ.get("RANKOPS_MLP_STREAM")
        os.environ["RANKOPS_MLP_STREAM"] = "1" if self.on else "0"

    def __exit__(self, *a):
        if self.old is None:
            os.environ.pop("RANKOPS_MLP_STREAM", None)
        else:
            os.environ["RANKOPS_MLP_STREAM"] = self.old


def _layers(K0, widths, act, bias, pre, post, seed, dev):
    g = torch.Generator().manual_seed(seed)
    spec, mls, keep = [], [], []
    k = K0
    for n in widths:
        w = (torch.rand(n, k, generator=g) - 0.5) * (2.0 / k ** 0.5)
        d = {"w": w}
        if bias:
            d["bias"] = torch.rand(n, generator=g) - 0.5
        if pre:
            d["pre_scale"], d["pre_shift"] = torch.rand(n, generator=g) + 0.5, torch.rand(n, generator=g) - 0.5
        if post:
            d["post_scale"], d["post_shift"] = torch.rand(n, generator=g) + 0.5, torch.rand(n, generator=g) - 0.5
        if act == "dice":
            d["act_scale"], d["act_shift"] = torch.rand(n, generator=g) + 0.5, torch.rand(n, generator=g) - 0.5
            d["act_alpha"] = torch.rand(n, generator=g) - 0.5
        elif act == "prelu1":
            d["act_alpha"] = torch.rand(1, generator=g) * 0.5
        elif act == "prelu":
            d["act_alpha"] = torch.rand(n, generator=g) * 0.5
        d = {kk: v.to(dev) for kk, v in d.items()}
        kw = {kk: v for kk, v in d.items() if kk != "w"}
        a = {"prelu1": "prelu"}.get(act, act)
        if act.startswith("prelu"):
            kw["act_alpha_len"] = d["act_alpha"].numel()
        packed = ops.pack_mlp_weight(d["w"])
        mls.append(ops.make_mlp_layer(d["w"], packed, act=a, slope=0.125 if act == "leaky" else 0.0, **kw))
        keep += [packed, d]
        spec.append((d, act))
        k = n
    return spec, mls, keep


def _ref64(x, spec, hw, hb):
    h = x.double()
    for d, act in spec:
        z = h @ d["w"].double().t()
        if "bias" in d:
            z = z + d["bias"].double()
        if "pre_scale" in d:
            z = z * d["pre_scale"].double() + d["pre_shift"].double()
        if act == "relu":
            z = torch.relu(z)
        elif act == "leaky":
            z = torch.where(z > 0, z, z * 0.125)
        elif act.startswith("prelu"):
            z = torch.where(z > 0, z, z * d["act_alpha"].double())
        elif act == "dice":
            p = torch.sigmoid(z * d["act_scale"].double() + d["act_shift"].double())
            z = d["act_alpha"].double() * (1 - p) * z + p * z
        if "post_scale" in d:
            z = z * d["post_scale"].double() + d["post_shift"].double()
        h = z
    return h @ hw.double() + hb.double()


def _run_mlp(x, mls, hw, hb, on):
    logit = torch.empty(x.shape[0], device=x.device)
    prob = torch.empty(x.shape[0], device=x.device)
    ep = ops.make_epilogue(head_w=hw, head_b=hb, head_logit=logit, head_prob=prob)
    with _stream_env(on):
        ops.mlp_forward(x, mls, ep)
    torch.cuda.synchronize()
    return logit, prob


PLANS = [(50, (512, 256, 128)), (114, (512, 256, 128)), (178, (512, 256, 128)), (256, (512, 256, 128)),
         (512, (256, 128))]
ACTS = [("relu", True, True, False), ("none", True, False, False), ("leaky", False, False, True),
        ("prelu1", True, False, True), ("prelu", True, True, True), ("dice", True, False, True)]


@pytest.mark.gpu
@pytest.mark.parametrize("K0,widths", PLANS)
@pytest.mark.parametrize("act,bias,pre,post", ACTS)
def test_stream_mlp_equals_generic_and_float64(K0, widths, act, bias, pre, post):
    dev = torch.device("cuda")
    spec, mls, keep = _layers(K0, widths, act, bias, pre, post, seed=K0 + len(act), dev=dev)
    g = torch.Generator().manual_seed(7)
    hw = ((torch.rand(widths[-1], generator=g) - 0.5) * 0.2).to(dev)
    hb = torch.tensor([0.05], device=dev)
    for B in (1, 17, 1000):
        x = (torch.rand(B, K0, generator=g) * 2 - 1).to(dev)
        ls, ps = _run_mlp(x, mls, hw, hb, True)
        lg, pg = _run_mlp(x, mls, hw, hb, False)
        assert torch.equal(ls, lg), (B, (ls - lg).abs().max().item())
        assert torch.equal(ps, pg)
        ref = _ref64(x.cpu(), [({k: v.cpu() for k, v in d.items()}, a) for d, a in spec], hw.cpu(), hb.cpu())
        torch.testing.assert_close(ls.cpu().double(), ref, atol=ATOL, rtol=RTOL)


@pytest.mark.gpu
@pytest.mark.parametrize("K0,widths", PLANS)
def test_stream_mlp_32_row_workgroups_bit_identical(K0, widths, monkeypatch):
    """RANKOPS_MLP_ROWS=32 (two 16-row tiles per workgroup, each weight float4 feeding both) against
    =16 on every compiled plan: equal bit for bit at ragged batches; the default takes 32 once the
    batch gives every CU a 32-row workgroup (8197 here) and equals both."""
    dev = torch.device("cuda")
    spec, mls, keep = _layers(K0, widths, "prelu", True, True, True, seed=K0 + 5, dev=dev)
    g = torch.Generator().manual_seed(9)
    hw = ((torch.rand(widths[-1], generator=g) - 0.5) * 0.2).to(dev)
    hb = torch.tensor([0.05], device=dev)
    for B in (1, 33, 1000, 8197):
        x = (torch.rand(B, K0, generator=g) * 2 - 1).to(dev)
        got = []
        for rows in ("16", "32", None):
            if rows is None:
                monkeypatch.delenv("RANKOPS_MLP_ROWS", raising=False)
            else:
                monkeypatch.setenv("RANKOPS_MLP_ROWS", rows)
            got.append(_run_mlp(x, mls, hw, hb, True))
        for o in got[1:]:
            assert torch.equal(o[0], got[0][0]) and torch.equal(o[1], got[0][1]), B
    ref = _ref64(x.cpu(), [({k: v.cpu() for k, v in d.items()}, a) for d, a in spec], hw.cpu(), hb.cpu())
    torch.testing.assert_close(got[1][0].cpu().double(), ref, atol=ATOL, rtol=RTOL)


@pytest.mark.gpu
def test_stream_mlp_unaligned_input_stride():
    """x with a row stride that is not a multiple of 4 (the scalar staging path)."""
    dev = torch.device("cuda")
    spec, mls, keep = _layers(50, (512, 256, 128), "relu", True, True, False, seed=3, dev=dev)
    hw = torch.rand(128, device=dev) - 0.5
    hb = torch.tensor([0.1], device=dev)
    base = torch.rand(333, 53, device=dev)
    x = base[:, 1:51]
    ls, _ = _run_mlp(x, mls, hw, hb, True)
    lg, _ = _run_mlp(x, mls, hw, hb, False)
    assert torch.equal(ls, lg)


def _model_pair(name, cfg, B, seed=1000):
    """The model's eval outputs with the streamed plan and with mlp_rows (fresh modules of the same
    seed, so no launch cache or prepared plan crosses the two settings), plus the oracle."""
    inp = H.make_inputs(name, cfg, B, seed=seed)
    outs = []
    for on in (True, False):
        with _stream_env(on):
            model = H.build(name, cfg).cuda().eval()
            with torch.no_grad():
                o = H.as_tuple(H.call_model(model, name, H.to_device(inp, "cuda")))
            torch.cuda.synchronize()
            outs.append(tuple(x.clone() if isinstance(x, torch.Tensor) else x for x in o))
    return outs, inp


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 15, 17, 4096])
def test_dcn_stream_equals_generic(B):
    cfg = {"vocab": H.WECHAT_VOCAB, "interaction_weights": "frozen"}
    (s, g), _ = _model_pair("dcn", cfg, B)
    for a, b in zip(s, g):
        if isinstance(a, torch.Tensor):
            assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("B", [8197, 8192 + 31])
def test_dcn_row_tiles_ragged(B, monkeypatch):
    """dcn_fused_kernel's 32-row workgroups (RT = 2, the default from 8,192 rows) at a
    ragged batch — the last workgroup's second 16-row tile partly or wholly dead, its side waves'
    cross rows past `rows` — against the 16-row form bit for bit, with an out-of-range index in the
    second row tile of a workgroup (flagged, a zero row in both), and against the oracle."""
    import rankops
    cfg = {"vocab": H.WECHAT_VOCAB, "interaction_weights": "frozen"}
    model = H.build("dcn", cfg)
    p = H.cpu_params(model)
    inp = H.make_inputs("dcn", cfg, B, seed=31)
    inp["category"]["userid"][32 * 7 + 16 + 5] = model.embeddings["userid"].num_embeddings  # one past the table
    model = model.cuda().eval()
    d = H.to_device(inp, "cuda")
    outs = {}
    torch.manual_seed(0)  # the frozen cross weights are drawn at the first forward, as the oracle's
    for rt in ("1", "2", None):
        if rt is None:
            monkeypatch.delenv("RANKOPS_DCN_ROW_TILES", raising=False)
        else:
            monkeypatch.setenv("RANKOPS_DCN_ROW_TILES", rt)
        rankops.error_flags(reset=True)
        with torch.no_grad():
            outs[rt] = tuple(o.clone() for o in H.as_tuple(H.call_model(model, "dcn", d)) if isinstance(o, torch.Tensor))
        torch.cuda.synchronize()
        assert rankops.error_flags(reset=True) & 1, rt
    for rt in ("2", None):
        for a, b in zip(outs[rt], outs["1"]):
            assert torch.equal(a, b), rt
    # the oracle on the same inputs with the out-of-range row read as zeros (the kernel's contract)
    emb = p["embeddings.userid.weight"]
    p["embeddings.userid.weight"] = torch.cat([emb, torch.zeros(1, emb.shape[1])], 0)
    torch.manual_seed(0)
    with torch.no_grad():
        ref = H.as_tuple(H.call_oracle("dcn", cfg, p, inp))
    for o, r in zip(outs[None], ref):
        if isinstance(r, torch.Tensor):
            torch.testing.assert_close(o.cpu(), r, atol=ATOL, rtol=RTOL)


@pytest.mark.gpu
def test_dcn_stream_matches_oracle():
    cfg = {"vocab": H.WECHAT_VOCAB, "interaction_weights": "frozen"}
    model = H.build("dcn", cfg)
    p = H.cpu_params(model)
    inp = H.make_inputs("dcn", cfg, 300)
    torch.manual_seed(0)
    with torch.no_grad():
        ref = H.as_tuple(H.call_oracle("dcn", cfg, p, inp))
    with _stream_env(True):
        model = model.cuda().eval()
        torch.manual_seed(0)
        with torch.no_grad():
            out = H.as_tuple(H.call_model(model, "dcn", H.to_device(inp, "cuda")))
    for o, r in zip(out, ref):
        if isinstance(r, torch.Tensor):
            torch.testing.assert_close(o.cpu(), r, atol=ATOL, rtol=RTOL)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["plain", "softmax", "prelu", "balanced", "T130"])
def test_din_stream_equals_generic(variant, monkeypatch):
    cfg = {"T": 50, "dim": 32, "interaction_weights": "frozen", "vocab": H.WECHAT_VOCAB}
    if variant == "softmax":
        cfg["softmax"] = True
    if variant == "prelu":
        cfg["activation"] = "prelu"
    if variant == "balanced":
        monkeypatch.setenv("RANKOPS_DIN_BALANCE", "1")
    if variant == "T130":
        cfg["T"] = 130
    (s, g), inp = _model_pair("din", cfg, 1000)
    for a, b in zip(s, g):
        if isinstance(a, torch.Tensor):
            assert torch.equal(a, b), variant


@pytest.mark.gpu
def test_din_stream_matches_oracle():
    cfg = {"T": 50, "dim": 32, "interaction_weights": "frozen"}
    model = H.build("din", cfg)
    H.randomize_eval_stats(model)
    p = H.cpu_params(model)
    inp = H.make_inputs("din", cfg, 257)
    torch.manual_seed(0)
    with torch.no_grad():
        ref = H.as_tuple(H.call_oracle("din", cfg, p, inp))
    with _stream_env(True):
        model = model.cuda().eval()
        torch.manual_seed(0)
        with torch.no_grad():
            out = H.as_tuple(H.call_model(model, "din", H.to_device(inp, "cuda")))
    for o, r in zip(out, ref):
        if isinstance(r, torch.Tensor):
            torch.testing.assert_close(o.cpu(), r, atol=ATOL, rtol=RTOL)


@pytest.mark.gpu
def test_deepfm_tail_stream_equals_generic(monkeypatch):
    """The tail after rk_fm_linear_packed (the one-launch rk_deepfm_forward off: it has no generic
    twin to be bit-identical to)."""
    from rankops import deepfm as deepfm_mod
    monkeypatch.setattr(deepfm_mod, "FUSED_WHOLE", False)
    cfg = {"dim": 32, "fields": {f"field_{i:02d}": 5000 for i in range(30)}}
    (s, g), _ = _model_pair("deepfm", cfg, 4096)
    for a, b in zip(s, g):
        if isinstance(a, torch.Tensor):
            assert torch.equal(a, b)


@pytest.mark.gpu
def test_bst_tail_stream_equals_generic():
    cfg = {"T": 64, "dim": 128, "heads": 4, "max_len": 64, "vocab": H.WECHAT_VOCAB}
    (s, g), _ = _model_pair("bst", cfg, 300)
    for a, b in zip(s, g):
        if isinstance(a, torch.Tensor):
            assert torch.equal(a, b)


@pytest.mark.gpu
def test_dcn_prepare_equals_forward():
    """DCNModel.prepare: the bound rk_dcn_forward launch recomputes from the inputs' current contents."""
    cfg = {"vocab": H.WECHAT_VOCAB, "interaction_weights": "frozen"}
    model = H.build("dcn", cfg).cuda().eval()
    d = H.to_device(H.make_inputs("dcn", cfg, 1000, seed=8), "cuda")
    run = model.prepare(d["dense"], d["category"])
    with torch.no_grad():
        a = tuple(o.clone() for o in run())
        ref = model(d["dense"], d["category"])
    for x, y in zip(a, ref):
        assert torch.equal(x, y)
    e = H.to_device(H.make_inputs("dcn", cfg, 1000, seed=9), "cuda")
    d["dense"].copy_(e["dense"])
    for k in d["category"]:
        d["category"][k].copy_(e["category"][k])
    with torch.no_grad():
        b = run()
        ref = model(e["dense"], e["category"])
    for x, y in zip(b, ref):
        assert torch.equal(x, y)


@pytest.mark.gpu
def test_prepared_plan_keeps_its_weight_images_after_an_update():
    """A prepared forward pins the packed images it binds: a weight update followed by a forward
    (which repacks) gives the forward the new weights and leaves the plan on the old ones (ADVICE r3:
    no in-place rewrite under a plan that may run on another stream)."""
    cfg = {"vocab": H.WECHAT_VOCAB, "interaction_weights": "frozen"}
    model = H.build("dcn", cfg).cuda().eval()
    d = H.to_device(H.make_inputs("dcn", cfg, 500, seed=12), "cuda")
    run = model.prepare(d["dense"], d["category"])
    with torch.no_grad():
        before = run()[0].clone()
        model._tail[0].linear.weight.mul_(0.5)  # an in-place update: version bump
        after_fwd = model(d["dense"], d["category"])[0].clone()
        plan_again = run()[0].clone()
    assert torch.equal(plan_again, before)
    assert not torch.equal(after_fwd, before)
