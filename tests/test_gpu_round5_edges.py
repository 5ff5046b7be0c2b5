"""GPU: edge shapes of the round-5 kernels, called through the C ABI with synthetic tensors and
checked against plain PyTorch fp32 references of the same ops (tolerance 1e-4, the north star's):
afm_mfma_kernel at 2 and 16 fields (1 and 120 pairs: one and eight pair tiles), D 4 / 16, unit
counts off a multiple of 16; rk_mlp_forward_gather with overlapping segments (the last covering one
wins), an uncovered column, a ragged batch, a row width that is not a multiple of 4 and an
out-of-range index (zero row, flagged)."""
import pytest
import torch

import helpers as H
import rankops
from rankops import ops

ATOL = RTOL = 1e-4


def _afm_reference(tables, idx, dense, dw, db, aw, ab, ah, ahb, pw, pb):
    e = [t[i] for t, i in zip(tables, idx)]
    pairs = torch.stack([e[i] * e[j] for i in range(len(e)) for j in range(i + 1, len(e))], 1)
    scores = torch.relu(pairs @ aw.T + ab) @ ah.T + ahb
    w = torch.softmax(scores, 1)
    logit = dense @ dw.T + db + (pairs * w).sum(1) @ pw.T + pb
    return torch.sigmoid(logit), logit


@pytest.mark.gpu
@pytest.mark.parametrize("S", ["0", "2", "4"])  # afm_mfma_kernel (one sample per wave), afm_tiles_kernel S = 2 / 4
@pytest.mark.parametrize("F,D,A,B", [(2, 8, 128, 100), (16, 4, 37, 257), (9, 16, 128, 64), (16, 16, 16, 33),
                                     (7, 8, 128, 4099), (11, 4, 100, 37), (3, 16, 128, 1)])
def test_afm_mfma_edges(F, D, A, B, S, monkeypatch):
    monkeypatch.setenv("RANKOPS_AFM_S", S)
    g = torch.Generator(device="cuda").manual_seed(F * 100 + D)
    rows = 50
    tables = [torch.randn(rows, D, device="cuda", generator=g) * 0.5 for _ in range(F)]
    idx = [torch.randint(0, rows, (B,), device="cuda", generator=g) for _ in range(F)]
    nd = 5
    dense = torch.randn(B, nd, device="cuda", generator=g)
    dw, db = torch.randn(1, nd, device="cuda", generator=g), torch.randn(1, device="cuda", generator=g)
    aw, ab = torch.randn(A, D, device="cuda", generator=g) * 0.3, torch.randn(A, device="cuda", generator=g) * 0.1
    ah, ahb = torch.randn(1, A, device="cuda", generator=g) * 0.3, torch.randn(1, device="cuda", generator=g)
    pw, pb = torch.randn(1, D, device="cuda", generator=g), torch.randn(1, device="cuda", generator=g)
    logit = torch.empty(B, 1, device="cuda")
    prob = torch.empty(B, 1, device="cuda")
    segs = [ops.table_segment(t, i, 0) for t, i in zip(tables, idx)]
    ops.afm_forward(segs, D, B, dense, dw, db, aw, ab, ah, ahb, pw, pb, logit, prob)
    want_p, want_l = _afm_reference(tables, idx, dense, dw, db, aw, ab, ah, ahb, pw, pb)
    torch.testing.assert_close(logit, want_l, atol=ATOL, rtol=RTOL)
    torch.testing.assert_close(prob, want_p, atol=ATOL, rtol=RTOL)


@pytest.mark.gpu
def test_mlp_forward_gather_edges():
    torch.manual_seed(3)
    B, width, hidden = 37, 43, 64
    dense = torch.randn(B, 6, device="cuda")
    t1, t2 = torch.randn(20, 16, device="cuda"), torch.randn(30, 12, device="cuda")
    i1 = torch.randint(0, 20, (B,), device="cuda")
    i2 = torch.randint(0, 30, (B,), device="cuda")
    i2[5] = 30  # one past the table: a zero row, flagged
    # columns: dense 0..5 | t1 6..21 | t2 20..31 (overlaps t1's last two: t2 wins) | 32..41 none | dense 42
    segs = [ops.dense_segment(dense, 6, 0), ops.table_segment(t1, i1, 6), ops.table_segment(t2, i2, 20),
            ops.dense_segment(dense, 1, 42, col_offset=2)]
    x = torch.zeros(B, width, device="cuda")
    x[:, 0:6] = dense
    x[:, 6:22] = t1[i1]
    ok = (i2 < 30)[:, None]
    x[:, 20:32] = t2[i2.clamp(max=29)] * ok
    x[:, 42] = dense[:, 2]
    w1, b1 = torch.randn(hidden, width, device="cuda") * 0.2, torch.randn(hidden, device="cuda") * 0.1
    w2, b2 = torch.randn(width, hidden, device="cuda") * 0.2, torch.randn(width, device="cuda") * 0.1
    hw, hb = torch.randn(1, width, device="cuda") * 0.2, torch.randn(1, device="cuda")
    p1, p2 = ops.pack_mlp_weight(w1), ops.pack_mlp_weight(w2)
    layers = [ops.make_mlp_layer(w1, p1, bias=b1, act="relu"),
              ops.make_mlp_layer(w2, p2, bias=b2, act="relu", residual=1)]
    logit = torch.empty(B, 1, device="cuda")
    prob = torch.empty(B, 1, device="cuda")
    head = ops.make_epilogue(head_w=hw, head_b=hb, head_logit=logit, head_prob=prob)
    lib = ops._lib.load()
    ops._lib.ensure_device(x.device)
    rankops.error_flags(reset=True)
    larr = (ops._lib.MlpLayer * 2)(*layers)
    ops.check(lib.rk_mlp_forward_gather(ops._seg_array(segs), len(segs), width, B, larr, 2, ops.ctypes.byref(head),
                                        ops._lib.stream_of(prob)), "rk_mlp_forward_gather")
    torch.cuda.synchronize()
    assert rankops.error_flags(reset=True) & 1
    h = torch.relu(x @ w1.T + b1)
    y = torch.relu(x + (h @ w2.T + b2))
    want = y @ hw.T + hb
    torch.testing.assert_close(logit, want, atol=ATOL, rtol=RTOL)
    torch.testing.assert_close(prob, torch.sigmoid(want), atol=ATOL, rtol=RTOL)


@pytest.mark.gpu
def test_prepare_rejects_converted_index_copies():
    """prepare() binds its index tensors by address, so an input that would need a
    converted copy (int32 indices, a non-contiguous sequence) is refused instead of silently bound
    to a copy that stops following the caller's tensor."""
    cfg = {"vocab": H.WECHAT_VOCAB, "dim": 8, "att": 128}
    model = H.build("afm", cfg).cuda().eval()
    d = H.to_device(H.make_inputs("afm", cfg, 64, seed=3), "cuda")
    model.prepare(d["dense_input"], d["category_input"])  # int64: bound
    name = next(iter(d["category_input"]))
    d["category_input"][name] = d["category_input"][name].int()
    with pytest.raises(TypeError):
        model.prepare(d["dense_input"], d["category_input"])
    cfg = {"vocab": H.WECHAT_VOCAB, "T": 50, "dim": 16, "heads": 4, "max_len": 50}
    model = H.build("bst", cfg).cuda().eval()
    d = H.to_device(H.make_inputs("bst", cfg, 64, seed=4), "cuda")
    wide = torch.zeros(64, 100, dtype=torch.int64, device="cuda")
    wide[:, ::2] = d["seq_feedid"]
    with pytest.raises(ValueError):
        model.prepare(d["dense"], d["category"], wide[:, ::2], d["seq_length"])


@pytest.mark.gpu
@pytest.mark.parametrize("S", ["0", "2", "4"])
def test_afm_out_of_range_index_zero_row(S, monkeypatch):
    """An out-of-range index reads a zero embedding row (and raises RK_FLAG_INDEX_OOB) in every AFM
    kernel: the outputs equal the reference with that row zeroed."""
    monkeypatch.setenv("RANKOPS_AFM_S", S)
    g = torch.Generator(device="cuda").manual_seed(5)
    F, D, A, B, rows = 7, 8, 128, 77, 40
    tables = [torch.randn(rows, D, device="cuda", generator=g) * 0.5 for _ in range(F)]
    idx = [torch.randint(0, rows, (B,), device="cuda", generator=g) for _ in range(F)]
    idx[3][10] = rows  # one past the table
    dense = torch.randn(B, 4, device="cuda", generator=g)
    dw, db = torch.randn(1, 4, device="cuda", generator=g), torch.randn(1, device="cuda", generator=g)
    aw, ab = torch.randn(A, D, device="cuda", generator=g) * 0.3, torch.randn(A, device="cuda", generator=g) * 0.1
    ah, ahb = torch.randn(1, A, device="cuda", generator=g) * 0.3, torch.randn(1, device="cuda", generator=g)
    pw, pb = torch.randn(1, D, device="cuda", generator=g), torch.randn(1, device="cuda", generator=g)
    logit, prob = torch.empty(B, 1, device="cuda"), torch.empty(B, 1, device="cuda")
    segs = [ops.table_segment(t, i, 0) for t, i in zip(tables, idx)]
    rankops.error_flags(reset=True)
    ops.afm_forward(segs, D, B, dense, dw, db, aw, ab, ah, ahb, pw, pb, logit, prob)
    torch.cuda.synchronize()
    assert rankops.error_flags(reset=True) & 1
    padded = [torch.cat([t, torch.zeros(1, D, device="cuda")]) for t in tables]
    want_p, want_l = _afm_reference(padded, idx, dense, dw, db, aw, ab, ah, ahb, pw, pb)
    torch.testing.assert_close(logit, want_l, atol=ATOL, rtol=RTOL)
    torch.testing.assert_close(prob, want_p, atol=ATOL, rtol=RTOL)
