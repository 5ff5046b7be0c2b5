"""GPU parity of the fused DeepFM front end (rk_fm_linear_packed: packed-table gather, fm1, fm2 and
the first deep layer in one launch; deepfm.py:100-112,122-142) — directly against a float64 torch
restatement on ragged shapes, and through rankops.DeepFM at the configs[1] field shape against the
CPU oracle.  Tolerance as every forward test: atol = rtol = 1e-4 (fp32)."""
import pytest
import torch

import helpers as H
import rankops
from rankops import common, ops
from rankops import deepfm as deepfm_mod

ATOL = RTOL = 1e-4
FIELDS30 = {f"field_{i:02d}": 1000 + 37 * i for i in range(30)}


def _case(M, F, D, n, seed, oob=False):
    g = torch.Generator().manual_seed(seed)
    RS = (D + 1 + 3) // 4 * 4
    rows = [50 + 13 * f for f in range(F)]
    tables = [torch.randn(V, RS, generator=g).cuda() for V in rows]
    idx = [torch.randint(0, V, (M,), generator=g).cuda() for V in rows]
    for f in range(F):  # first and last row of every table
        idx[f][0], idx[f][M - 1] = 0, rows[f] - 1
    if oob:
        idx[F // 2][M // 3] = rows[F // 2] + 5
    K = F * D
    w = (0.05 * torch.randn(n, K, generator=g)).cuda()
    b = torch.randn(n, generator=g).cuda()
    sc = (1 + 0.1 * torch.randn(n, generator=g)).cuda()
    sh = (0.1 * torch.randn(n, generator=g)).cuda()
    return tables, idx, w, b, sc, sh


def _reference(tables, idx, D, w, b, sc, sh, oob_rows=()):
    rows = []
    for t, i in zip(tables, idx):
        ok = (i >= 0) & (i < t.shape[0])
        r = t.double()[torch.where(ok, i, 0)]
        rows.append(torch.where(ok[:, None], r, torch.zeros_like(r)))
    emb = torch.stack([r[:, :D] for r in rows], 1)          # [M, F, D]
    fm1 = torch.stack([r[:, D] for r in rows], 1).sum(1, keepdim=True)
    s = emb.sum(1)
    fm2 = 0.5 * (s * s - (emb * emb).sum(1)).sum(1, keepdim=True)
    z = (emb.reshape(emb.shape[0], -1) @ w.double().T + b.double()) * sc.double() + sh.double()
    y = torch.relu(z)
    return y.float(), fm1.float(), fm2.float()


@pytest.mark.gpu
@pytest.mark.parametrize("M,F,D,n", [(4100, 30, 32, 512), (333, 7, 8, 50), (1000, 3, 256, 200), (70, 32, 4, 130),
                                     (64, 1, 64, 64)])
def test_fm_linear_packed_direct(M, F, D, n):
    """Ragged batches (not a multiple of 64), widths (not a multiple of 128), K = F * D not a
    multiple of the 256-wide LDS block, every supported dim class, tables' first and last rows."""
    tables, idx, w, b, sc, sh = _case(M, F, D, n, seed=M + F + D)
    segs = [ops.packed_segment(t, i, D, f * D) for f, (t, i) in enumerate(zip(tables, idx))]
    packed = ops.pack_mlp_weight(w)
    layer = ops.make_mlp_layer(w, packed, bias=b, pre_scale=sc, pre_shift=sh, act="relu")
    y = torch.full((M, n), float("nan"), device="cuda")
    fm1 = torch.full((M, 1), float("nan"), device="cuda")
    fm2 = torch.full((M, 1), float("nan"), device="cuda")
    rankops.error_flags(reset=True)
    ops.fm_linear_packed(segs, D, M, layer, y, fm1, fm2)
    torch.cuda.synchronize()
    assert rankops.error_flags(reset=True) == 0
    ry, r1, r2 = _reference(tables, idx, D, w, b, sc, sh)
    torch.testing.assert_close(y, ry.cuda(), atol=ATOL, rtol=RTOL)
    torch.testing.assert_close(fm1, r1.cuda(), atol=ATOL, rtol=RTOL)
    torch.testing.assert_close(fm2, r2.cuda(), atol=ATOL, rtol=RTOL)


@pytest.mark.gpu
def test_fm_linear_packed_out_of_range_reads_zero_row_and_flags():
    M, F, D, n = 300, 6, 32, 128
    tables, idx, w, b, sc, sh = _case(M, F, D, n, seed=9, oob=True)
    segs = [ops.packed_segment(t, i, D, f * D) for f, (t, i) in enumerate(zip(tables, idx))]
    packed = ops.pack_mlp_weight(w)  # the layer holds its pointer only: keep the image alive
    layer = ops.make_mlp_layer(w, packed, bias=b, pre_scale=sc, pre_shift=sh, act="relu")
    y, fm1, fm2 = (torch.empty(M, n, device="cuda"), torch.empty(M, 1, device="cuda"), torch.empty(M, 1, device="cuda"))
    rankops.error_flags(reset=True)
    ops.fm_linear_packed(segs, D, M, layer, y, fm1, fm2)
    torch.cuda.synchronize()
    assert rankops.error_flags(reset=True) & 1
    ry, r1, r2 = _reference(tables, idx, D, w, b, sc, sh)
    torch.testing.assert_close(y, ry.cuda(), atol=ATOL, rtol=RTOL)
    torch.testing.assert_close(fm2, r2.cuda(), atol=ATOL, rtol=RTOL)


@pytest.mark.gpu
def test_fm_linear_packed_rejects_bad_layouts():
    M, F, D, n = 64, 4, 8, 64
    tables, idx, w, b, sc, sh = _case(M, F, D, n, seed=2)
    packed = ops.pack_mlp_weight(w)
    layer = ops.make_mlp_layer(w, packed, bias=b, act="relu")
    y, fm1, fm2 = (torch.empty(M, n, device="cuda"), torch.empty(M, 1, device="cuda"), torch.empty(M, 1, device="cuda"))
    bad_col = [ops.packed_segment(t, i, D, f * D + (4 if f == 2 else 0)) for f, (t, i) in enumerate(zip(tables, idx))]
    with pytest.raises(rankops._lib.RankOpsError):
        ops.fm_linear_packed(bad_col, D, M, layer, y, fm1, fm2)
    segs = [ops.packed_segment(t, i, D, f * D) for f, (t, i) in enumerate(zip(tables, idx))]
    with pytest.raises(rankops._lib.RankOpsError):  # dim 12 is not a power of two
        ops.fm_linear_packed(segs, 12, M, layer, y, fm1, fm2)


@pytest.mark.gpu
@pytest.mark.parametrize("B", [4096, 4100])
def test_deepfm_fused_front_against_oracle(B, monkeypatch):
    """rankops.DeepFM at configs[1]'s field shape (30 fields x 32, 512-256-128) and a batch that
    tiles the first layer, with the one-launch forward off (FUSED_WHOLE, tests/test_gpu_deepfm_fused.py):
    the eval forward is rk_fm_linear_packed + rk_mlp_forward, equal to the oracle and to the unfused
    gather + tiled-layer path."""
    monkeypatch.setattr(deepfm_mod, "FUSED_WHOLE", False)
    cfg = {"dim": 32, "fields": FIELDS30}
    model = H.build("deepfm", cfg)
    H.randomize_eval_stats(model, 5)
    p = H.cpu_params(model)
    inp = H.make_inputs("deepfm", cfg, B)
    with torch.no_grad():
        ref = H.as_tuple(H.call_oracle("deepfm", cfg, p, inp))
    model = model.cuda().eval()
    d = H.to_device(inp, "cuda")
    with torch.no_grad():
        out = H.as_tuple(model(d["category"]))
    torch.cuda.synchronize()
    entry = next(iter(model.__dict__["_eager"]._d.values()))
    assert [name for name, _ in entry[0]] == ["rk_fm_linear_packed", "rk_mlp_forward"]
    for i, (o, r) in enumerate(zip(out, ref)):
        torch.testing.assert_close(o.cpu(), r, atol=ATOL, rtol=RTOL, msg=lambda m: f"fused[{i}]: {m}")
    deepfm_mod.FUSED_FRONT = False
    try:
        model.__dict__.pop("_eager")
        with torch.no_grad():
            plain = H.as_tuple(model(d["category"]))
        entry = next(iter(model.__dict__["_eager"]._d.values()))
        assert [name for name, _ in entry[0]] == ["rk_fm_gather_packed", "rk_linear_tiled", "rk_mlp_forward"]
    finally:
        deepfm_mod.FUSED_FRONT = True
    for o, q in zip(out, plain):
        torch.testing.assert_close(o, q, atol=ATOL, rtol=RTOL)
