"""GPU parity of the packed DeepFM eval tables (rk_fm_pack_table + rk_fm_gather_packed) and of
the table-sharded DeepFM at P = 1, both against the CPU oracle (deepfm.py:122-151 restated in
oracle/reference_forward.py).  Tolerance as every forward test: atol = rtol = 1e-4 (fp32)."""
import numpy as np
import pytest
import torch

import helpers as H
import rankops
from rankops import deepfm as deepfm_mod
from rankops import ops, sharded

ATOL = RTOL = 1e-4
FIELDS30 = {f"field_{i:02d}": 1000 + 37 * i for i in range(30)}


def _oracle(model, cfg, inp):
    p = H.cpu_params(model)
    with torch.no_grad():
        return H.as_tuple(H.call_oracle("deepfm", cfg, p, inp))


def _close(out, ref, what):
    for i, (o, r) in enumerate(zip(H.as_tuple(out), ref)):
        torch.testing.assert_close(o.detach().cpu(), r, atol=ATOL, rtol=RTOL, msg=lambda m: f"{what}[{i}]: {m}")


@pytest.mark.gpu
def test_pack_table_layout_is_exact():
    """Packed row r = [second[r, :D], first[r, 0], 0 pad]: a pure copy, bit-exact."""
    for V, D in ((1, 4), (37, 8), (1000, 32), (5, 64)):
        g = torch.Generator().manual_seed(V + D)
        second = torch.randn(V, D, generator=g).cuda()
        first = torch.randn(V, 1, generator=g).cuda()
        RS = (D + 1 + 3) // 4 * 4
        pk = ops.fm_pack_table(second, first, RS)
        torch.cuda.synchronize()
        want = torch.zeros(V, RS)
        want[:, :D] = second.cpu()
        want[:, D] = first.cpu()[:, 0]
        assert torch.equal(pk.cpu(), want), (V, D)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [{}, {"dim": 32, "fields": FIELDS30}, {"dim": 16, "batch_norm": False},
                                 {"dim": 4}], ids=["wechat-dim8", "30fields-dim32", "dim16-nobn", "dim4"])
def test_packed_equals_unpacked_and_oracle(cfg, monkeypatch):
    """The packed gather gives the same bits as the two-table gather (same rows, same order of
    additions) and matches the oracle."""
    model = H.build("deepfm", cfg)
    inp = H.make_inputs("deepfm", cfg, 517)
    ref = _oracle(model, cfg, inp)
    model = model.cuda().eval()
    dinp = H.to_device(inp, "cuda")
    with torch.no_grad():
        packed = H.as_tuple(model(dinp["category"]))
        monkeypatch.setattr(deepfm_mod, "PACKED_TABLES", False)
        plain = H.as_tuple(model(dinp["category"]))
    torch.cuda.synchronize()
    for a, b in zip(packed, plain):
        assert torch.equal(a, b)
    _close(packed, ref, "deepfm-packed")


@pytest.mark.gpu
def test_packed_tables_follow_weight_updates():
    """The packed image is rebuilt after an in-place weight update, load_state_dict and .to()."""
    cfg = {"dim": 8}
    model = H.build("deepfm", cfg).cuda().eval()
    inp = H.make_inputs("deepfm", cfg, 64)
    dinp = H.to_device(inp, "cuda")
    with torch.no_grad():
        model(dinp["category"])
        name = next(iter(model.second_order_embeddings))
        model.second_order_embeddings[name].weight.mul_(2.0)   # in-place: version bump
        model.first_order_embeddings[name].weight.add_(0.25)
        out = model(dinp["category"])
    _close(out, _oracle(model.cpu(), cfg, inp), "after in-place update")
    model = model.cuda()
    sd = {k: (v * 0.5 if "embeddings" in k else v) for k, v in model.state_dict().items()}
    model.load_state_dict(sd)
    with torch.no_grad():
        out = model(dinp["category"])
    _close(out, _oracle(model.cpu(), cfg, inp), "after load_state_dict")


@pytest.mark.gpu
def test_packed_out_of_range_index_is_flagged():
    cfg = {"dim": 8}
    model = H.build("deepfm", cfg).cuda().eval()
    inp = H.to_device(H.make_inputs("deepfm", cfg, 64), "cuda")
    rankops.error_flags(reset=True)
    name = next(iter(model.second_order_embeddings))
    inp["category"][name][5] = model.vocab_sizes[name] + 3
    with torch.no_grad():
        model(inp["category"])
    assert rankops.error_flags(reset=True) & 1


@pytest.mark.gpu
def test_sharded_p1_against_oracle_configs4_shape():
    """ShardedDeepFM at P = 1 (configs[4]'s field shape: 30 fields, dim 32, the 512-256-128 tail)
    against the oracle, not against rankops.DeepFM.  Reduced rows per field so the oracle runs in
    seconds; ids cover row 0 and the last row."""
    cfg = {"dim": 32, "fields": {f"field_{i:02d}": 3000 + 11 * i for i in range(30)}}
    full = H.build("deepfm", cfg)
    H.randomize_eval_stats(full, 43)
    inp = H.make_inputs("deepfm", cfg, 1024)
    for f, n in cfg["fields"].items():
        inp["category"][f][0] = 0
        inp["category"][f][1] = n  # last addressable row (table has n + 1 rows)
    ref = _oracle(full, cfg, inp)
    sh = sharded.ShardedDeepFM.from_deepfm(full.cuda().eval(), rank=0, world_size=1)
    with torch.no_grad():
        out = sh(H.to_device(inp, "cuda")["category"])
    _close(out, ref, "sharded-p1")


@pytest.mark.gpu
def test_sharded_gather_local_rows_are_packed_rows():
    """Step 2 of the P > 1 path (one concat gather of whole packed rows) on one device: the
    [R][f_me][RS] send rows equal the packed tables at the received indices, bit-exact."""
    cfg = {"dim": 32, "fields": {f"f{i:02d}": 200 + i for i in range(6)}}
    full = H.build("deepfm", cfg).cuda().eval()
    sh = sharded.ShardedDeepFM.from_deepfm(full, rank=0, world_size=1)
    rng = np.random.default_rng(3)
    R, F = 77, len(cfg["fields"])
    recv = torch.from_numpy(np.stack([rng.integers(0, n + 1, R) for n in cfg["fields"].values()], 1)
                            .astype(np.int64).reshape(-1)).cuda()
    rows = sh.gather_local(recv, R)
    torch.cuda.synchronize()
    RS = sharded.row_stride(32)
    got = rows.view(R, F, RS).cpu()
    for j, f in enumerate(sh.local_fields):
        idx = recv.view(R, F)[:, j].cpu()
        want = torch.zeros(R, RS)
        want[:, :32] = full.second_order_embeddings[f].weight.detach().cpu()[idx]
        want[:, 32] = full.first_order_embeddings[f].weight.detach().cpu()[idx, 0]
        assert torch.equal(got[:, j], want), f


def _fm64(tables2, tables1, idx, D):
    """float64 FM sums and the deep-input row (deepfm.py:122-140), out-of-range rows as zeros."""
    e, w = [], []
    for t2, t1, i in zip(tables2, tables1, idx):
        ok = (i >= 0) & (i < t2.shape[0])
        ci = i.clamp(0, t2.shape[0] - 1)
        e.append(t2[ci].double() * ok[:, None])
        w.append(t1[ci, 0].double() * ok)
    E = torch.stack(e, 1)
    fm1 = torch.stack(w, 1).sum(1)
    fm2 = 0.5 * (E.sum(1) ** 2 - (E ** 2).sum(1)).sum(1)
    return E.reshape(E.shape[0], -1), fm1, fm2


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["tables", "shared_idx", "packed", "dense"])
@pytest.mark.parametrize("D,B", [(32, 16389), (8, 16400), (64, 16385), (4, 16391)])
def test_field_major_gather_equals_sample_major(mode, D, B, monkeypatch):
    """rk_fm_gather / rk_fm_gather_packed's field-major kernel (round 6, from 16,384 samples by
    default; RANKOPS_FM_FMAJ_MIN) against the sample-major one (RANKOPS_FM_FMAJ_MIN=0) on the same
    inputs: the deep-input rows bit-identical (copies), fm1 / fm2 within fp32 rounding of each other
    and of a float64 restatement; ragged batches (the last wave's dead sample slots), 29 fields
    (the last round of fields partial), an out-of-range index in each mode that takes indices."""
    dev = "cuda"
    F, V = 29, 3000
    g = torch.Generator(device=dev).manual_seed(D + B)
    t2 = [torch.randn(V, D, device=dev, generator=g) for _ in range(F)]
    t1 = [torch.randn(V, 1, device=dev, generator=g) for _ in range(F)]
    idx = [torch.randint(0, V, (B,), device=dev, generator=g) for _ in range(F)]
    if mode != "dense":
        idx[7][B - 3] = V  # one past the table: a zero row, flagged
    E, f1, f2 = _fm64([t.cpu() for t in t2], [t.cpu() for t in t1], [i.cpu() for i in idx], D)
    outs = {}
    for fmaj in ("1", "0"):
        monkeypatch.setenv("RANKOPS_FM_FMAJ_MIN", fmaj)
        deep = torch.full((B, F * D + 4), float("nan"), device=dev)
        fm1 = torch.empty(B, device=dev)
        fm2 = torch.empty(B, device=dev)
        rankops.error_flags(reset=True)
        if mode == "packed":
            packed = [ops.fm_pack_table(a, b, (D + 1 + 3) // 4 * 4) for a, b in zip(t2, t1)]
            segs = [ops.packed_segment(p, i, D, f * D) for f, (p, i) in enumerate(zip(packed, idx))]
            ops.fm_gather_packed(segs, D, B, deep, fm1, fm2)
        elif mode == "dense":  # rows already gathered: row b of a [B, D] block per field
            rows2 = [t[i] for t, i in zip(t2, idx)]
            rows1 = [t[i] for t, i in zip(t1, idx)]
            second = [ops.dense_segment(r, D, f * D) for f, r in enumerate(rows2)]
            first = [ops.dense_segment(r, 1, f) for f, r in enumerate(rows1)]
            ops.fm_gather(second, first, D, B, deep, fm1, fm2)
        else:
            second = [ops.table_segment(t, i, f * D) for f, (t, i) in enumerate(zip(t2, idx))]
            if mode == "tables":  # first-order indices through their own (strided) view
                first = [ops.table_segment(t, i, f) for f, (t, i) in enumerate(zip(t1, [x.clone() for x in idx]))]
            else:
                first = [ops.table_segment(t, i, f) for f, (t, i) in enumerate(zip(t1, idx))]
            ops.fm_gather(second, first, D, B, deep, fm1, fm2)
        torch.cuda.synchronize()
        flagged = rankops.error_flags(reset=True) & 1
        assert bool(flagged) == (mode != "dense"), (fmaj, mode)
        outs[fmaj] = (deep.clone(), fm1.clone(), fm2.clone())
    (d1, a1, b1), (d0, a0, b0) = outs["1"], outs["0"]
    assert torch.equal(d1[:, :F * D], d0[:, :F * D])
    assert torch.isnan(d1[:, F * D:]).all()  # columns past the fields untouched
    torch.testing.assert_close(d1[:, :F * D].cpu().double(), E)
    for got in ((a1, b1), (a0, b0)):
        torch.testing.assert_close(got[0].cpu().double(), f1, atol=ATOL, rtol=RTOL)
        torch.testing.assert_close(got[1].cpu().double(), f2, atol=1e-3, rtol=RTOL)
    torch.testing.assert_close(a1, a0, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(b1, b0, atol=1e-3, rtol=1e-4)
