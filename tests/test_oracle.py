"""CPU tests of the oracle (test infrastructure): it reproduces the committed golden fixtures,
agrees with the independent float64 numpy restatement, and encodes the reference's edge
semantics (SURVEY.md §8 hazards H1-H4)."""
import glob
import json
import os

import numpy as np
import pytest
import torch

import helpers as H
from golden.make_golden import unflatten
from oracle import reference_forward as ref
from oracle import reference_np as rnp

GOLDEN = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz")))


def load_golden(path):
    z = np.load(path, allow_pickle=False)
    arrs = {k: z[k] for k in z.files}
    meta = json.loads(str(arrs.pop("meta")))
    p = unflatten(arrs, "p")
    inp = unflatten(arrs, "in")
    outs = [torch.from_numpy(np.array(arrs[f"out::{i}"])) for i in range(sum(k.startswith("out::") for k in arrs))]
    h2 = [torch.from_numpy(np.array(arrs[f"h2::{i}"])) for i in range(sum(k.startswith("h2::") for k in arrs))]
    return meta, p, inp, outs, h2


def test_golden_present():
    assert len(GOLDEN) >= 9


@pytest.mark.parametrize("path", GOLDEN, ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_reproduces_golden(path):
    meta, p, inp, outs, _ = load_golden(path)
    torch.manual_seed(meta["draw_seed"])
    with torch.no_grad():
        got = H.as_tuple(H.call_oracle(meta["model"], meta["cfg"], p, inp))
    assert len(got) == len(outs)
    for g, o in zip(got, outs):
        g = g if isinstance(g, torch.Tensor) else torch.tensor(g, dtype=torch.float32)
        torch.testing.assert_close(g.reshape(o.shape), o, atol=1e-6, rtol=1e-6, equal_nan=True)


def _np(x):
    if isinstance(x, dict):
        return {k: _np(v) for k, v in x.items()}
    return x.numpy() if isinstance(x, torch.Tensor) else x


@pytest.mark.parametrize("path", GOLDEN, ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_matches_numpy_float64(path):
    """Two independent codings of the reference lines agree (fp32 vs fp64)."""
    meta, p, inp, outs, h2 = load_golden(path)
    name, cfg = meta["model"], meta["cfg"]
    P = _np(p)
    I = _np(inp)
    nh = len(cfg.get("hidden", [512, 256, 128]))
    if name == "dcn":
        cross = [(h2[2 * i].numpy(), h2[2 * i + 1].numpy()) for i in range(len(h2) // 2)]
        got = rnp.dcn(P, I["dense"], I["category"], cross, nh)
    elif name == "deepfm":
        got = rnp.deepfm(P, I["category"], list(I["category"].keys()), ref.deepfm_layout(nh))
    elif name == "din":
        got = rnp.din(P, I["dense"], I["category"], I["sequence"], I["target"],
                      ref.din_layout(nh, cfg.get("activation", "dice")), cfg.get("activation", "dice"),
                      cfg.get("softmax", False), cfg.get("l2", 0.2), [t.numpy() for t in h2])
    elif name == "afm":
        got = rnp.afm(P, I["dense_input"], I["category_input"], list(I["category_input"].keys()))
    elif name == "deepcrossing":
        units = [[h2[4 * i + j].numpy() for j in range(4)] for i in range(len(h2) // 4)]
        got = rnp.deepcrossing(P, I["dense"], I["category"], units)
    elif name == "bst":
        layout, last = ref.bst_dnn_layout(nh)
        got = rnp.bst(P, I["dense"], I["category"], I["seq_feedid"], I["seq_length"], cfg.get("heads", 4),
                      cfg.get("blocks", 1), layout, last, cfg.get("pooling", "sum"))
    else:
        raise AssertionError(name)
    for g, o in zip(got, outs):
        np.testing.assert_allclose(np.asarray(g, np.float64).reshape(o.shape), o.numpy().astype(np.float64),
                                   rtol=2e-5, atol=2e-5)


def test_din_softmax_empty_history_is_uniform():
    """(-2**32+1) padding is finite in fp32 (din.py:74): a length-0 row softmaxes to 1/T."""
    g = torch.Generator().manual_seed(0)
    keys = torch.randn(3, 6, 4, generator=g)
    q = torch.randn(3, 4, generator=g)
    att = ref.draw_din_att(4)
    out = ref.din_attention(q, keys, torch.tensor([0, 6, 2]), True, att)
    torch.testing.assert_close(out[0], keys[0].mean(0), atol=1e-6, rtol=1e-6)
    plain = ref.din_attention(q, keys, torch.tensor([0, 6, 2]), False, att)
    assert torch.count_nonzero(plain[0]) == 0


def test_bst_empty_sequence_gives_nan():
    meta, p, inp, outs, _ = load_golden(os.path.join(os.path.dirname(__file__), "golden", "bst.npz"))
    assert torch.isnan(outs[1][0]).all() and not torch.isnan(outs[1][1:]).any()


def test_cross_layer_draw_statistics():
    """xavier_normal_ on a (d, 1) tensor: std = sqrt(2 / (d + 1)) (dcn.py:40); b = 0."""
    torch.manual_seed(0)
    ws = torch.cat([ref.draw_cross(50, 1)[0][0].flatten() for _ in range(400)])
    assert abs(float(ws.std()) - (2 / 51) ** 0.5) < 0.01
    assert float(ref.draw_cross(50, 1)[0][1].abs().sum()) == 0.0


def test_product_draws_equal_oracle_draws():
    """rankops re-implements the H2 draws; with the same seed they are identical to the oracle's."""
    import rankops.common as C
    torch.manual_seed(5)
    a = ref.draw_cross(50, 3)
    torch.manual_seed(5)
    bw, bb = C.draw_cross_layers(50, 3)
    for i, (w, b) in enumerate(a):
        assert torch.equal(w.flatten(), bw[i]) and torch.equal(b.flatten(), bb[i])
    torch.manual_seed(6)
    a = ref.draw_din_att(32)
    torch.manual_seed(6)
    b = C.draw_din_attention(32)
    assert all(torch.equal(x, y) for x, y in zip(a, b))
    torch.manual_seed(8)
    a = [ref.draw_residual(50, 64) for _ in range(2)]
    torch.manual_seed(8)
    b = C.draw_residual_units(50, 64, 2)
    assert all(torch.equal(x, y) for u, v in zip(a, b) for x, y in zip(u, v))
