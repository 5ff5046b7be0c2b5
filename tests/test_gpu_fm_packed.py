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
