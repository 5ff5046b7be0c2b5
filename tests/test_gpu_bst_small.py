"""GPU: rk_bst_forward_blocks at the reference script's own width, d_model 16 (bst.py:192 hard-codes
it; bst_small_kernel in csrc/bst_small.hip: one wave per sample, lane = position), against the CPU
oracle (oracle.reference_forward: bst.py:66-91, 216-247) and against the per-layer path
(common.FUSED_BST = False).  Heads 1/2/4/8, T 1..64, 1-3 blocks, sum and mean pooling, lengths
0 (NaN, as torch's all-masked softmax) / 1 / T / past T, out-of-range sequence indices."""
import pytest
import torch

import helpers as H
import rankops
from test_gpu_parity import _compare, run_pair

ATOL = RTOL = 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [
    {"T": 50, "heads": 4},                      # the reference script's defaults
    {"T": 50, "heads": 4, "pooling": "mean"},
    {"T": 64, "heads": 1, "max_len": 64},
    {"T": 33, "heads": 2, "blocks": 2},
    {"T": 17, "heads": 8, "blocks": 3, "batch_norm": False},
    {"T": 1, "heads": 4},
])
def test_small_bst_matches_oracle(cfg):
    model = H.build("bst", cfg)
    assert model._fused_blocks(cfg["T"]) is not None  # the d_model 16 fused path is taken
    inp = H.make_inputs("bst", cfg, 200, seed=31)
    inp["seq_length"][:3] = torch.tensor([0, 1, cfg["T"]])
    if cfg["T"] > 1:
        inp["seq_length"][3] = cfg["T"] + 5  # longer than the padded width: every key valid
    out, ref = run_pair("bst", cfg, B=200, inputs=inp, model=model)
    _compare(out, ref, f"bst16-{cfg}")
    assert torch.isnan(out[1][0].cpu()).all()  # length 0: all keys masked -> NaN like the reference
    assert rankops.error_flags() == 0


@pytest.mark.gpu
def test_small_bst_equals_per_layer_path_at_bench_shape(monkeypatch):
    cfg = {"T": 50, "heads": 4, "vocab": H.WECHAT_VOCAB}
    model = H.build("bst", cfg).cuda()
    inp = H.to_device(H.make_inputs("bst", cfg, 4096, seed=5), "cuda")
    with torch.no_grad():
        fused = H.as_tuple(H.call_model(model, "bst", inp))
        monkeypatch.setattr(rankops.common, "FUSED_BST", False)
        plain = H.as_tuple(H.call_model(model, "bst", inp))
    for a, b in zip(fused, plain):
        torch.testing.assert_close(a, b, atol=ATOL, rtol=RTOL, equal_nan=True)


@pytest.mark.gpu
def test_small_bst_oob_sequence_index_is_flagged():
    cfg = {"T": 16, "heads": 4}
    model = H.build("bst", cfg).cuda()
    inp = H.to_device(H.make_inputs("bst", cfg, 64, seed=9), "cuda")
    inp["seq_feedid"][5, 2] = model.embeddings["feedid"].num_embeddings  # one past the table
    rankops.error_flags(reset=True)
    with torch.no_grad():
        H.call_model(model, "bst", inp)
    assert rankops.error_flags(reset=True) & 1


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,batch", [
    ({"T": 50, "heads": 4, "vocab": H.WECHAT_VOCAB}, 4096),   # the bench leg (models.bst_ref)
    ({"T": 50, "heads": 4, "pooling": "mean"}, 4133),           # a partial last workgroup
    ({"T": 64, "heads": 1, "max_len": 64}, 300),
    ({"T": 33, "heads": 2, "blocks": 2}, 17),
    ({"T": 17, "heads": 8, "blocks": 3, "batch_norm": False}, 64),
])
def test_small_bst_one_launch_equals_three_launches(monkeypatch, cfg, batch):
    """rk_bst_small_forward (the whole d_model-16 forward in one launch: row gather, blocks, pooling,
    DNN tail, head) against rk_concat_gather + rk_bst_forward_blocks + rk_mlp_forward on the same
    inputs: the same gather, the same per-sample block code and the same streamed tail, so the
    outputs agree bit for bit (NaN rows of length-0 sequences included)."""
    model = H.build("bst", cfg).cuda().eval()
    inp = H.make_inputs("bst", cfg, batch, seed=41)
    inp["seq_length"][:2] = torch.tensor([0, cfg["T"]])
    d = H.to_device(inp, "cuda")
    calls = []
    real = rankops.ops.bst_small_forward
    monkeypatch.setattr(rankops.ops, "bst_small_forward", lambda *a, **k: calls.append(1) or real(*a, **k))
    with torch.no_grad():
        one = H.as_tuple(H.call_model(model, "bst", d))
        assert calls, "the one-launch path was not taken"
        monkeypatch.setattr(rankops.common, "FUSED_BST_FWD", False)
        three = H.as_tuple(H.call_model(model, "bst", d))
    for a, b in zip(one, three):
        torch.testing.assert_close(a, b, atol=0, rtol=0, equal_nan=True)


@pytest.mark.gpu
def test_small_bst_one_launch_oob_category_index_is_flagged():
    cfg = {"T": 16, "heads": 4}
    model = H.build("bst", cfg).cuda().eval()
    inp = H.to_device(H.make_inputs("bst", cfg, 64, seed=9), "cuda")
    inp["category"]["userid"][3] = model.embeddings["userid"].num_embeddings + 7
    rankops.error_flags(reset=True)
    with torch.no_grad():
        H.call_model(model, "bst", inp)
    assert rankops.error_flags(reset=True) & 1


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [{"T": 50, "heads": 4, "vocab": H.WECHAT_VOCAB},
                                 {"T": 64, "heads": 4, "max_len": 64, "pooling": "mean", "blocks": 2},
                                 {"T": 7, "heads": 4, "max_len": 8}])
def test_small_bst_mfma_equals_valu_kernel(monkeypatch, cfg):
    """4 heads run on the matrix cores (bst_mfma_sample); RANKOPS_BST_MFMA=0 selects the VALU kernel:
    the two agree within the fp32 tolerance on the whole forward and on the blocks-only launch."""
    model = H.build("bst", cfg).cuda()
    inp = H.to_device(H.make_inputs("bst", cfg, 1000, seed=13), "cuda")
    inp["seq_length"][:4] = torch.tensor([1, cfg["T"], cfg["T"] + 3, 2], device="cuda")
    with torch.no_grad():
        mf = H.as_tuple(H.call_model(model, "bst", inp))
        launch = model.blocks_kernel_launcher(inp["seq_feedid"], inp["seq_length"])
        pm = launch()
        pm = pm.clone() if isinstance(pm, torch.Tensor) else None
        monkeypatch.setenv("RANKOPS_BST_MFMA", "0")
        va = H.as_tuple(H.call_model(model, "bst", inp))
    torch.cuda.synchronize()
    for a, b in zip(mf, va):
        torch.testing.assert_close(a, b, atol=ATOL, rtol=RTOL, equal_nan=True)


@pytest.mark.gpu
def test_small_bst_prepare_equals_forward():
    """BSTModel.prepare: the bound one-launch forward (rk_bst_small_forward) equals the module's
    forward bit for bit, recomputes from the inputs' current contents, and keeps reading live
    images after a generation bump and a normal forward rebuild the caches (folded BatchNorm)."""
    cfg = {"T": 50, "heads": 4, "vocab": H.WECHAT_VOCAB}
    model = H.build("bst", cfg)
    H.randomize_eval_stats(model, 7)
    model = model.cuda().eval()
    d = H.to_device(H.make_inputs("bst", cfg, 3000, seed=11), "cuda")
    run = model.prepare(d["dense"], d["category"], d["seq_feedid"], d["seq_length"])
    with torch.no_grad():
        first = tuple(o.clone() for o in run())
        ref = H.as_tuple(H.call_model(model, "bst", d))
    for a, b in zip(first, ref):
        assert torch.equal(a, b)
    e = H.to_device(H.make_inputs("bst", cfg, 3000, seed=12), "cuda")
    d["dense"].copy_(e["dense"])
    d["seq_feedid"].copy_(e["seq_feedid"])
    d["seq_length"].copy_(e["seq_length"])
    for k in d["category"]:
        d["category"][k].copy_(e["category"][k])
    with torch.no_grad():
        b = tuple(o.clone() for o in run())
        ref = H.as_tuple(H.call_model(model, "bst", e))
    for x, y in zip(b, ref):
        assert torch.equal(x, y)
    model.eval()  # generation bump: the next forward refolds BatchNorm
    with torch.no_grad():
        H.call_model(model, "bst", e)
        scratch = [torch.randn(1 << 20, device="cuda") for _ in range(32)]  # reuse freed blocks
        again = run()
    torch.cuda.synchronize()
    for x, y in zip(b, again):
        assert torch.equal(x, y)
    del scratch


def test_small_bst_prepare_rejects_train_mode():
    """(CPU) prepare() is an eval-only binding."""
    model = H.build("bst", {"T": 8, "heads": 4})
    d = H.make_inputs("bst", {"T": 8, "heads": 4}, 16, seed=1)
    with pytest.raises(RuntimeError):
        model.train().prepare(d["dense"], d["category"], d["seq_feedid"], d["seq_length"])
