"""GPU: the d-128 BST blocks on pre-packed projection weights (rk_bst_pack_block_weight +
rk_bst_forward_blocks_packed, round 6).  The packed layout only changes where the block kernel's
weight loads read from, so the pooled rows must equal the unpacked entry point's bit for bit; the
model forward keeps its packed images in step with in-place weight updates (bst.py:66-91,224-241)."""
import pytest
import torch

import helpers as H
from rankops import _lib, ops

RK_ERR_INVALID = 1  # include/rankops.h


def _torch_pack(w):
    # the header's formula: float 4096 j + 1024 g + 256 c + 4 l + e = W[32 j + l % 32][32 g + 8 c + 4 (l / 32) + e]
    return w.view(4, 32, 4, 4, 2, 4).permute(0, 2, 3, 4, 1, 5).contiguous().view(128, 128)


@pytest.mark.gpu
def test_pack_block_weight_layout():
    torch.manual_seed(0)
    w = torch.randn(128, 128, device="cuda")
    got = ops.pack_bst_weight(w)
    torch.cuda.synchronize()
    assert torch.equal(got, _torch_pack(w))
    # rewritten in place into a previous image
    w2 = torch.randn(128, 128, device="cuda")
    again = ops.pack_bst_weight(w2, out=got)
    torch.cuda.synchronize()
    assert again.data_ptr() == got.data_ptr() and torch.equal(again, _torch_pack(w2))


@pytest.mark.gpu
def test_pack_block_weight_rejects_in_place_and_misaligned():
    lib = _lib.load()
    w = torch.randn(128 * 128 + 4, device="cuda")
    assert lib.rk_bst_pack_block_weight(w.data_ptr(), w.data_ptr(), None) == RK_ERR_INVALID
    assert lib.rk_bst_pack_block_weight(w.data_ptr() + 4, w.data_ptr() + 4 * 16400, None) == RK_ERR_INVALID


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [{"T": 64, "dim": 128, "max_len": 64}, {"T": 37, "dim": 128, "blocks": 2, "max_len": 40},
                                 {"T": 50, "dim": 128, "pooling": "mean"}], ids=str)
def test_packed_entry_equals_unpacked(cfg):
    model = H.build("bst", cfg).cuda().eval()
    B = 600  # > 256 CUs: the persistent loop walks a second and third sample
    inp = H.to_device(H.make_inputs("bst", cfg, B, seed=5), "cuda")
    inp["seq_length"][:2] = 0
    inp["seq_length"][2:5] = 1
    inp["seq_length"][5:8] = cfg["T"]
    seq = ops.bound_index(inp["seq_feedid"], "seq", contiguous=True)
    sl = ops.bound_index(inp["seq_length"], "len")
    blocks = model._fused_blocks(cfg["T"])
    assert blocks is not None
    mean = cfg.get("pooling") == "mean"
    tab = model.embeddings["feedid"].weight
    rows = {}
    for packed in (False, True):
        r = torch.full((B, 136), 7.0, device="cuda")
        blk = model._packed_blocks(blocks) if packed else blocks
        ops.bst_forward_blocks(tab, seq, sl, 128, 4, blk, _lib.fptr(r, 4), 136, mean, packed=packed)
        rows[packed] = r
    torch.cuda.synchronize()
    a, b = rows[False], rows[True]
    assert torch.equal(torch.isnan(a), torch.isnan(b))
    assert torch.equal(torch.nan_to_num(a), torch.nan_to_num(b))
    assert (a[:, :4] == 7.0).all() and (a[:, 132:] == 7.0).all()  # only the pooled columns written
    assert torch.isnan(a[:2, 4:132]).all()  # length 0: NaN, as torch's softmax over all -inf


@pytest.mark.gpu
def test_packed_entry_rejects_d16():
    cfg = {"T": 20}
    model = H.build("bst", cfg).cuda().eval()
    inp = H.to_device(H.make_inputs("bst", cfg, 8), "cuda")
    blocks = model._fused_blocks(20)
    r = torch.zeros(8, 16, device="cuda")
    with pytest.raises(RuntimeError, match="rk_bst_forward_blocks_packed"):
        ops.bst_forward_blocks(model.embeddings["feedid"].weight, inp["seq_feedid"], inp["seq_length"], 16, 4,
                               blocks, _lib.fptr(r, 0), 16, False, packed=True)


@pytest.mark.gpu
def test_forward_follows_in_place_weight_updates():
    """An optimizer-style in-place update of a projection weight bumps its version: the next eval
    forward repacks it (common.BST_PACKED) and still matches the oracle."""
    cfg = {"T": 40, "dim": 128, "max_len": 64}
    B = 64
    inp = H.make_inputs("bst", cfg, B, seed=9)
    model = H.build("bst", cfg).cuda().eval()
    dev_inp = H.to_device(inp, "cuda")
    with torch.no_grad():
        first = H.call_model(model, "bst", dev_inp)
        blk = model.transformer_blocks[0]
        for lin in (blk.w_q, blk.w_v, blk.ffn[3]):
            lin.weight.mul_(1.5)
        second = H.call_model(model, "bst", dev_inp)
    torch.cuda.synchronize()
    assert not torch.allclose(first[1], second[1])
    with torch.no_grad():
        ref = H.call_oracle("bst", cfg, H.cpu_params(model), inp)
    for o, r in zip(H.as_tuple(second), H.as_tuple(ref)):
        torch.testing.assert_close(o.cpu(), r, atol=1e-4, rtol=1e-4, equal_nan=True)
