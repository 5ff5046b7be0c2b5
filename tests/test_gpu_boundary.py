"""The reference's standalone entry points called with the reference's own signatures, on the
HIP path, against the CPU oracle (atol = rtol = 1e-4, fp32):

  din_attention(query, keys, keys_length, is_softmax=False)          din.py:42-84
  Dice(num_features, eps=1e-9).forward(x)  (eval and train mode)      din.py:26-36
  BSTTransformer(d_model, nhead, max_len).forward(queries, keys, values, key_padding_mask=None)
                                                                      bst.py:42-91
"""
import pytest
import torch

import helpers as H
import rankops
from oracle import reference_forward as ref

ATOL = 1e-4
RTOL = 1e-4


def _close(got, expect, what=""):
    assert got.device.type == "cuda", f"{what}: not produced on the GPU"
    torch.testing.assert_close(got.detach().cpu(), expect, atol=ATOL, rtol=RTOL, equal_nan=True,
                               msg=lambda m: f"{what}: {m}")


# ------------------------------------------------------------------ din_attention

@pytest.mark.gpu
@pytest.mark.parametrize("H_,T", [(8, 5), (16, 13), (32, 50), (32, 64), (64, 33), (16, 77)])
@pytest.mark.parametrize("sm", [False, True])
def test_din_attention_reference_signature(H_, T, sm):
    g = torch.Generator().manual_seed(H_ * 100 + T)
    B = 67
    keys = torch.randn(B, T, H_, generator=g)
    query = torch.randn(B, H_, generator=g)
    lens = torch.randint(0, T + 1, (B,), generator=g)
    lens[:4] = torch.tensor([0, 1, T, min(T, 32)])
    torch.manual_seed(5)
    expect = ref.din_attention(query, keys, lens, sm)
    torch.manual_seed(5)  # the attention MLP is drawn from the CPU generator in the same order
    got = rankops.din_attention(query.cuda(), keys.cuda(), lens.cuda(), sm)
    _close(got, expect, f"din_attention H{H_} T{T} softmax={sm}")
    # the positional form and the default
    torch.manual_seed(5)
    got = rankops.din_attention(query.cuda(), keys.cuda(), lens.cuda())
    torch.manual_seed(5)
    _close(got, ref.din_attention(query, keys, lens, False), "din_attention default is_softmax")


@pytest.mark.gpu
def test_din_attention_strided_keys_and_lengths_beyond_T():
    """keys as a non-contiguous view (a slice of a wider tensor), lengths > T (all positions
    valid, as the reference's mask does), int32 lengths."""
    g = torch.Generator().manual_seed(9)
    B, T, Hd = 40, 21, 32
    wide = torch.randn(B, T, 2 * Hd, generator=g)
    keys = wide[:, :, Hd:]
    query = torch.randn(B, Hd, generator=g)
    lens = torch.randint(0, 2 * T, (B,), generator=g)
    for sm in (False, True):
        torch.manual_seed(21)
        expect = ref.din_attention(query, keys, lens, sm)
        torch.manual_seed(21)
        got = rankops.din_attention(query.cuda(), wide.cuda()[:, :, Hd:], lens.int().cuda(), sm)
        _close(got, expect, f"strided keys softmax={sm}")


@pytest.mark.gpu
def test_din_attention_frozen_weights_match_din_model_kernel():
    """With explicit weights the dense-keys entry equals the table-gather entry on the same rows."""
    g = torch.Generator().manual_seed(4)
    B, T, Hd = 100, 50, 32
    table = torch.randn(500, Hd, generator=g)
    seq = torch.randint(0, 500, (B, T), generator=g)
    lens = torch.randint(0, T + 1, (B,), generator=g)
    q = torch.randn(B, Hd, generator=g)
    w = [t.cuda() for t in ref.draw_din_att(Hd)]
    for sm in (False, True):
        a = rankops.din_attention(q.cuda(), table[seq].cuda(), lens.cuda(), sm, weights=w)
        b = rankops.din_attention_gather(q.cuda(), table.cuda(), seq.cuda(), lens.cuda(), sm, weights=w)
        torch.testing.assert_close(a, b, atol=1e-6, rtol=1e-6)


# ------------------------------------------------------------------ Dice

def _dice_params(dice):
    return {f"d.{k}": v.detach().cpu().clone() for k, v in dice.state_dict().items()}


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 32, 512, 300])
def test_dice_eval(n):
    torch.manual_seed(0)
    dice = rankops.Dice(n)
    H.randomize_eval_stats(dice, 3)
    dice.eval()
    x = torch.randn(129, n) * 2
    expect = ref.dice_eval(x, _dice_params(dice), "d.")
    dice = dice.cuda()
    with torch.no_grad():
        got = dice(x.cuda())
    _close(got, expect, f"Dice eval n={n}")


@pytest.mark.gpu
@pytest.mark.parametrize("n", [16, 256])
def test_dice_train_forward_backward(n):
    """Train mode: batch statistics, running statistics updated (momentum 0.1, unbiased
    variance), gradients w.r.t. x and alpha against torch autograd on the oracle."""
    torch.manual_seed(1)
    dice = rankops.Dice(n)
    H.randomize_eval_stats(dice, 5)
    dice.train()
    p = _dice_params(dice)
    x = torch.randn(300, n) * 1.5 + 0.3
    gy = torch.randn(300, n)
    xr = x.clone().requires_grad_(True)
    alpha = p["d.alpha"].clone().requires_grad_(True)
    p["d.alpha"] = alpha
    y_ref = ref.dice_train(xr, p, "d.")
    (y_ref * gy).sum().backward()

    dice = dice.cuda()
    xg = x.cuda().requires_grad_(True)
    y = dice(xg)
    (y * gy.cuda()).sum().backward()
    _close(y, y_ref.detach(), "Dice train forward")
    _close(xg.grad, xr.grad, "Dice dx")
    _close(dice.alpha.grad, alpha.grad, "Dice dalpha")
    _close(dice.bn.running_mean, p["d.bn.running_mean"], "running_mean")
    _close(dice.bn.running_var, p["d.bn.running_var"], "running_var")
    assert int(dice.bn.num_batches_tracked) == int(p["d.bn.num_batches_tracked"])
    # eval after the train step uses the updated running statistics
    dice.eval()
    with torch.no_grad():
        got = dice(x.cuda())
    p2 = _dice_params(dice.cpu())
    _close(got, ref.dice_eval(x, p2, "d."), "Dice eval after train")


# ------------------------------------------------------------------ BSTTransformer

def _block(d, nhead, max_len, seed):
    torch.manual_seed(seed)
    blk = rankops.BSTTransformer(d, nhead, max_len)
    H.randomize_eval_stats(blk, seed + 1)
    blk.eval()
    p = {f"b.{k}": v.detach().cpu().clone() for k, v in blk.state_dict().items()}
    return blk, p


@pytest.mark.gpu
@pytest.mark.parametrize("d,nhead,T", [(16, 4, 50), (128, 4, 64), (32, 2, 9), (64, 8, 20)])
@pytest.mark.parametrize("mask_kind", ["none", "lengths", "random"])
def test_bst_transformer_forward(d, nhead, T, mask_kind):
    blk, p = _block(d, nhead, T + 1, seed=d + T)
    g = torch.Generator().manual_seed(d * T)
    B = 37
    q = torch.randn(B, T, d, generator=g)
    k = torch.randn(B, T, d, generator=g)
    v = torch.randn(B, T, d, generator=g)
    if mask_kind == "none":
        mask = None
    elif mask_kind == "lengths":  # BSTModel's mask (bst.py:228-229), including an empty row -> NaN
        lens = torch.randint(1, T + 1, (B,), generator=g)
        lens[0] = 0
        mask = torch.arange(T).expand(B, T) >= lens.unsqueeze(1)
    else:  # an arbitrary padding mask, one row fully masked and one unmasked
        mask = torch.rand(B, T, generator=g) < 0.4
        mask[1] = True
        mask[2] = False
    expect = ref.bst_block(p, "b.", q, k, v, nhead, mask)
    blk = blk.cuda()
    m = mask.cuda() if mask is not None else None
    with torch.no_grad():
        got = blk(q.cuda(), k.cuda(), v.cuda(), m)
        _close(got, expect, f"BSTTransformer d{d} h{nhead} T{T} mask={mask_kind}")
        # keyword form and self-attention (q = k = v: the packed [W_q; W_k] GEMM)
        got = blk(queries=q.cuda(), keys=q.cuda(), values=q.cuda(), key_padding_mask=m)
        _close(got, ref.bst_block(p, "b.", q, q, q, nhead, mask), "self-attention, keywords")
        x = q.cuda()
        got = blk(x, x, x, m)
        _close(got, ref.bst_block(p, "b.", q, q, q, nhead, mask), "self-attention, one tensor")


@pytest.mark.gpu
def test_bst_transformer_stacked_like_bstmodel():
    """Two blocks chained the way BSTModel.forward chains them (bst.py:230-236) equal the oracle."""
    d, nhead, T, B = 16, 4, 30, 25
    b1, p1 = _block(d, nhead, 51, 1)
    b2, p2 = _block(d, nhead, 51, 2)
    g = torch.Generator().manual_seed(8)
    x = torch.randn(B, T, d, generator=g)
    lens = torch.randint(1, T + 1, (B,), generator=g)
    mask = torch.arange(T).expand(B, T) >= lens.unsqueeze(1)
    e = ref.bst_block(p1, "b.", x, x, x, nhead, mask)
    e = ref.bst_block(p2, "b.", e, e, e, nhead, mask)
    b1, b2 = b1.cuda(), b2.cuda()
    with torch.no_grad():
        y = b1(x.cuda(), x.cuda(), x.cuda(), mask.cuda())
        y = b2(y, y, y, mask.cuda())
    _close(y, e, "two stacked blocks")


@pytest.mark.gpu
def test_bst_transformer_errors():
    blk, _ = _block(16, 4, 10, 0)
    blk = blk.cuda()
    x = torch.randn(2, 11, 16, device="cuda")
    with pytest.raises(IndexError):
        blk(x, x, x)
    x = torch.randn(2, 5, 16, device="cuda")
    with pytest.raises(ValueError):
        blk(x, x, x, torch.zeros(2, 5, device="cuda"))  # float mask: the reference needs bool
    blk.train()
    with pytest.raises(NotImplementedError):
        blk(x, x, x)
