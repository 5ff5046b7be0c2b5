"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py) — parity unpinned.

Independent float64 numpy restatement of the same reference forwards as
`reference_forward` (no torch ops), used to cross-check that restatement: two codings of
the cited reference lines that agree to ~1e-6 cannot share an op-order or masking mistake.
Parameters come as a dict of numpy arrays keyed like the reference state_dict; the H2
per-call layers are passed in explicitly (drawn by `reference_forward.draw_*`).
"""
from __future__ import annotations

import numpy as np

EPS_BN = 1e-5


def _f(p, k):
    return np.asarray(p[k], dtype=np.float64)


def _lin(x, p, prefix):
    return x @ _f(p, prefix + "weight").T + _f(p, prefix + "bias")


def _bn(x, p, prefix, affine=True):
    y = (x - _f(p, prefix + "running_mean")) / np.sqrt(_f(p, prefix + "running_var") + EPS_BN)
    if affine:
        y = y * _f(p, prefix + "weight") + _f(p, prefix + "bias")
    return y


def _relu(x):
    return np.maximum(x, 0.0)


def _sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def _emb(p, key, idx):
    return _f(p, key)[np.asarray(idx)]


def _softmax(x, axis):
    m = np.max(x, axis=axis, keepdims=True)
    e = np.exp(x - m)
    return e / np.sum(e, axis=axis, keepdims=True)


FIELDS6 = ["userid", "device", "authorid", "bgm_song_id", "bgm_singer_id", "manual_tag_list"]


def dcn(p, dense, category, cross, num_hidden):
    """dcn.py:161-180 with cross = [(w (d,1), b (d,1))]."""
    x0 = np.concatenate([np.asarray(dense, np.float64)] + [_emb(p, f"embeddings.{c}.weight", category[c])
                                                          for c in FIELDS6], axis=1)
    xl = x0
    for w, b in cross:
        xl = x0 * (xl @ np.asarray(w, np.float64)) + np.asarray(b, np.float64).T + xl
    h = x0
    for i in range(num_hidden):
        h = _relu(_lin(h, p, f"dnn.{2 * i}."))
    logit = _lin(np.concatenate([xl, h], 1), p, "output_layer.")
    return _sigmoid(logit), logit


def deepfm(p, category, fields, layout):
    """deepfm.py:121-151; layout = [(linear_idx, bn_idx or None)]."""
    e1 = np.stack([_emb(p, f"first_order_embeddings.{c}.weight", category[c])[:, 0] for c in fields], 1)
    fm1 = e1.sum(1, keepdims=True)
    e2 = np.stack([_emb(p, f"second_order_embeddings.{c}.weight", category[c]) for c in fields], 1)
    s = e2.sum(1)
    fm2 = 0.5 * (s * s - (e2 * e2).sum(1)).sum(1, keepdims=True)
    h = e2.reshape(e2.shape[0], -1)
    for lin, bn in layout:
        h = _lin(h, p, f"deep_layers.{lin}.")
        if bn is not None:
            h = _bn(h, p, f"deep_layers.{bn}.")
        h = _relu(h)
    deep = _lin(h, p, "deep_output_layer.")
    total = _lin(np.concatenate([fm1, fm2, deep], 1), p, "final_layer.")
    return _sigmoid(total), total, fm1, fm2, deep


def din_attention(q, keys, lengths, softmax, att):
    w1, b1, w2, b2, w3, b3 = [np.asarray(t, np.float64) for t in att]
    B, T, H = keys.shape
    qe = np.broadcast_to(q[:, None, :], keys.shape)
    cross = np.concatenate([qe, keys, qe - keys, qe * keys], 2)
    h = _relu(cross @ w1.T + b1)
    h = _relu(h @ w2.T + b2)
    s = (h @ w3.T + b3)[..., 0]
    mask = np.arange(T)[None, :] < np.asarray(lengths)[:, None]
    if softmax:
        s = np.where(mask, s, float(np.float32(-2 ** 32 + 1))) / np.sqrt(H)
        w = _softmax(s, 1)
    else:
        w = np.where(mask, s, 0.0)
    return (w[:, :, None] * keys).sum(1)


def din(p, dense, category, sequence, target, layout, activation, softmax, l2_lambda, att):
    """din.py:294-323; layout = [(linear_idx, act_idx, bn_idx or None)]."""
    dense_in = np.stack([np.asarray(v, np.float64) for v in dense.values()], 1)
    cat = [_emb(p, f"embeddings.{c}.weight", category[c]) for c in FIELDS6 if c in category]
    tgt = _emb(p, "embeddings.feedid.weight", target["feedid"])
    keys = _emb(p, "embeddings.his_read_comment_7d_seq.weight", sequence["his_read_comment_7d_seq"])
    att_out = din_attention(tgt, keys, sequence["his_read_comment_7d_seq_length"], softmax, att)
    net = np.concatenate([dense_in] + cat + [tgt, att_out], 1)
    for lin, act, bn in layout:
        net = _lin(net, p, f"fcn.{lin}.")
        if activation == "dice":
            xp = _sigmoid(_bn(net, p, f"fcn.{act}.bn.", affine=False))
            alpha = _f(p, f"fcn.{act}.alpha")
            net = alpha * (1.0 - xp) * net + xp * net
        else:
            a = _f(p, f"fcn.{act}.weight")
            net = np.where(net > 0, net, a * net)
        if bn is not None:
            net = _bn(net, p, f"fcn.{bn}.")
    logit = _lin(net, p, "output_layer.")
    l2 = 0.0
    if l2_lambda > 0:
        ev = np.concatenate(cat + [tgt, att_out], 1)
        l2 = l2_lambda * np.sqrt((ev * ev).sum(1)).mean()
    return _sigmoid(logit), logit, l2


def afm(p, dense, category, fields):
    """afm.py:92-119."""
    dl = _lin(np.asarray(dense, np.float64), p, "dense_layer.")
    e = [_emb(p, f"embeddings.{c}.weight", category[c]) for c in fields]
    pairs = np.stack([e[i] * e[j] for i in range(len(e)) for j in range(i + 1, len(e))], 1)
    score = _lin(_relu(_lin(pairs, p, "attention.0.")), p, "attention.2.")
    w = _softmax(score, 1)
    logit = dl + _lin((pairs * w).sum(1), p, "p.")
    return _sigmoid(logit), logit


def deepcrossing(p, dense, category, units):
    """deepcrossing.py:146-163 with units = [(w1, b1, w2, b2)]."""
    x = np.concatenate([np.asarray(dense, np.float64)] + [_emb(p, f"embeddings.{c}.weight", category[c])
                                                         for c in FIELDS6], 1)
    for w1, b1, w2, b2 in units:
        w1, b1, w2, b2 = [np.asarray(t, np.float64) for t in (w1, b1, w2, b2)]
        x = _relu(x + (_relu(x @ w1.T + b1) @ w2.T + b2))
    logit = _lin(x, p, "output_layer.")
    return _sigmoid(logit), logit


def _ln(x, g, b):
    m = x.mean(-1, keepdims=True)
    v = ((x - m) ** 2).mean(-1, keepdims=True)
    return (x - m) / np.sqrt(v + 1e-5) * g + b


def bst_block(p, pre, x, lengths, nhead):
    B, T, d = x.shape
    pos = _f(p, pre + "position_embedding.weight")[:T][None]
    qk_in = x + pos
    q = _lin(qk_in, p, pre + "w_q.").reshape(B, T, nhead, -1).transpose(0, 2, 1, 3)
    k = _lin(qk_in, p, pre + "w_k.").reshape(B, T, nhead, -1).transpose(0, 2, 1, 3)
    v = _lin(x, p, pre + "w_v.").reshape(B, T, nhead, -1).transpose(0, 2, 1, 3)
    s = q @ k.transpose(0, 1, 3, 2) / np.sqrt(q.shape[-1])
    pad = np.arange(T)[None, :] >= np.asarray(lengths)[:, None]
    s = np.where(pad[:, None, None, :], -np.inf, s)
    with np.errstate(invalid="ignore"):
        a = _softmax(s, -1)
    ctx = (a @ v).transpose(0, 2, 1, 3).reshape(B, T, d)
    o1 = _ln(qk_in + _lin(ctx, p, pre + "w_o."), _f(p, pre + "norm1.weight"), _f(p, pre + "norm1.bias"))
    f = _lin(o1, p, pre + "ffn.0.")
    f = np.where(f > 0, f, 0.01 * f)
    return _ln(o1 + _lin(f, p, pre + "ffn.3."), _f(p, pre + "norm2.weight"), _f(p, pre + "norm2.bias"))


def bst(p, dense, category, seq, lengths, nhead, num_blocks, layout, last, pooling="sum"):
    """bst.py:216-247; layout = [(linear_idx, bn_idx or None)], last = index of the final Linear."""
    cat = np.concatenate([_emb(p, f"embeddings.{c}.weight", category[c]) for c in FIELDS6], 1)
    x = _emb(p, "embeddings.feedid.weight", seq)
    for i in range(num_blocks):
        x = bst_block(p, f"transformer_blocks.{i}.", x, lengths, nhead)
    pooled = x.sum(1)
    if pooling != "sum":
        pooled = pooled / np.asarray(lengths, np.float64)[:, None]
    h = np.concatenate([np.asarray(dense, np.float64), cat, pooled], 1)
    for lin, bn in layout:
        h = _lin(h, p, f"dnn.{lin}.")
        if bn is not None:
            h = _bn(h, p, f"dnn.{bn}.")
        h = np.where(h > 0, h, 0.01 * h)
    logit = _lin(h, p, f"dnn.{last}.")
    return _sigmoid(logit), logit
