"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py) — parity unpinned.

CPU fp32 restatement of the reference eval forwards, written against the cited reference
lines (paths relative to the reference snapshot).  Every function works on a parameter
dict `p` keyed exactly like the reference `state_dict`, so a rankops module's
`state_dict()` can be fed in unchanged.  Eval semantics throughout: BatchNorm uses running
statistics, Dropout is identity (the `evaluate()` loops, e.g. dcn.py:214-239).

Per-call random layers (reference hazard H2) are drawn with the same torch.nn.init /
nn.Linear calls, in the same order, from the default CPU generator (`draw_*`).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

DCN_FIELDS = ["userid", "device", "authorid", "bgm_song_id", "bgm_singer_id", "manual_tag_list"]


# ---------------------------------------------------------------------------- H2 draws

def draw_cross(d: int, num_layers: int):
    """dcn.py:37-41 — per layer: wl = zeros(d,1), bl = zeros(d,1), xavier_normal_(wl), zeros_(bl)."""
    out = []
    for _ in range(num_layers):
        wl = nn.Parameter(torch.zeros(d, 1), requires_grad=True)
        bl = nn.Parameter(torch.zeros(d, 1), requires_grad=True)
        nn.init.xavier_normal_(wl)
        nn.init.zeros_(bl)
        out.append((wl.detach(), bl.detach()))
    return out


def draw_din_att(embedding_dim: int):
    """din.py:61-67 — nn.Sequential(Linear(4H,64), ReLU, Linear(64,32), ReLU, Linear(32,1))."""
    net = nn.Sequential(nn.Linear(4 * embedding_dim, 64), nn.ReLU(), nn.Linear(64, 32), nn.ReLU(),
                        nn.Linear(32, 1))
    return [t.detach() for t in (net[0].weight, net[0].bias, net[2].weight, net[2].bias, net[4].weight,
                                 net[4].bias)]


def draw_residual(d: int, internal_dim: int):
    """deepcrossing.py:37-39 — Linear(d, I) is built (and applied) before Linear(I, d)."""
    a = nn.Linear(d, internal_dim)
    b = nn.Linear(internal_dim, d)
    return [t.detach() for t in (a.weight, a.bias, b.weight, b.bias)]


# ---------------------------------------------------------------------------- shared pieces

def _bn_eval(x, p, prefix, affine=True, eps=1e-5):
    return F.batch_norm(x, p[prefix + "running_mean"], p[prefix + "running_var"],
                        p[prefix + "weight"] if affine else None, p[prefix + "bias"] if affine else None,
                        training=False, momentum=0.0, eps=eps)


def _lin(x, p, prefix):
    return F.linear(x, p[prefix + "weight"], p[prefix + "bias"])


def _cat_fields(p, category, fields, prefix="embeddings."):
    return [F.embedding(category[c], p[f"{prefix}{c}.weight"]) for c in fields if c in category]


# ---------------------------------------------------------------------------- DCN

def dcn_cross_layer(x0, xl, wl, bl):
    """dcn.py:47-49."""
    xl_wl = torch.matmul(xl, wl)
    x0_xl_wl = torch.mul(x0, xl_wl)
    return x0_xl_wl + bl.t() + xl


def dcn_forward(p, dense, category, num_cross_layer=1, num_hidden=3, cross=None):
    """DCNModel.forward, dcn.py:161-180.  `cross` = list of (w (d,1), b (d,1)); drawn per call
    when None."""
    emb = torch.cat(_cat_fields(p, category, DCN_FIELDS), dim=1)
    concat_all = torch.cat([dense, emb], dim=1)
    if cross is None:
        cross = draw_cross(concat_all.shape[-1], num_cross_layer)
    cross_vec = concat_all
    for wl, bl in cross:
        cross_vec = dcn_cross_layer(concat_all, cross_vec, wl, bl)
    h = concat_all
    for i in range(num_hidden):
        h = torch.relu(_lin(h, p, f"dnn.{2 * i}."))
    logit = _lin(torch.cat([cross_vec, h], dim=1), p, "output_layer.")
    return torch.sigmoid(logit), logit


# ---------------------------------------------------------------------------- DeepFM

def deepfm_layout(num_hidden, batch_norm=True, dropout_rate=0.1):
    """Module indices of deep_layers (deepfm.py:100-109): per unit Linear, [BN], ReLU, [Dropout]."""
    idx, out = 0, []
    for _ in range(num_hidden):
        lin = idx
        idx += 1
        bn = None
        if batch_norm:
            bn = idx
            idx += 1
        idx += 1  # ReLU
        if dropout_rate > 0:
            idx += 1
        out.append((lin, bn))
    return out


def deepfm_forward(p, category, fields, num_hidden=3, batch_norm=True, dropout_rate=0.1):
    """DeepFM.forward, deepfm.py:121-151."""
    first = [F.embedding(category[c], p[f"first_order_embeddings.{c}.weight"]) for c in fields if c in category]
    fm_first = torch.sum(torch.cat(first, dim=1), dim=1, keepdim=True)
    second = [F.embedding(category[c], p[f"second_order_embeddings.{c}.weight"]) for c in fields if c in category]
    sum_embedding = torch.sum(torch.stack(second, dim=1), dim=1)
    sum_embedding_square = torch.square(sum_embedding)
    square_sum_embedding = torch.sum(torch.stack([torch.square(e) for e in second], dim=1), dim=1)
    fm_second = 0.5 * torch.sum(sum_embedding_square - square_sum_embedding, dim=1, keepdim=True)
    h = torch.cat(second, dim=1)
    for lin, bn in deepfm_layout(num_hidden, batch_norm, dropout_rate):
        h = _lin(h, p, f"deep_layers.{lin}.")
        if bn is not None:
            h = _bn_eval(h, p, f"deep_layers.{bn}.")
        h = torch.relu(h)
    deep_logit = _lin(h, p, "deep_output_layer.")
    total = _lin(torch.cat([fm_first, fm_second, deep_logit], dim=1), p, "final_layer.")
    return torch.sigmoid(total), total, fm_first, fm_second, deep_logit


def deepfm_forward_train(p, category, fields, num_hidden=3, batch_norm=True, dropout_rate=0.1, masks=None,
                         momentum=0.1, eps=1e-5):
    """DeepFM.forward in model.train() (deepfm.py:121-151): BatchNorm1d with batch statistics
    (running_mean / running_var in `p` updated in place, num_batches_tracked += 1), Dropout as the
    given per-unit multiplier masks (0 or 1/(1-p)); differentiable w.r.t. the tensors in `p`."""
    first = [F.embedding(category[c], p[f"first_order_embeddings.{c}.weight"]) for c in fields if c in category]
    fm_first = torch.sum(torch.cat(first, dim=1), dim=1, keepdim=True)
    second = [F.embedding(category[c], p[f"second_order_embeddings.{c}.weight"]) for c in fields if c in category]
    sum_embedding = torch.sum(torch.stack(second, dim=1), dim=1)
    sum_embedding_square = torch.square(sum_embedding)
    square_sum_embedding = torch.sum(torch.stack([torch.square(e) for e in second], dim=1), dim=1)
    fm_second = 0.5 * torch.sum(sum_embedding_square - square_sum_embedding, dim=1, keepdim=True)
    h = torch.cat(second, dim=1)
    for u, (lin, bn) in enumerate(deepfm_layout(num_hidden, batch_norm, dropout_rate)):
        h = _lin(h, p, f"deep_layers.{lin}.")
        if bn is not None:
            pre = f"deep_layers.{bn}."
            h = F.batch_norm(h, p[pre + "running_mean"], p[pre + "running_var"], p[pre + "weight"], p[pre + "bias"],
                             training=True, momentum=momentum, eps=eps)
            p[pre + "num_batches_tracked"] += 1
        h = torch.relu(h)
        if masks is not None and masks[u] is not None:
            h = h * masks[u]
    deep_logit = _lin(h, p, "deep_output_layer.")
    total = _lin(torch.cat([fm_first, fm_second, deep_logit], dim=1), p, "final_layer.")
    return torch.sigmoid(total), total, fm_first, fm_second, deep_logit


# ---------------------------------------------------------------------------- DIN

def dice_eval(x, p, prefix):
    """Dice.forward, din.py:33-36 (BatchNorm1d(affine=False) eval)."""
    x_normed = _bn_eval(x, p, prefix + "bn.", affine=False)
    x_p = torch.sigmoid(x_normed)
    return p[prefix + "alpha"] * (1.0 - x_p) * x + x_p * x


def din_attention(query, keys, keys_length, is_softmax=False, att=None):
    """din_attention, din.py:42-84; `att` = (W1, b1, W2, b2, W3, b3), drawn per call when None."""
    batch_size, max_length, embedding_dim = keys.size()
    if att is None:
        att = draw_din_att(embedding_dim)
    w1, b1, w2, b2, w3, b3 = att
    query = query.unsqueeze(1).expand_as(keys)
    cross = torch.cat([query, keys, query - keys, query * keys], dim=2)
    h = torch.relu(F.linear(cross, w1, b1))
    h = torch.relu(F.linear(h, w2, b2))
    att_score = F.linear(h, w3, b3).squeeze(2)
    mask = torch.arange(max_length).expand(batch_size, max_length) < keys_length.unsqueeze(1)
    if is_softmax:
        paddings = torch.ones_like(att_score) * (-2 ** 32 + 1)
        att_score = torch.where(mask, att_score, paddings)
        att_score = att_score / (embedding_dim ** 0.5)
        att_weight = torch.softmax(att_score, dim=1)
    else:
        att_weight = att_score.masked_fill(~mask, 0.0)
    return torch.sum(att_weight.unsqueeze(2) * keys, dim=1)


def din_layout(num_hidden, activation="dice", batch_norm=True, dropout_rate=0.1):
    """Module indices of fcn (din.py:272-284): Linear, Dice|PReLU, [BN], [Dropout]."""
    idx, out = 0, []
    for _ in range(num_hidden):
        lin, act = idx, idx + 1
        idx += 2
        bn = None
        if batch_norm:
            bn = idx
            idx += 1
        if dropout_rate > 0:
            idx += 1
        out.append((lin, act, bn))
    return out


DIN_EMB = ["userid", "device", "authorid", "bgm_song_id", "bgm_singer_id", "manual_tag_list", "feedid",
           "his_read_comment_7d_seq"]


def din_forward(p, dense, category, sequence, target, num_hidden=3, activation="dice", batch_norm=True,
                dropout_rate=0.1, use_softmax=False, l2_lambda=0.2, mini_batch_aware_regularization=True,
                att=None):
    """DIN.forward, din.py:294-323."""
    dense_input = torch.cat([dense[c].unsqueeze(1) for c in dense], dim=1)
    category_emb = [F.embedding(category[c], p[f"embeddings.{c}.weight"]) for c in DIN_EMB if c in category]
    target_feed_emb = F.embedding(target["feedid"], p["embeddings.feedid.weight"])
    seq_emb = F.embedding(sequence["his_read_comment_7d_seq"], p["embeddings.his_read_comment_7d_seq.weight"])
    seq_length = sequence["his_read_comment_7d_seq_length"]
    attention_output = din_attention(target_feed_emb, seq_emb, seq_length, use_softmax, att)
    net = torch.cat([dense_input] + category_emb + [target_feed_emb, attention_output], dim=1)
    for lin, act, bn in din_layout(num_hidden, activation, batch_norm, dropout_rate):
        net = _lin(net, p, f"fcn.{lin}.")
        if activation == "dice":
            net = dice_eval(net, p, f"fcn.{act}.")
        else:
            net = F.prelu(net, p[f"fcn.{act}.weight"])
        if bn is not None:
            net = _bn_eval(net, p, f"fcn.{bn}.")
    logit = _lin(net, p, "output_layer.")
    probability = torch.sigmoid(logit)
    l2_reg = 0.0
    if mini_batch_aware_regularization and l2_lambda > 0:
        embedding_vars = torch.cat([torch.cat(category_emb, dim=1), target_feed_emb, attention_output], dim=1)
        l2_reg = l2_lambda * torch.norm(embedding_vars, p=2, dim=1).mean()
    return probability, logit, l2_reg


def dice_train(x, p, prefix, momentum=0.1, eps=1e-5):
    """Dice.forward in model.train() (din.py:33-36): its BatchNorm1d(affine=False) normalises with the
    batch statistics and updates the running statistics held in `p`."""
    pre = prefix + "bn."
    x_normed = F.batch_norm(x, p[pre + "running_mean"], p[pre + "running_var"], None, None, training=True,
                            momentum=momentum, eps=eps)
    p[pre + "num_batches_tracked"] += 1
    x_p = torch.sigmoid(x_normed)
    return p[prefix + "alpha"] * (1.0 - x_p) * x + x_p * x


def din_forward_train(p, dense, category, sequence, target, num_hidden=3, batch_norm=True, dropout_rate=0.1,
                      use_softmax=False, l2_lambda=0.2, mini_batch_aware_regularization=True, att=None, masks=None,
                      momentum=0.1, eps=1e-5, activation="dice"):
    """DIN.forward in model.train() (din.py:294-323): Dice (or nn.PReLU with activation='prelu',
    din.py:275-279) and BatchNorm1d with batch statistics (running statistics in `p` updated in
    place), Dropout as the given per-unit multiplier masks (0 or 1/(1-p)); differentiable w.r.t. the
    tensors in `p`."""
    dense_input = torch.cat([dense[c].unsqueeze(1) for c in dense], dim=1)
    category_emb = [F.embedding(category[c], p[f"embeddings.{c}.weight"]) for c in DIN_EMB if c in category]
    target_feed_emb = F.embedding(target["feedid"], p["embeddings.feedid.weight"])
    seq_emb = F.embedding(sequence["his_read_comment_7d_seq"], p["embeddings.his_read_comment_7d_seq.weight"])
    seq_length = sequence["his_read_comment_7d_seq_length"]
    attention_output = din_attention(target_feed_emb, seq_emb, seq_length, use_softmax, att)
    net = torch.cat([dense_input] + category_emb + [target_feed_emb, attention_output], dim=1)
    for u, (lin, act, bn) in enumerate(din_layout(num_hidden, activation, batch_norm, dropout_rate)):
        net = _lin(net, p, f"fcn.{lin}.")
        if activation == "dice":
            net = dice_train(net, p, f"fcn.{act}.", momentum, eps)
        else:
            net = F.prelu(net, p[f"fcn.{act}.weight"])
        if bn is not None:
            pre = f"fcn.{bn}."
            net = F.batch_norm(net, p[pre + "running_mean"], p[pre + "running_var"], p[pre + "weight"],
                               p[pre + "bias"], training=True, momentum=momentum, eps=eps)
            p[pre + "num_batches_tracked"] += 1
        if masks is not None and masks[u] is not None:
            net = net * masks[u]
    logit = _lin(net, p, "output_layer.")
    probability = torch.sigmoid(logit)
    l2_reg = 0.0
    if mini_batch_aware_regularization and l2_lambda > 0:
        embedding_vars = torch.cat([torch.cat(category_emb, dim=1), target_feed_emb, attention_output], dim=1)
        l2_reg = l2_lambda * torch.norm(embedding_vars, p=2, dim=1).mean()
    return probability, logit, l2_reg


# ---------------------------------------------------------------------------- AFM

def afm_forward(p, dense_input, category_input, category_features):
    """AFM.forward, afm.py:92-119."""
    dense_logit = _lin(dense_input, p, "dense_layer.")
    embs = [F.embedding(category_input[c], p[f"embeddings.{c}.weight"]) for c in category_features]
    pairs = []
    n = len(embs)
    for i in range(n):
        for j in range(i + 1, n):
            pairs.append(torch.mul(embs[i], embs[j]))
    pairs = torch.stack(pairs, dim=1)
    scores = _lin(torch.relu(_lin(pairs, p, "attention.0.")), p, "attention.2.")
    weights = torch.softmax(scores, dim=1)
    weighted_sum = torch.sum(pairs * weights, dim=1)
    afm_logit = _lin(weighted_sum, p, "p.")
    total = dense_logit + afm_logit
    return torch.sigmoid(total), total


# ---------------------------------------------------------------------------- DeepCrossing

def residual_unit(x, w1, b1, w2, b2):
    """deepcrossing.py:37-41."""
    h = torch.relu(F.linear(x, w1, b1))
    h = F.linear(h, w2, b2)
    return torch.relu(x + h)


def deepcrossing_forward(p, dense, category, residual_internal_dim=128, residual_network_num=1, units=None):
    """DeepCrossingModel.forward, deepcrossing.py:146-163; `units` drawn per call when None."""
    emb = torch.cat(_cat_fields(p, category, DCN_FIELDS), dim=1)
    net = torch.cat([dense, emb], dim=1)
    for i in range(residual_network_num):
        if units is None:
            w = draw_residual(net.shape[-1], residual_internal_dim)
        else:
            w = units[i]
        net = residual_unit(net, *w)
    logit = _lin(net, p, "output_layer.")
    return torch.sigmoid(logit), logit


# ---------------------------------------------------------------------------- BST

def bst_block(p, prefix, queries, keys, values, nhead, key_padding_mask=None, eps=1e-5):
    """BSTTransformer.forward, bst.py:66-91."""
    batch_size, seq_len, d_model = queries.size()
    pos_indices = torch.arange(seq_len).expand(batch_size, -1)
    pos = F.embedding(pos_indices, p[prefix + "position_embedding.weight"])
    queries = queries + pos
    keys = keys + pos
    q = _lin(queries, p, prefix + "w_q.").view(batch_size, seq_len, nhead, -1).transpose(1, 2)
    k = _lin(keys, p, prefix + "w_k.").view(batch_size, seq_len, nhead, -1).transpose(1, 2)
    v = _lin(values, p, prefix + "w_v.").view(batch_size, seq_len, nhead, -1).transpose(1, 2)
    scores = torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(q.size(-1))
    if key_padding_mask is not None:
        scores = scores.masked_fill(key_padding_mask.unsqueeze(1).unsqueeze(2), float("-inf"))
    attn = F.softmax(scores, dim=-1)
    context = torch.matmul(attn, v).transpose(1, 2).contiguous().view(batch_size, seq_len, -1)
    out1 = F.layer_norm(queries + _lin(context, p, prefix + "w_o."), (d_model,), p[prefix + "norm1.weight"],
                        p[prefix + "norm1.bias"], eps)
    ffn = _lin(F.leaky_relu(_lin(out1, p, prefix + "ffn.0."), 0.01), p, prefix + "ffn.3.")
    return F.layer_norm(out1 + ffn, (d_model,), p[prefix + "norm2.weight"], p[prefix + "norm2.bias"], eps)


def bst_block_train(p, prefix, queries, keys, values, nhead, key_padding_mask=None, masks=None, eps=1e-5):
    """BSTTransformer.forward in model.train() (bst.py:66-91): the three Dropout sites as given
    multiplier masks [B*T, d] (w_o output, inside the FFN, FFN output), or identity when None."""
    batch_size, seq_len, d_model = queries.size()

    def drop(t, k):
        if masks is None or masks[k] is None:
            return t
        return t * masks[k].view(batch_size, seq_len, d_model)

    pos_indices = torch.arange(seq_len).expand(batch_size, -1)
    pos = F.embedding(pos_indices, p[prefix + "position_embedding.weight"])
    queries = queries + pos
    keys = keys + pos
    q = _lin(queries, p, prefix + "w_q.").view(batch_size, seq_len, nhead, -1).transpose(1, 2)
    k = _lin(keys, p, prefix + "w_k.").view(batch_size, seq_len, nhead, -1).transpose(1, 2)
    v = _lin(values, p, prefix + "w_v.").view(batch_size, seq_len, nhead, -1).transpose(1, 2)
    scores = torch.matmul(q, k.transpose(-2, -1)) / math.sqrt(q.size(-1))
    if key_padding_mask is not None:
        scores = scores.masked_fill(key_padding_mask.unsqueeze(1).unsqueeze(2), float("-inf"))
    attn = F.softmax(scores, dim=-1)
    context = torch.matmul(attn, v).transpose(1, 2).contiguous().view(batch_size, seq_len, -1)
    out1 = F.layer_norm(queries + drop(_lin(context, p, prefix + "w_o."), 0), (d_model,), p[prefix + "norm1.weight"],
                        p[prefix + "norm1.bias"], eps)
    ffn = _lin(drop(F.leaky_relu(_lin(out1, p, prefix + "ffn.0."), 0.01), 1), p, prefix + "ffn.3.")
    return F.layer_norm(out1 + drop(ffn, 2), (d_model,), p[prefix + "norm2.weight"], p[prefix + "norm2.bias"], eps)


def bst_forward_train(p, dense, category, seq_feedid, seq_length, nhead=4, num_blocks=1, num_hidden=3,
                      batch_norm=True, dropout_rate=0.1, pooling_method="sum", block_masks=None, dnn_masks=None,
                      momentum=0.1, eps=1e-5):
    """BSTModel.forward in model.train() (bst.py:216-247): BatchNorm1d with batch statistics (running
    statistics in `p` updated), Dropout as the given multiplier masks; differentiable w.r.t. `p`."""
    category_emb = torch.cat(_cat_fields(p, category, DCN_FIELDS + ["feedid"]), dim=1)
    seq_emb = F.embedding(seq_feedid, p["embeddings.feedid.weight"])
    max_len = seq_feedid.size(1)
    mask = torch.arange(max_len).expand(len(seq_length), max_len) >= seq_length.unsqueeze(1)
    out = seq_emb
    for i in range(num_blocks):
        out = bst_block_train(p, f"transformer_blocks.{i}.", out, out, out, nhead, mask,
                              block_masks[i] if block_masks is not None else None)
    if pooling_method == "sum":
        out = torch.sum(out, dim=1)
    else:
        out = torch.sum(out, dim=1) / seq_length.unsqueeze(1).float()
    h = torch.cat([dense, category_emb, out], dim=1)
    layout, last = bst_dnn_layout(num_hidden, batch_norm, dropout_rate)
    for u, (lin, bn) in enumerate(layout):
        h = _lin(h, p, f"dnn.{lin}.")
        if bn is not None:
            pre = f"dnn.{bn}."
            h = F.batch_norm(h, p[pre + "running_mean"], p[pre + "running_var"], p[pre + "weight"], p[pre + "bias"],
                             training=True, momentum=momentum, eps=eps)
            p[pre + "num_batches_tracked"] += 1
        h = F.leaky_relu(h, 0.01)
        if dnn_masks is not None and dnn_masks[u] is not None:
            h = h * dnn_masks[u]
    logits = _lin(h, p, f"dnn.{last}.")
    return torch.sigmoid(logits), logits


def bst_dnn_layout(num_hidden, batch_norm=True, dropout_rate=0.1):
    """Module indices of dnn (bst.py:203-213): Linear, [BN], LeakyReLU, [Dropout]; last Linear."""
    idx, out = 0, []
    for _ in range(num_hidden):
        lin = idx
        idx += 1
        bn = None
        if batch_norm:
            bn = idx
            idx += 1
        idx += 1
        if dropout_rate > 0:
            idx += 1
        out.append((lin, bn))
    return out, idx


def bst_forward(p, dense, category, seq_feedid, seq_length, nhead=4, num_blocks=1, num_hidden=3,
                batch_norm=True, dropout_rate=0.1, pooling_method="sum"):
    """BSTModel.forward, bst.py:216-247."""
    category_emb = torch.cat(_cat_fields(p, category, DCN_FIELDS + ["feedid"]), dim=1)
    seq_emb = F.embedding(seq_feedid, p["embeddings.feedid.weight"])
    max_len = seq_feedid.size(1)
    mask = torch.arange(max_len).expand(len(seq_length), max_len) >= seq_length.unsqueeze(1)
    out = seq_emb
    for i in range(num_blocks):
        out = bst_block(p, f"transformer_blocks.{i}.", out, out, out, nhead, mask)
    if pooling_method == "sum":
        out = torch.sum(out, dim=1)
    else:
        out = torch.sum(out, dim=1) / seq_length.unsqueeze(1).float()
    h = torch.cat([dense, category_emb, out], dim=1)
    layout, last = bst_dnn_layout(num_hidden, batch_norm, dropout_rate)
    for lin, bn in layout:
        h = _lin(h, p, f"dnn.{lin}.")
        if bn is not None:
            h = _bn_eval(h, p, f"dnn.{bn}.")
        h = F.leaky_relu(h, 0.01)
    logits = _lin(h, p, f"dnn.{last}.")
    return torch.sigmoid(logits), logits
