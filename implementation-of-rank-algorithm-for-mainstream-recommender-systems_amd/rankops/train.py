"""Training on the rankops engine.

The reference scripts train with autograd and torch.optim.Adam:

    model.train(); optimizer = optim.Adam(model.parameters(), lr=...)          # dcn.py:275
    optimizer.zero_grad(); prob, logit = model(dense, category)                # dcn.py:195-196
    loss = criterion(logit.squeeze(), label); loss.backward(); optimizer.step()  # dcn.py:198-201

A rankops model in train mode returns outputs attached to a `torch.autograd.Function` whose
forward runs the HIP forward kernels with the activations the backward needs kept in HBM, and
whose backward runs the HIP backward kernels (include/rankops.h, "training") and hands the
parameter gradients back to autograd — so `loss.backward()` fills every `.grad` as the
reference does and the unchanged loop works with `torch.optim.Adam` or with `rankops.Adam`
(the same update as one fused launch over all tensors, `rk_adam_step`).

Every model trains: DCNModel (`dcn.py:114-180`), DeepCrossingModel (`deepcrossing.py:106-163`)
and AFM (`afm.py:64-119`) — no BatchNorm / Dropout, train and eval forwards coincide —, DeepFM
(`deepfm.py:73-151`: BatchNorm batch statistics, Dropout), DIN (`din.py:225-323`: Dice and
BatchNorm batch statistics, Dropout, attention backward, l2 term), BSTModel (`bst.py:42-247`:
Dropout inside the transformer blocks, LayerNorm, attention backward) and FwFM (`fwfm.py:87-139`).
Dropout masks are a counter hash on the device (train_common.h): a random choice like torch's own
masks, so parity tests hand the engine's masks to the oracle.
"""
from __future__ import annotations

import os

import torch
import torch.optim.optimizer as _optim_mod

from . import common, ops
from .common import PACKED, const, fused_mlp_fits


# BST blocks: the O / FFN2 projections and the residual LayerNorms after them as one launch each
# (rk_linear_res_dropout_ln) where the shape allows (d_model 128); False: two launches each.
FUSED_LN = os.environ.get("RANKOPS_FUSED_LN", "1") != "0"


# ---------------------------------------------------------------- shared pieces

def mlp_relu_forward(x, linears, head_w, head_b, partial, logit, prob):
    """Linear+ReLU stack with the Linear(N,1)+sigmoid head; returns the activations [x, h1, ...].
    The head reads head_partial (the other input block's share of the logit) when given."""
    B, dev = x.shape[0], x.device
    hs = [x] + [torch.empty(B, lin.out_features, device=dev, dtype=torch.float32) for lin in linears]
    if common.FUSED_MLP and fused_mlp_fits(x.shape[1], [lin.out_features for lin in linears]):
        # one rk_mlp_forward launch, each layer's activations also stored for the backward
        # under graph capture the packing is captured too (replays repack the updated weights);
        # a cached image would be frozen into the graph
        pack = ops.pack_mlp_weight if torch.cuda.is_current_stream_capturing() else PACKED
        # the packed images must stay referenced until the launch: the layer descriptors hold raw
        # pointers, and a freed image's block would be handed to the next allocation
        packed = [pack(lin.weight) for lin in linears]
        mls = [ops.make_mlp_layer(lin.weight, pw, bias=lin.bias, act="relu", store=y, ld_store=y.stride(0))
               for lin, pw, y in zip(linears, packed, hs[1:])]
        ep = ops.make_epilogue(head_w=head_w, head_b=head_b, head_logit=logit, head_prob=prob,
                               head_partial=partial)
        ops.mlp_forward(x, mls, ep)
        del packed
        return hs
    h = x
    for i, lin in enumerate(linears):
        last = i == len(linears) - 1
        y = hs[i + 1]
        if last and lin.out_features <= 256:
            ep = ops.make_epilogue(bias=lin.bias, act="relu", head_w=head_w, head_b=head_b, head_logit=logit,
                                   head_prob=prob, head_partial=partial)
        else:
            ep = ops.make_epilogue(bias=lin.bias, act="relu")
        ops.linear(h, lin.weight, y, epilogue=ep)
        h = y
    if linears[-1].out_features > 256:  # head as its own N = 1 GEMM
        ep = ops.make_epilogue(bias=head_b, head_w=const(dev, 1.0), head_b=const(dev, 0.0), head_logit=logit,
                               head_prob=prob, head_partial=partial)
        ops.linear(h, head_w, None, epilogue=ep)
    return hs


def mlp_relu_backward(dh, hs, linears):
    """Backward of mlp_relu_forward's hidden stack from dL/d(last activation); returns
    (dL/dx, [(dW, db) per layer])."""
    grads = [None] * len(linears)
    for i in range(len(linears) - 1, -1, -1):
        dx, dW, db = ops.linear_backward(dh, hs[i], linears[i].weight, relu_out=hs[i + 1])
        grads[i] = (dW, db)
        dh = dx
    return dh, grads


def zero_grads(weights, device):
    """Zero-filled gradient tensors shaped like `weights`, carved from one flat buffer (one fill) at
    256-B aligned offsets, so the row-vector (float4) scatter kernels apply to every table."""
    offs, total = [], 0
    for w in weights:
        offs.append(total)
        total += (w.numel() + 63) // 64 * 64
    flat = torch.zeros(max(total, 1), device=device, dtype=torch.float32)
    return [flat[o:o + w.numel()].view(w.shape) for o, w in zip(offs, weights)]


def embedding_grads(weights, idx, col0, dx, cols=None):
    """Dense nn.Embedding gradients of the tables whose rows sit side by side in dx from column
    col0 on (or at the given `cols`): one zero-filled flat buffer for all tables (one fill),
    then rk_embedding_backward."""
    grads = zero_grads(weights, dx.device)
    if cols is None:
        cols, col = [], col0
        for g in grads:
            cols.append(col)
            col += g.shape[1]
    ops.embedding_backward(ops.table_seg_array(grads, idx, cols), dx.shape[0], dx)
    return grads


def _grad_out(g, like):
    if g is None:
        return None
    return g.to(torch.float32).reshape(like.shape).contiguous()


# ---------------------------------------------------------------- DCN

class _DCNTrain(torch.autograd.Function):
    """DCNModel forward + backward; inputs after the fixed arguments are the module parameters in
    `_dcn_params` order."""

    @staticmethod
    def forward(ctx, model, dense, idx, cw, cb, *params):
        B, dev = dense.shape[0], dense.device
        d = model.input_dim
        segs = ops.dense_table_seg_array(dense, model.num_dense_features, [e.weight for e in model.embeddings.values()],
                                         idx)
        x0 = torch.empty(B, d, device=dev, dtype=torch.float32)
        xl = torch.empty(B, d, device=dev, dtype=torch.float32)
        partial = torch.empty(B, device=dev, dtype=torch.float32)
        w_out = model.output_layer.weight
        ops.dcn_cross(segs, B, d, cw, cb, model.num_cross_layer, w_out.data_ptr(), x0, partial, dev, xl_out=xl)
        logit = torch.empty(B, 1, device=dev, dtype=torch.float32)
        prob = torch.empty(B, 1, device=dev, dtype=torch.float32)
        linears = [m for m in model.dnn if isinstance(m, torch.nn.Linear)]
        hs = mlp_relu_forward(x0, linears, w_out[:, d:], model.output_layer.bias, partial, logit, prob)
        ctx.model = model
        ctx.idx = idx
        ctx.save_for_backward(x0, xl, prob, cw, cb, *hs[1:])
        return prob, logit

    @staticmethod
    def backward(ctx, dprob, dlogit):
        model = ctx.model
        x0, xl, prob, cw, cb, *hidden = ctx.saved_tensors
        hs = [x0] + hidden
        B, d = x0.shape
        dev = x0.device
        w_out = model.output_layer.weight
        dprob, dlogit = _grad_out(dprob, prob), _grad_out(dlogit, prob)
        dxl = torch.empty(B, d, device=dev, dtype=torch.float32)
        dh = torch.empty_like(hs[-1])
        dw_out = torch.empty_like(w_out)
        db_out = torch.empty(1, device=dev, dtype=torch.float32)
        ops.logit_head_backward(dlogit, dprob, prob, xl, hs[-1], w_out, dxl, dh, dw_out, db_out)
        linears = [m for m in model.dnn if isinstance(m, torch.nn.Linear)]
        dx0, lin_grads = mlp_relu_backward(dh, hs, linears)
        ops.dcn_cross_backward(x0, cw, cb, model.num_cross_layer, dxl, dx0, accumulate=True)
        emb_grads = embedding_grads([e.weight for e in model.embeddings.values()], ctx.idx,
                                    model.num_dense_features, dx0)
        flat = [t for pair in lin_grads for t in pair]
        return (None, None, None, None, None, *emb_grads, *flat, dw_out, db_out)


def _dcn_params(model):
    linears = [m for m in model.dnn if isinstance(m, torch.nn.Linear)]
    return ([e.weight for e in model.embeddings.values()] + [t for l in linears for t in (l.weight, l.bias)]
            + [model.output_layer.weight, model.output_layer.bias])


def dcn_train_forward(model, dense, idx, cw, cb):
    if model.output_layer.bias is None or any(m.bias is None for m in model.dnn if isinstance(m, torch.nn.Linear)):
        raise NotImplementedError("rankops DCN training expects the reference's biased Linear layers")
    return _DCNTrain.apply(model, dense, idx, cw, cb, *_dcn_params(model))


# ---------------------------------------------------------------- DeepCrossing

class _DeepCrossingTrain(torch.autograd.Function):
    """DeepCrossingModel forward + backward (deepcrossing.py:146-163): gather, residual units
    (per-call Linear(d, I) / Linear(I, d) drawn like the reference — not module parameters, so
    only the gradient w.r.t. their input is propagated), output_layer + sigmoid."""

    @staticmethod
    def forward(ctx, model, dense, idx, units, *params):
        B, dev = dense.shape[0], dense.device
        d, I = model.input_dim, model.residual_internal_dim
        segs = [ops.dense_segment(dense, model.num_dense_features, 0)]
        col = model.num_dense_features
        for emb, i in zip(model.embeddings.values(), idx):
            segs.append(ops.table_segment(emb.weight, i, col))
            col += emb.embedding_dim
        x0 = torch.empty(B, d, device=dev, dtype=torch.float32)
        ops.concat_gather(segs, B, x0)
        logit = torch.empty(B, 1, device=dev, dtype=torch.float32)
        prob = torch.empty(B, 1, device=dev, dtype=torch.float32)
        head = dict(head_w=model.output_layer.weight, head_b=model.output_layer.bias, head_logit=logit,
                    head_prob=prob)
        acts = []  # h_1, y_1, h_2, y_2, ...
        for _ in units:
            acts += [torch.empty(B, I, device=dev, dtype=torch.float32),
                     torch.empty(B, d, device=dev, dtype=torch.float32)]
        widths = [w for _ in units for w in (I, d)]
        if units and common.FUSED_MLP and fused_mlp_fits(d, widths):
            pack = ops.pack_mlp_weight if torch.cuda.is_current_stream_capturing() else PACKED
            packed = [(pack(w1), pack(w2)) for w1, b1, w2, b2 in units]
            layers = []
            for (w1, b1, w2, b2), (p1, p2), j in zip(units, packed, range(0, len(acts), 2)):
                layers.append(ops.make_mlp_layer(w1, p1, bias=b1, act="relu", store=acts[j], ld_store=I))
                layers.append(ops.make_mlp_layer(w2, p2, bias=b2, act="relu", residual=1, store=acts[j + 1],
                                                 ld_store=d))
            ops.mlp_forward(x0, layers, ops.make_epilogue(**head))
            del packed
        else:
            x = x0
            for (w1, b1, w2, b2), j in zip(units, range(0, len(acts), 2)):
                ops.linear(x, w1, acts[j], epilogue=ops.make_epilogue(bias=b1, act="relu"))
                ops.linear(acts[j], w2, acts[j + 1], epilogue=ops.make_epilogue(
                    bias=b2, residual=x, ld_residual=x.stride(0), act="relu"))
                x = acts[j + 1]
            ep = ops.make_epilogue(bias=model.output_layer.bias, head_w=const(dev, 1.0), head_b=const(dev, 0.0),
                                   head_logit=logit, head_prob=prob)
            ops.linear(x, model.output_layer.weight, None, epilogue=ep)
        ctx.model, ctx.idx = model, idx
        ctx.save_for_backward(x0, prob, *[t for u in units for t in (u[0], u[2])], *acts)
        return prob, logit

    @staticmethod
    def backward(ctx, dprob, dlogit):
        model = ctx.model
        x0, prob, *rest = ctx.saved_tensors
        n = (len(rest)) // 4
        ws, acts = rest[:2 * n], rest[2 * n:]
        B, d = x0.shape
        dev = x0.device
        last = acts[-1] if n else x0
        dy = torch.empty(B, d, device=dev, dtype=torch.float32)
        dw_out = torch.empty_like(model.output_layer.weight)
        db_out = torch.empty(1, device=dev, dtype=torch.float32)
        ops.logit_head_backward(_grad_out(dlogit, prob), _grad_out(dprob, prob), prob, last, None,
                                model.output_layer.weight, dy, None, dw_out, db_out)
        for u in range(n - 1, -1, -1):
            w1, w2 = ws[2 * u], ws[2 * u + 1]
            h, y = acts[2 * u], acts[2 * u + 1]
            I = h.shape[1]
            # y = relu(x + h W2^T + b2), h = relu(x W1^T + b1)
            dh = torch.empty(B, I, device=dev, dtype=torch.float32)
            ops.gemm(False, True, B, I, d, dy, d, w2, I, dh, A_mask=y)           # dz2 W2
            dx = torch.empty(B, d, device=dev, dtype=torch.float32)
            ops.relu_backward(dy, y, dx)                                        # residual path
            ops.gemm(False, True, B, d, I, dh, I, w1, d, dx, A_mask=h, accumulate=True)  # + dz1 W1
            dy = dx
        emb_grads = embedding_grads([e.weight for e in model.embeddings.values()], ctx.idx,
                                    model.num_dense_features, dy)
        return (None, None, None, None, *emb_grads, dw_out, db_out)


def deepcrossing_train_forward(model, dense, idx, units):
    params = [e.weight for e in model.embeddings.values()] + [model.output_layer.weight, model.output_layer.bias]
    return _DeepCrossingTrain.apply(model, dense, idx, units, *params)


# ---------------------------------------------------------------- DeepFM

def deep_units(layers):
    """(Linear, BatchNorm1d or None, ReLU?, dropout p) per unit of a Linear/[BN]/ReLU/[Dropout]
    sequence (deepfm.py:100-109)."""
    units = []
    for m in layers:
        if isinstance(m, torch.nn.Linear):
            units.append([m, None, False, 0.0])
        elif isinstance(m, torch.nn.BatchNorm1d):
            units[-1][1] = m
        elif isinstance(m, torch.nn.ReLU):
            units[-1][2] = True
        elif isinstance(m, torch.nn.Dropout):
            units[-1][3] = float(m.p) if m.training else 0.0
        else:
            raise NotImplementedError(f"rankops training: unsupported layer {type(m).__name__}")
    for lin, bn, relu, _ in units:
        if bn is not None and (bn.momentum is None or not bn.training):
            raise NotImplementedError("rankops training: BatchNorm1d needs a numeric momentum and train mode")
    return units


class DropoutStreams:
    """Per-model dropout stream counter on the device (advanced by rk_rng_next once per train
    forward, so hipGraph replays draw fresh masks) and the seed (torch.initial_seed() when first
    used: seeded runs repeat their masks)."""

    def __init__(self):
        self.counter = None
        self.seed = None

    def next(self, device):
        if self.counter is None or self.counter.device != device:
            self.counter = torch.zeros(1, dtype=torch.int64, device=device)
            self.seed = int(torch.initial_seed()) & 0xFFFFFFFFFFFFFFFF
        slot = torch.empty(1, dtype=torch.int64, device=device)
        ops.rng_next(self.counter, slot)
        return self.seed, slot


def deep_stack_forward(x, units, seed, slot):
    """Train-mode Linear -> [BN] -> ReLU -> [Dropout] stack; returns per-unit saved tensors."""
    B, dev = x.shape[0], x.device
    saved = []
    h = x
    for u, unit in enumerate(units):
        lin, bn, act, p = unit[:4]
        slope = unit[4] if len(unit) > 4 else 0.0
        n = lin.out_features
        z = torch.empty(B, n, device=dev, dtype=torch.float32)
        ops.gemm(False, False, B, n, lin.in_features, h, h.stride(0), lin.weight, lin.weight.stride(0), z)
        y = torch.empty(B, n, device=dev, dtype=torch.float32)
        mean = torch.empty(n, device=dev, dtype=torch.float32)
        invstd = torch.empty(n, device=dev, dtype=torch.float32)
        ws = torch.empty(2 * n, device=dev, dtype=torch.float64)
        ops.bn_act_train_forward(z, lin.bias, bn, act, p, seed + u, slot, y, mean, invstd, ws, slope=slope)
        saved.append((z, y, mean, invstd))
        h = y
    return saved


def deep_stack_backward(dy, x, units, saved, seed, slot):
    """Backward of deep_stack_forward from dL/d(last output); returns (dL/dx, per-unit grads
    [dW, db, (dgamma, dbeta)])."""
    B, dev = x.shape[0], x.device
    grads = [None] * len(units)
    for u in range(len(units) - 1, -1, -1):
        lin, bn, act, p = units[u][:4]
        slope = units[u][4] if len(units[u]) > 4 else 0.0
        z, y, mean, invstd = saved[u]
        n, K = lin.out_features, lin.in_features
        h_in = saved[u - 1][1] if u > 0 else x
        dz = torch.empty(B, n, device=dev, dtype=torch.float32)
        ws = torch.empty(2 * n, device=dev, dtype=torch.float64)
        dg = torch.empty(n, device=dev, dtype=torch.float32) if bn is not None and bn.weight is not None else None
        dbt = torch.empty(n, device=dev, dtype=torch.float32) if bn is not None and bn.bias is not None else None
        ops.bn_act_backward(dy, z, lin.bias, bn, act, p, seed + u, slot, mean, invstd, ws, dz, dg, dbt, slope=slope)
        dW = torch.empty(n, K, device=dev, dtype=torch.float32)
        db = torch.empty(n, device=dev, dtype=torch.float32)
        ops.gemm(True, True, n, K, B, dz, dz.stride(0), h_in, h_in.stride(0), dW, row_sums=db)
        dx = torch.empty(B, K, device=dev, dtype=torch.float32)
        ops.gemm(False, True, B, K, n, dz, dz.stride(0), lin.weight, lin.weight.stride(0), dx)
        g = [dW, db if lin.bias is not None else None]
        if bn is not None:
            g += [t for t in (dg, dbt) if t is not None]
        grads[u] = g
        dy = dx
    return dy, grads


def _unit_params(units):
    out = []
    for unit in units:
        lin, bn = unit[0], unit[1]
        out += [lin.weight] + ([lin.bias] if lin.bias is not None else [])
        if bn is not None:
            out += [t for t in (bn.weight, bn.bias) if t is not None]
    return out


class _DeepFMTrain(torch.autograd.Function):
    """DeepFM forward + backward in train mode (deepfm.py:121-151): FM gather, Linear -> BN(batch
    statistics) -> ReLU -> Dropout units, deep_output_layer, final_layer + sigmoid."""

    @staticmethod
    def forward(ctx, model, names, idx, *params):
        D = model.embedding_dim
        F = len(names)
        B, dev = idx[0].shape[0], idx[0].device
        second = ops.table_seg_array([model.second_order_embeddings[n].weight for n in names], idx,
                                     [f * D for f in range(F)])
        first = ops.table_seg_array([model.first_order_embeddings[n].weight for n in names], idx, list(range(F)))
        deep_in = torch.empty(B, F * D, device=dev, dtype=torch.float32)
        fm1 = torch.empty(B, 1, device=dev, dtype=torch.float32)
        fm2 = torch.empty(B, 1, device=dev, dtype=torch.float32)
        ops.fm_gather(second, first, D, B, deep_in, fm1, fm2)
        units = deep_units(model.deep_layers)
        seed, slot = model._dropout.next(dev)
        saved = deep_stack_forward(deep_in, units, seed, slot)
        last = saved[-1][1] if saved else deep_in
        deep = torch.empty(B, 1, device=dev, dtype=torch.float32)
        total = torch.empty(B, 1, device=dev, dtype=torch.float32)
        prob = torch.empty(B, 1, device=dev, dtype=torch.float32)
        ep = ops.make_epilogue(head_w=model.deep_output_layer.weight, head_b=model.deep_output_layer.bias, fm1=fm1,
                               fm2=fm2, final_w=model.final_layer.weight, final_b=model.final_layer.bias,
                               head_aux=deep, head_logit=total, head_prob=prob)
        ops.mlp_forward(last, [], ep)
        ctx.model, ctx.names, ctx.idx, ctx.units, ctx.seed = model, names, idx, units, seed
        ctx.save_for_backward(deep_in, fm1, fm2, deep, prob, slot, *[t for s in saved for t in s])
        return prob, total, fm1, fm2, deep

    @staticmethod
    def backward(ctx, dprob, dtotal, dfm1_o, dfm2_o, ddeep_o):
        model, units = ctx.model, ctx.units
        deep_in, fm1, fm2, deep, prob, slot, *flat = ctx.saved_tensors
        saved = [tuple(flat[4 * u:4 * u + 4]) for u in range(len(units))]
        B, dev = deep_in.shape[0], deep_in.device
        D, F = model.embedding_dim, len(ctx.names)
        go = [_grad_out(g, prob) for g in (dprob, dtotal, dfm1_o, dfm2_o, ddeep_o)]
        dfm1 = torch.empty(B, 1, device=dev, dtype=torch.float32)
        dfm2 = torch.empty(B, 1, device=dev, dtype=torch.float32)
        ddeep = torch.empty(B, 1, device=dev, dtype=torch.float32)
        dfinal_w = torch.empty_like(model.final_layer.weight)
        dfinal_b = torch.empty(1, device=dev, dtype=torch.float32)
        ops.fm_combine_backward(*go, prob, fm1, fm2, deep, model.final_layer.weight, dfm1, dfm2, ddeep, dfinal_w,
                                dfinal_b)
        last = saved[-1][1] if saved else deep_in
        dy = torch.empty_like(last)
        dw_do = torch.empty_like(model.deep_output_layer.weight)
        db_do = torch.empty(1, device=dev, dtype=torch.float32)
        ops.logit_head_backward(ddeep, None, None, last, None, model.deep_output_layer.weight, dy, None, dw_do, db_do)
        d_deep_in, unit_grads = deep_stack_backward(dy, deep_in, units, saved, ctx.seed, slot)
        d_second = torch.empty(B, F * D, device=dev, dtype=torch.float32)
        ops.fm_backward(deep_in, d_deep_in, dfm2, F, D, d_second)
        g2 = embedding_grads([model.second_order_embeddings[n].weight for n in ctx.names], ctx.idx, 0, d_second)
        g1 = embedding_grads([model.first_order_embeddings[n].weight for n in ctx.names], ctx.idx, 0, dfm1,
                             cols=[0] * F)
        flat_g = [t for g in unit_grads for t in g if t is not None]
        return (None, None, None, *g1, *g2, *flat_g, dw_do, db_do, dfinal_w, dfinal_b)


def deepfm_train_forward(model, names, idx):
    if model.deep_output_layer.bias is None or model.final_layer.bias is None:
        raise NotImplementedError("rankops DeepFM training expects the reference's biased output layers")
    units = deep_units(model.deep_layers)
    params = ([model.first_order_embeddings[n].weight for n in names]
              + [model.second_order_embeddings[n].weight for n in names] + _unit_params(units)
              + [model.deep_output_layer.weight, model.deep_output_layer.bias, model.final_layer.weight,
                 model.final_layer.bias])
    return _DeepFMTrain.apply(model, names, idx, *params)


# ---------------------------------------------------------------- DIN

def din_units(model):
    """(Linear, Dice or PReLU module, BatchNorm1d or None, dropout p) per fcn unit (din.py:272-284)."""
    units = []
    for m in model.fcn:
        if isinstance(m, torch.nn.Linear):
            units.append([m, None, None, 0.0])
        elif isinstance(m, torch.nn.BatchNorm1d):
            units[-1][2] = m
        elif isinstance(m, torch.nn.Dropout):
            units[-1][3] = float(m.p) if m.training else 0.0
        else:  # Dice, or nn.PReLU with activation='prelu' (din.py:275-279)
            units[-1][1] = m
    for lin, act, bn, _ in units:
        if lin.bias is None or act is None:
            raise NotImplementedError("rankops DIN training expects the reference's Linear + Dice / PReLU units")
        if (not isinstance(act, torch.nn.PReLU) and act.bn.momentum is None) or (bn is not None and bn.momentum is None):
            raise NotImplementedError("rankops DIN training: BatchNorm1d needs a numeric momentum")
    return units


class _DINTrain(torch.autograd.Function):
    """DIN forward + backward in train mode (din.py:294-323): gather, din_attention (att_net's
    layers as GEMMs on rk_linear with the activations kept for the backward, the weights drawn per
    call like the reference and not trained), fcn units Linear -> Dice / PReLU -> BatchNorm1d -> Dropout
    with batch statistics, output_layer + sigmoid, and the mini-batch-aware l2 term.
    Inputs after the fixed arguments are the parameters in `_din_params` order."""

    @staticmethod
    def forward(ctx, model, pl, att, emb_plan, *params):
        B, dev, H = pl["B"], pl["dev"], pl["H"]
        q_col, att_col, width, cat_col0 = pl["q_col"], pl["att_col"], pl["width"], pl["cat_col0"]
        seq, seq_len = pl["seq"], pl["seq_len"]
        T = seq.shape[1]
        f32 = dict(device=dev, dtype=torch.float32)
        x = torch.empty(B, width, **f32)
        ops.concat_gather(pl["segs"], B, x)  # [dense | category | target]; the attention columns below
        w1, b1, w2, b2, w3, b3 = att
        keys = torch.empty(B, T, H, **f32)
        cross = torch.empty(B * T, 4 * H, **f32)
        ops.din_att_cross(x, q_col, model.embeddings[pl["seq_key"]].weight, seq, T, H, keys, cross)
        a1 = torch.empty(B * T, w1.shape[0], **f32)
        ops.linear(cross, w1, a1, epilogue=ops.make_epilogue(bias=b1, act="relu"))
        a2 = torch.empty(B * T, w2.shape[0], **f32)
        ops.linear(a1, w2, a2, epilogue=ops.make_epilogue(bias=b2, act="relu"))
        del cross
        wts = torch.empty(B, T, **f32)
        ops.din_att_pool_forward(a2, w3.reshape(-1), b3, keys, seq_len, T, H, model.use_softmax, wts, x, att_col)
        units = din_units(model)
        seed, slot = model._dropout.next(dev)
        saved = []
        h = x
        for u, (lin, dice, bn, p) in enumerate(units):
            n, K = lin.out_features, lin.in_features
            z = torch.empty(B, n, **f32)
            ops.gemm(False, False, B, n, K, h, h.stride(0), lin.weight, lin.weight.stride(0), z)
            y1 = torch.empty(B, n, **f32)
            m1, s1 = torch.empty(n, **f32), torch.empty(n, **f32)
            if isinstance(dice, torch.nn.PReLU):
                ops.prelu_train_forward(z, lin.bias, dice, y1)
            else:
                ops.dice_train_forward(z, lin.bias, dice, y1, m1, s1,
                                       torch.empty(2 * n, device=dev, dtype=torch.float64))
            y2, m2, s2 = y1, m1, s1
            if bn is not None or p > 0:
                y2 = torch.empty(B, n, **f32)
                m2, s2 = torch.empty(n, **f32), torch.empty(n, **f32)
                ops.bn_act_train_forward(y1, None, bn, False, p, seed + u, slot, y2, m2, s2,
                                         torch.empty(2 * n, device=dev, dtype=torch.float64))
            saved.append((z, y1, m1, s1, y2, m2, s2))
            h = y2
        logit = torch.empty(B, 1, **f32)
        prob = torch.empty(B, 1, **f32)
        ops.mlp_forward(h, [], ops.make_epilogue(head_w=model.output_layer.weight, head_b=model.output_layer.bias,
                                                 head_logit=logit, head_prob=prob))
        l2 = torch.zeros((), **f32)
        if pl["want_l2"]:
            ops.row_l2norm_mean(x, cat_col0, width - cat_col0, float(model.l2_lambda), l2)
        ctx.model, ctx.pl, ctx.units, ctx.seed, ctx.emb_plan = model, pl, units, seed, emb_plan
        ctx.save_for_backward(x, keys, a1, a2, wts, prob, slot, w1, w2, w3, *[t for s in saved for t in s])
        return prob, logit, l2

    @staticmethod
    def backward(ctx, dprob, dlogit, dl2):
        model, pl, units = ctx.model, ctx.pl, ctx.units
        x, keys, a1, a2, wts, prob, slot, w1, w2, w3, *flat = ctx.saved_tensors
        saved = [tuple(flat[7 * u:7 * u + 7]) for u in range(len(units))]
        B, dev, H = pl["B"], pl["dev"], pl["H"]
        T = keys.shape[1]
        f32 = dict(device=dev, dtype=torch.float32)
        last = saved[-1][4] if saved else x
        dy = torch.empty_like(last)
        w_out = model.output_layer.weight
        dw_out = torch.empty_like(w_out)
        db_out = torch.empty(1, **f32)
        ops.logit_head_backward(_grad_out(dlogit, prob), _grad_out(dprob, prob), prob, last, None, w_out, dy, None,
                                dw_out, db_out)
        unit_grads = [None] * len(units)
        for u in range(len(units) - 1, -1, -1):
            lin, dice, bn, p = units[u]
            z, y1, m1, s1, y2, m2, s2 = saved[u]
            n, K = lin.out_features, lin.in_features
            h_in = saved[u - 1][4] if u > 0 else x
            dy1 = dy
            dg = dbt = None
            if bn is not None or p > 0:
                dy1 = torch.empty(B, n, **f32)
                if bn is not None:
                    dg = torch.empty(n, **f32) if bn.weight is not None else None
                    dbt = torch.empty(n, **f32) if bn.bias is not None else None
                ops.bn_act_backward(dy, y1, None, bn, False, p, ctx.seed + u, slot, m2, s2,
                                    torch.empty(2 * n, device=dev, dtype=torch.float64), dy1, dg, dbt)
            dz = torch.empty(B, n, **f32)
            if isinstance(dice, torch.nn.PReLU):
                dalpha = torch.empty_like(dice.weight)
                ops.prelu_backward(dy1, z, lin.bias, dice, torch.empty(dice.weight.numel(), device=dev,
                                                                       dtype=torch.float64), dz, dalpha)
            else:
                dalpha = torch.empty(n, **f32)
                ops.dice_backward(dy1, z, lin.bias, dice, m1, s1, torch.empty(3 * n, device=dev, dtype=torch.float64),
                                  dz, dalpha)
            dW = torch.empty(n, K, **f32)
            db = torch.empty(n, **f32)
            ops.gemm(True, True, n, K, B, dz, dz.stride(0), h_in, h_in.stride(0), dW, row_sums=db)
            dx = torch.empty(B, K, **f32)
            ops.gemm(False, True, B, K, n, dz, dz.stride(0), lin.weight, lin.weight.stride(0), dx)
            unit_grads[u] = [dW, db, dalpha] + ([t for t in (dg, dbt) if t is not None] if bn is not None else [])
            dy = dx
        dxr = dy  # dL/d[dense | category | target | attention]
        if pl["want_l2"] and dl2 is not None:
            ops.row_l2norm_backward(x, pl["cat_col0"], pl["width"] - pl["cat_col0"], float(model.l2_lambda) / B,
                                    dl2.to(torch.float32).reshape(1).contiguous(), dxr)
        # din_attention backward: weighted sum and scores, then att_net (its weights are not trained)
        M = B * T
        dkeys = torch.empty(B, T, H, **f32)
        da2 = torch.empty(M, a2.shape[1], **f32)
        ops.din_att_pool_backward(dxr, pl["att_col"], wts, keys, a2, w3.reshape(-1), pl["seq_len"], T, H,
                                  model.use_softmax, dkeys, da2)
        da1 = torch.empty(M, a1.shape[1], **f32)
        ops.gemm(False, True, M, a1.shape[1], a2.shape[1], da2, da2.stride(0), w2, w2.stride(0), da1)
        dcross = torch.empty(M, 4 * H, **f32)
        ops.gemm(False, True, M, 4 * H, a1.shape[1], da1, da1.stride(0), w1, w1.stride(0), dcross, A_mask=a1)
        ops.din_cross_fold(dcross, x, pl["q_col"], keys, T, H, dkeys, dxr)
        del dcross
        # nn.Embedding gradients: one zeroed buffer per distinct table, every lookup scattered into it
        weights, looks = ctx.emb_plan
        grads = zero_grads(weights, dev)
        segs = [ops.table_segment(grads[k], i, col) for k, i, col in looks]
        ops.embedding_backward(segs, B, dxr)
        # History keys past seq_len get exactly zero gradient (their attention weight is 0 and so is
        # their score's gradient, din.py:61-84), so the padded positions that all map to row 0 add
        # nothing and the zero-skipping atomic scatter stays contention-free (the sorted
        # segment-reduce, whose radix sort alone costs ~85 us here, is only needed where padded
        # positions carry gradient: BST's sum pooling; the length-0 softmax case, where all T
        # weights are 1/T, is still exact, only slower).
        ops.embedding_backward([ops.table_segment(grads[pl["seq_slot"]], pl["seq"].reshape(-1), 0)], M,
                               dkeys.view(M, H))
        flat = [t for g in unit_grads for t in g]
        return (None, None, None, None, *grads, *flat, dw_out, db_out)


def _din_params(model, units):
    out = []
    for lin, act, bn, _ in units:
        out += [lin.weight, lin.bias, act.weight if isinstance(act, torch.nn.PReLU) else act.alpha]
        if bn is not None:
            out += [t for t in (bn.weight, bn.bias) if t is not None]
    return out + [model.output_layer.weight, model.output_layer.bias]


def din_train_forward(model, pl, att):
    """DIN train-mode forward with autograd (rankops.DIN.forward in model.train())."""
    units = din_units(model)
    # distinct embedding tables in first-use order and the (table slot, index, column) lookups
    weights, looks = [], []

    def slot_of(w):
        for k, t in enumerate(weights):
            if t is w:
                return k
        weights.append(w)
        return len(weights) - 1

    for w, idx, col in pl["lookups"]:
        looks.append((slot_of(w), idx, col))
    pl = dict(pl, seq_slot=slot_of(model.embeddings[pl["seq_key"]].weight))
    return _DINTrain.apply(model, pl, att, (weights, looks), *weights, *_din_params(model, units))


# ---------------------------------------------------------------- AFM

class _AFMTrain(torch.autograd.Function):
    """AFM forward + backward (afm.py:92-119; no train/eval difference in the module).  Inputs
    after the fixed arguments: dense_layer.{weight,bias}, the field embeddings, attention.0.{weight,
    bias}, attention.2.{weight,bias}, p.{weight,bias}."""

    @staticmethod
    def forward(ctx, model, dense, idx, *params):
        F, D = model.num_fields, model.embedding_dim
        wd, bd = params[0], params[1]
        tables = params[2:2 + F]
        w1, b1, w2, b2, wp, bp = params[2 + F:]
        B, dev = dense.shape[0], dense.device
        P = F * (F - 1) // 2
        f32 = dict(device=dev, dtype=torch.float32)
        emb = torch.empty(B, F * D, **f32)
        pairs = torch.empty(B * P, D, **f32)
        ops.afm_pairs([ops.table_segment(t, i, 0) for t, i in zip(tables, idx)], D, B, emb, pairs)
        a1 = torch.empty(B * P, w1.shape[0], **f32)
        ops.linear(pairs, w1, a1, epilogue=ops.make_epilogue(bias=b1, act="relu"))
        weights = torch.empty(B, P, **f32)
        ws = torch.empty(B, D, **f32)
        logit = torch.empty(B, 1, **f32)
        pred = torch.empty(B, 1, **f32)
        ops.afm_pool_forward(a1, w2.reshape(-1), b2, pairs, P, D, dense, wd.reshape(-1), bd, wp.reshape(-1), bp,
                             weights, ws, logit, pred)
        ctx.model, ctx.idx = model, idx
        ctx.save_for_backward(dense, emb, pairs, a1, weights, ws, pred, w1, w2, wp, *tables)
        return pred, logit

    @staticmethod
    def backward(ctx, dpred, dlogit):
        model, idx = ctx.model, ctx.idx
        dense, emb, pairs, a1, weights, ws, pred, w1, w2, wp, *tables = ctx.saved_tensors
        F, D = model.num_fields, model.embedding_dim
        B, dev = dense.shape[0], dense.device
        P, A, nd = F * (F - 1) // 2, w1.shape[0], dense.shape[1]
        f32 = dict(device=dev, dtype=torch.float32)
        d_pairs = torch.empty(B * P, D, **f32)
        da1 = torch.empty(B * P, A, **f32)
        acc = torch.empty(nd + 1 + D + 1 + A + 1, **f32)
        ops.afm_pool_backward(_grad_out(dpred, pred) if dpred is not None else None,
                              _grad_out(dlogit, pred) if dlogit is not None else None, pred, weights, ws, pairs, a1,
                              w2.reshape(-1), wp.reshape(-1), dense, P, D, d_pairs, da1, acc)
        dW1 = torch.empty_like(w1)
        db1 = torch.empty(A, **f32)
        M = B * P
        ops.gemm(True, True, A, D, M, da1, A, pairs, D, dW1, row_sums=db1)
        ops.gemm(False, True, M, D, A, da1, A, w1, D, d_pairs, accumulate=True)
        d_emb = torch.empty(B, F * D, **f32)
        ops.afm_pair_fold(d_pairs, emb, F, D, d_emb)
        g_emb = embedding_grads(list(tables), idx, 0, d_emb)
        o = 0
        dwd, dbd = acc[o:o + nd].view(1, nd), acc[o + nd:o + nd + 1]
        o += nd + 1
        dwp, dbp = acc[o:o + D].view(1, D), acc[o + D:o + D + 1]
        o += D + 1
        dw2, db2 = acc[o:o + A].view(1, A), acc[o + A:o + A + 1]
        return (None, None, None, dwd, dbd, *g_emb, dW1, db1, dw2, db2, dwp, dbp)


def afm_train_forward(model, dense, idx):
    att1, att2 = model.attention[0], model.attention[2]
    params = ([model.dense_layer.weight, model.dense_layer.bias]
              + [model.embeddings[c].weight for c in model.category_features]
              + [att1.weight, att1.bias, att2.weight, att2.bias, model.p.weight, model.p.bias])
    if any(t is None for t in params):
        raise NotImplementedError("rankops AFM training expects the reference's biased Linear layers")
    return _AFMTrain.apply(model, dense, idx, *params)


# ---------------------------------------------------------------- BST

def bst_units(model):
    """([Linear, BatchNorm1d or None, 'leaky', dropout p, slope] per dnn unit, last Linear)
    (bst.py:203-213)."""
    mods = list(model.dnn)
    units = []
    for m in mods[:-1]:
        if isinstance(m, torch.nn.Linear):
            units.append([m, None, "none", 0.0, 0.0])
        elif isinstance(m, torch.nn.BatchNorm1d):
            if m.momentum is None:
                raise NotImplementedError("rankops BST training: BatchNorm1d needs a numeric momentum")
            units[-1][1] = m
        elif isinstance(m, torch.nn.LeakyReLU):
            units[-1][2], units[-1][4] = "leaky", float(m.negative_slope)
        elif isinstance(m, torch.nn.Dropout):
            units[-1][3] = float(m.p) if m.training else 0.0
        else:
            raise NotImplementedError(f"rankops BST training: unsupported dnn layer {type(m).__name__}")
    return units, mods[-1]


def _block_params(blk):
    return [blk.position_embedding.weight, blk.w_q.weight, blk.w_q.bias, blk.w_k.weight, blk.w_k.bias,
            blk.w_v.weight, blk.w_v.bias, blk.w_o.weight, blk.w_o.bias, blk.norm1.weight, blk.norm1.bias,
            blk.norm2.weight, blk.norm2.bias, blk.ffn[0].weight, blk.ffn[0].bias, blk.ffn[3].weight, blk.ffn[3].bias]


def bst_dropout_seed(seed, block, site):
    """Dropout stream seed of transformer block `block`, site 0 (w_o output), 1 (inside the FFN),
    2 (FFN output); the dnn units use seed + unit."""
    return seed + 100 + 3 * block + site


def _lin_grads(dy, x, w, need_dx=True, dx=None, accumulate=False):
    """y = x W^T + b backward with dy row stride dy.stride(0): (dW, db[, dx])."""
    M, N = dy.shape[0], w.shape[0]
    K = w.shape[1]
    dW = torch.empty(N, K, device=dy.device, dtype=torch.float32)
    db = torch.empty(N, device=dy.device, dtype=torch.float32)
    ops.gemm(True, True, N, K, M, dy, dy.stride(0), x, x.stride(0), dW, row_sums=db)
    if need_dx:
        if dx is None:
            dx = torch.empty(M, K, device=dy.device, dtype=torch.float32)
        ops.gemm(False, True, M, K, N, dy, dy.stride(0), w, w.stride(0), dx, accumulate=accumulate)
    return dW, db, dx


class _BSTTrain(torch.autograd.Function):
    """BSTModel forward + backward in train mode (bst.py:216-247 with BSTTransformer.forward
    bst.py:66-91): Dropout in every block (w_o output, inside and after the FFN) and in the dnn,
    BatchNorm1d with batch statistics.  Inputs after the fixed arguments: the distinct embedding
    tables of `plan`, then per block `_block_params`, then the dnn unit parameters and the last
    Linear."""

    @staticmethod
    def forward(ctx, model, plan, *params):
        seq, seq_len, B, T, width, col = plan["seq"], plan["seq_len"], plan["B"], plan["T"], plan["width"], plan["col"]
        dev, d = seq.device, model.d_model
        M = B * T
        f32 = dict(device=dev, dtype=torch.float32)
        row = torch.empty(B, width, **f32)
        ops.concat_gather(plan["segs"], B, row)
        feed = model.embeddings["feedid"].weight
        x = torch.empty(M, d, **f32)
        seed, slot = model._dropout.next(dev)
        saves = []
        for i, blk in enumerate(model.transformer_blocks):
            p_o, p_f = float(blk.dropout.p) if blk.training else 0.0, float(blk.ffn[2].p) if blk.training else 0.0
            h = blk.nhead
            xp = torch.empty(M, d, **f32)
            pos = blk.position_embedding.weight
            if i > 0 or not ops.bst_gather_pos(feed, seq.reshape(-1), T, pos, x, xp):
                if i == 0:
                    ops.concat_gather([ops.table_segment(feed, seq.view(-1), 0)], M, x)
                ops.bst_add_pos(x, pos, T, xp)
            qkv = torch.empty(M, 3 * d, **f32)
            ops.linear(xp, blk.w_q.weight, None, y_ptr=qkv.data_ptr(), ldy=3 * d,
                       epilogue=ops.make_epilogue(bias=blk.w_q.bias))
            ops.linear(xp, blk.w_k.weight, None, y_ptr=ops._lib.fptr(qkv, d), ldy=3 * d,
                       epilogue=ops.make_epilogue(bias=blk.w_k.bias))
            ops.linear(x, blk.w_v.weight, None, y_ptr=ops._lib.fptr(qkv, 2 * d), ldy=3 * d,
                       epilogue=ops.make_epilogue(bias=blk.w_v.bias))
            cx = torch.empty(M, d, **f32)
            # P is kept for the backward (recomputing it there measured slower at configs[3]: backward
            # 185 -> 242 us against forward 114 -> 108 us)
            probs = torch.empty(B * h * T * T, **f32)
            ops.bst_attn_train_forward(qkv, B, T, d, h, seq_len, probs, cx)
            r1, out1 = torch.empty(M, d, **f32), torch.empty(M, d, **f32)
            m1, s1 = torch.empty(M, **f32), torch.empty(M, **f32)
            # out1 = LN1(xp + dropout(w_o(cx))): one launch when the shape allows
            if not (FUSED_LN and ops.linear_res_dropout_ln(cx, blk.w_o.weight, blk.w_o.bias, xp, p_o,
                                                           bst_dropout_seed(seed, i, 0), slot, blk.norm1, r1, out1,
                                                           m1, s1)):
                o = torch.empty(M, d, **f32)
                ops.linear(cx, blk.w_o.weight, o, epilogue=ops.make_epilogue(bias=blk.w_o.bias))
                ops.bst_res_dropout_ln_forward(xp, o, p_o, bst_dropout_seed(seed, i, 0), slot, blk.norm1, r1, out1, m1,
                                               s1)
                del o
            f1 = torch.empty(M, d, **f32)
            ops.linear(out1, blk.ffn[0].weight, f1, epilogue=ops.make_epilogue(bias=blk.ffn[0].bias))
            a = torch.empty(M, d, **f32)
            ops.bst_leaky_dropout(None, f1, blk.ffn[1].negative_slope, p_f, bst_dropout_seed(seed, i, 1), slot, False, a)
            r2, out = torch.empty(M, d, **f32), torch.empty(M, d, **f32)
            m2, s2 = torch.empty(M, **f32), torch.empty(M, **f32)
            if not (FUSED_LN and ops.linear_res_dropout_ln(a, blk.ffn[3].weight, blk.ffn[3].bias, out1, p_o,
                                                           bst_dropout_seed(seed, i, 2), slot, blk.norm2, r2, out,
                                                           m2, s2)):
                f2 = torch.empty(M, d, **f32)
                ops.linear(a, blk.ffn[3].weight, f2, epilogue=ops.make_epilogue(bias=blk.ffn[3].bias))
                ops.bst_res_dropout_ln_forward(out1, f2, p_o, bst_dropout_seed(seed, i, 2), slot, blk.norm2, r2, out,
                                               m2, s2)
            saves.append((x, xp, qkv, probs, cx, r1, out1, m1, s1, f1, a, r2, m2, s2))
            x = out
        mean_pool = model.pooling_method != "sum"
        if not saves:  # no blocks: transformer_output = seq_emb (bst.py:229), pooled over all T positions
            ops.concat_gather([ops.table_segment(feed, seq.view(-1), 0)], M, x)
        ops.bst_pool(x, B, T, seq_len, mean_pool, row, col)
        units, last = bst_units(model)
        saved = deep_stack_forward(row, units, seed, slot)
        hid = saved[-1][1] if saved else row
        logit = torch.empty(B, 1, **f32)
        prob = torch.empty(B, 1, **f32)
        ops.mlp_forward(hid, [], ops.make_epilogue(head_w=last.weight, head_b=last.bias, head_logit=logit,
                                                   head_prob=prob))
        ctx.model, ctx.plan, ctx.units, ctx.seed, ctx.nsave = model, plan, units, seed, len(saves)
        ctx.save_for_backward(row, prob, slot, *[t for sv in saves for t in sv], *[t for sv in saved for t in sv])
        return prob, logit

    @staticmethod
    def backward(ctx, dprob, dlogit):
        model, plan, units, seed = ctx.model, ctx.plan, ctx.units, ctx.seed
        row, prob, slot, *flat = ctx.saved_tensors
        nb = ctx.nsave
        saves = [tuple(flat[14 * i:14 * i + 14]) for i in range(nb)]
        flat = flat[14 * nb:]
        saved = [tuple(flat[4 * u:4 * u + 4]) for u in range(len(units))]
        seq, seq_len, B, T, col = plan["seq"], plan["seq_len"], plan["B"], plan["T"], plan["col"]
        dev, d = row.device, model.d_model
        M = B * T
        f32 = dict(device=dev, dtype=torch.float32)
        _, last = bst_units(model)
        hid = saved[-1][1] if saved else row
        dh = torch.empty_like(hid)
        dw_last = torch.empty_like(last.weight)
        db_last = torch.empty(1, **f32)
        ops.logit_head_backward(_grad_out(dlogit, prob), _grad_out(dprob, prob), prob, hid, None, last.weight, dh,
                                None, dw_last, db_last)
        d_row, unit_grads = deep_stack_backward(dh, row, units, saved, seed, slot)
        mean_pool = model.pooling_method != "sum"
        dx = None  # the last block's LN2 backward reads the pooling gradient d_row directly
        tables, looks = plan["tables"], plan["looks"]
        tgrads = zero_grads(tables, dev)
        block_grads = [None] * nb
        for i in range(nb - 1, -1, -1):
            blk = model.transformer_blocks[i]
            x, xp, qkv, probs, cx, r1, out1, m1, s1, f1, a, r2, m2, s2 = saves[i]
            p_o, p_f = float(blk.dropout.p) if blk.training else 0.0, float(blk.ffn[2].p) if blk.training else 0.0
            # out = LN2(out1 + dropout(f2))
            d_out1 = torch.empty(M, d, **f32)
            df2 = torch.empty(M, d, **f32)
            dg2, dbe2 = torch.empty(d, **f32), torch.empty(d, **f32)
            if dx is None and not ops.bst_pool_ln_backward(d_row, col, T, seq_len, mean_pool, r2, m2, s2, blk.norm2,
                                                           p_o, bst_dropout_seed(seed, i, 2), slot, d_out1, df2, dg2,
                                                           dbe2):
                dx = torch.empty(M, d, **f32)
                ops.bst_pool_backward(d_row, col, B, T, d, seq_len, mean_pool, dx)
            if dx is not None:
                ops.bst_ln_backward(dx, r2, m2, s2, blk.norm2, p_o, bst_dropout_seed(seed, i, 2), slot, d_out1, df2,
                                    dg2, dbe2)
            dW2, db2, da = _lin_grads(df2, a, blk.ffn[3].weight)
            df1 = torch.empty(M, d, **f32)
            ops.bst_leaky_dropout(da, f1, blk.ffn[1].negative_slope, p_f, bst_dropout_seed(seed, i, 1), slot, True, df1)
            dW1, db1, _ = _lin_grads(df1, out1, blk.ffn[0].weight, dx=d_out1, accumulate=True)
            # out1 = LN1(xp + dropout(o))
            dxp = torch.empty(M, d, **f32)
            do = torch.empty(M, d, **f32)
            dg1, dbe1 = torch.empty(d, **f32), torch.empty(d, **f32)
            ops.bst_ln_backward(d_out1, r1, m1, s1, blk.norm1, p_o, bst_dropout_seed(seed, i, 0), slot, dxp, do, dg1,
                                dbe1)
            dWo, dbo, dcx = _lin_grads(do, cx, blk.w_o.weight)
            dqkv = torch.empty(M, 3 * d, **f32)
            ops.bst_attn_train_backward(qkv, probs, dcx, B, T, d, blk.nhead, dqkv)
            dQ, dK, dV = dqkv[:, :d], dqkv[:, d:2 * d], dqkv[:, 2 * d:]
            dWq, dbq, _ = _lin_grads(dQ, xp, blk.w_q.weight, dx=dxp, accumulate=True)
            dWk, dbk, _ = _lin_grads(dK, xp, blk.w_k.weight, dx=dxp, accumulate=True)
            # position embedding: every row m adds into pos[m % T]
            gpos = torch.zeros_like(blk.position_embedding.weight)
            ops.bst_pos_backward(dxp, B, T, gpos)
            # keys/queries carry x + pos, values carry x: dL/dx = dL/dxp + dV Wv
            dWv, dbv, _ = _lin_grads(dV, x, blk.w_v.weight, dx=dxp, accumulate=True)
            block_grads[i] = [gpos, dWq, dbq, dWk, dbk, dWv, dbv, dWo, dbo, dg1, dbe1, dg2, dbe2, dW1, db1, dW2, db2]
            dx = dxp
        if nb == 0:  # no blocks: the pooling gradient goes straight to the gathered sequence rows
            dx = torch.empty(M, d, **f32)
            ops.bst_pool_backward(d_row, col, B, T, d, seq_len, mean_pool, dx)
        # embedding tables: the category lookups from the dnn input row, the behaviour sequence from dx
        segs = [ops.table_segment(tgrads[k], idx, c) for k, idx, c in looks]
        if segs:
            ops.embedding_backward(segs, B, d_row)
        # padded positions all map to row 0 and carry non-zero gradients (sum pooling): their runs are
        # pre-summed per sample (rk_embedding_backward_seq), else the sorted segment-reduce
        if not ops.embedding_backward_seq(tgrads[plan["feed_slot"]], seq, dx):
            ops.embedding_backward_sorted(ops.table_segment(tgrads[plan["feed_slot"]], seq.view(-1), 0), M, dx)
        flat_units = [t for g in unit_grads for t in g if t is not None]
        return (None, None, *tgrads, *[t for g in block_grads for t in g], *flat_units, dw_last, db_last)


def bst_train_forward(model, dense, category, seq, seq_len):
    """BSTModel train-mode forward with autograd (rankops.BSTModel.forward in model.train())."""
    B, T = seq.shape
    d = model.d_model
    for blk in model.transformer_blocks:
        if T > 64 or d // blk.nhead > 64 or d % blk.nhead or d > 256:
            raise NotImplementedError("rankops BST training: T <= 64, d_model <= 256, d_model / nhead <= 64")
    segs = [ops.dense_segment(dense, model.num_dense_features, 0)]
    col = model.num_dense_features
    tables, looks = [], []

    def slot_of(w):
        for k, t in enumerate(tables):
            if t is w:
                return k
        tables.append(w)
        return len(tables) - 1

    for name, emb in model.embeddings.items():
        if name in category:
            idx = ops.as_index(category[name], f"category[{name!r}]")
            segs.append(ops.table_segment(emb.weight, idx, col))
            looks.append((slot_of(emb.weight), idx, col))
            col += emb.embedding_dim
    feed_slot = slot_of(model.embeddings["feedid"].weight)
    plan = dict(seq=seq, seq_len=seq_len, B=B, T=T, width=col + d, col=col, segs=segs, tables=tables, looks=looks,
                feed_slot=feed_slot)
    units, last = bst_units(model)
    params = (tables + [t for blk in model.transformer_blocks for t in _block_params(blk)] + _unit_params(units)
              + [last.weight, last.bias])
    return _BSTTrain.apply(model, plan, *params)


# ---------------------------------------------------------------- FwFM

class _FwFMTrain(torch.autograd.Function):
    """FwFM forward (rk_fwfm_forward, fwfm.py:114-139; no train/eval difference) + backward
    (rk_fwfm_backward, then the table scatters).  Inputs after the fixed arguments: the linear
    tables, the embedding tables, field_weight, bias."""

    @staticmethod
    def forward(ctx, model, idx, want_logit, *params):
        F = model.num_fields
        lin_w, emb_w = params[:F], params[F:2 * F]
        field_weight, bias = params[2 * F], params[2 * F + 1]
        B, dev = idx[0].shape[0], idx[0].device
        zeros = [0] * F
        emb = ops.table_seg_array(emb_w, idx, zeros)
        lin = ops.table_seg_array(lin_w, idx, zeros)
        prob = torch.empty(B, device=dev, dtype=torch.float32)
        logit = torch.empty(B, device=dev, dtype=torch.float32) if want_logit else None
        ops.fwfm_forward(emb, lin, model.embed_dim, B, field_weight, bias, logit, prob)
        ctx.model, ctx.idx = model, idx
        ctx.save_for_backward(prob, field_weight, *emb_w, *lin_w)
        if want_logit:
            ctx.mark_non_differentiable(logit)
            return prob, logit
        return prob

    @staticmethod
    def backward(ctx, dprob, *_):
        model, idx = ctx.model, ctx.idx
        F, D = model.num_fields, model.embed_dim
        prob, field_weight, *tabs = ctx.saved_tensors
        emb_w, lin_w = tabs[:F], tabs[F:]
        B, dev = prob.shape[0], prob.device
        f32 = dict(device=dev, dtype=torch.float32)
        d_emb = torch.empty(B, F * D, **f32)
        dz = torch.empty(B, 1, **f32)
        d_r = torch.empty_like(field_weight)
        d_b = torch.empty(1, **f32)
        ops.fwfm_backward(ops.table_seg_array(emb_w, idx, [0] * F), D, B, field_weight, prob,
                          _grad_out(dprob, prob), d_emb, dz, d_r, d_b)
        g_emb = embedding_grads(list(emb_w), idx, 0, d_emb)
        g_lin = embedding_grads(list(lin_w), idx, 0, dz, cols=[0] * F)
        return (None, None, None, *g_lin, *g_emb, d_r, d_b)


def fwfm_train_forward(model, idx, want_logit):
    params = ([m.weight for m in model.linear] + [m.weight for m in model.embedding]
              + [model.field_weight, model.bias])
    return _FwFMTrain.apply(model, idx, want_logit, *params)


# ---------------------------------------------------------------- optimizer

class Adam(torch.optim.Optimizer):
    """torch.optim.Adam with the update as one rk_adam_step launch over all tensors of a group.
    Same constructor, param_groups and state layout (`step`, `exp_avg`, `exp_avg_sq`), so state
    dicts move between this class and torch.optim.Adam.  amsgrad / maximize / differentiable /
    sparse gradients are not implemented and raise."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False, *,
                 maximize=False, foreach=None, capturable=False, differentiable=False, fused=None):
        if amsgrad or maximize or differentiable:
            raise NotImplementedError("rankops.Adam: amsgrad / maximize / differentiable are not implemented")
        if not 0.0 <= float(lr):
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameters: {betas}")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad, maximize=maximize,
                        foreach=foreach, capturable=capturable, differentiable=differentiable, fused=fused)
        super().__init__(params, defaults)

    def step(self, closure=None):
        """torch.optim's step wrapper (a record_function scope and the step hooks) is taken only when
        a profiler or a hook is there to see it: on the eager loop its cost is of the order of the
        fused update itself."""
        if (torch.autograd.profiler._is_profiler_enabled or _optim_mod._global_optimizer_pre_hooks
                or _optim_mod._global_optimizer_post_hooks or self._optimizer_step_pre_hooks
                or self._optimizer_step_post_hooks):
            return _hooked_step(self, closure)
        return self._step(closure)

    step.hooked = True  # torch.optim.Optimizer._patch_step_function: do not wrap again

    def zero_grad(self, set_to_none: bool = True):
        """Optimizer.zero_grad; with set_to_none (the default, the reference's loop) a plain reset of
        every .grad outside a profiler."""
        if not set_to_none or torch.autograd.profiler._is_profiler_enabled:
            return super().zero_grad(set_to_none)
        for group in self.param_groups:
            for p in group["params"]:
                p.grad = None

    @torch.no_grad()
    def _step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            if not group["capturable"] and self._fast_step(gi, group):
                continue
            if self.__dict__.get("_fast", {}).pop(gi, None) is not None:
                # the general path moves step counts one parameter at a time: give every parameter
                # its own step tensor again (the fast path shares one per group)
                for p in group["params"]:
                    st = self.state.get(p)
                    if st and "step" in st:
                        st["step"] = st["step"].clone()
            beta1, beta2 = group["betas"]
            capturable = group["capturable"]
            by_step = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise NotImplementedError("rankops.Adam: sparse gradients")
                if p.device.type != "cuda" or p.dtype != torch.float32 or not p.is_contiguous():
                    raise RuntimeError("rankops.Adam: parameters must be contiguous float32 ROCm tensors")
                state = self.state[p]
                if len(state) == 0:
                    # torch's layout: a float32 step tensor, on the device when capturable
                    state["step"] = torch.zeros((), dtype=torch.float32, device=p.device) if capturable \
                        else torch.tensor(0.0, dtype=torch.float32)
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                g = p.grad if p.grad.is_contiguous() and p.grad.dtype == torch.float32 else \
                    p.grad.to(torch.float32).contiguous()
                if capturable:  # incremented on the device by rk_adam_step: graph-capturable
                    if state["step"].device != p.device:
                        state["step"] = state["step"].to(p.device)
                    by_step.setdefault(0, []).append((p, g, state["exp_avg"], state["exp_avg_sq"], state["step"]))
                else:
                    if state["step"].device.type != "cpu":
                        state["step"] = state["step"].cpu()
                    state["step"] += 1
                    by_step.setdefault(int(state["step"].item()), []).append(
                        (p, g, state["exp_avg"], state["exp_avg_sq"]))
            for step, entries in by_step.items():
                dev = entries[0][0].device
                ops.adam_step(entries, float(group["lr"]), beta1, beta2, group["eps"], group["weight_decay"], step,
                              ops._lib.raw_stream(dev))
                # the kernel wrote through raw pointers: bump the version counters as torch's
                # in-place ops would, so weight-derived caches (packed MLP images) are rebuilt
                torch.autograd.graph.increment_version([t for e in entries for t in (e[0], e[2], e[3])])
        return loss

    def _fast_step(self, gi, group) -> bool:
        """The eager step with the marshalled rk_adam_step argument block reused: valid while the
        group's parameters and their states stay the same and every parameter is at the same step
        count (the reference's loop: every parameter gets a gradient every step); new gradient
        storages are patched into the block.  Per step: one increment of the shared CPU step tensor,
        one launch, one version bump.  Anything else (first step, a missing gradient, mixed step
        counts) takes the general path, which rebuilds the block next time."""
        params = group["params"]
        grads = [p.grad for p in params]
        if not params or any(g is None for g in grads):
            return False
        cache = self.__dict__.setdefault("_fast", {})
        key = tuple(p.data_ptr() for p in params)
        gkey = tuple(g.data_ptr() for g in grads)
        hit = cache.get(gi)
        if hit is not None and hit[0] == key and hit[7] != gkey:
            # new gradient storages (the caching allocator need not hand last step's addresses back
            # after zero_grad(set_to_none=True)): patch the pointers into the block, no rebuild
            if any(g.dtype != torch.float32 or not g.is_contiguous() or g.is_sparse or g.numel() != p.numel()
                   or g.device != p.device for g, p in zip(grads, params)):
                return False
            arr = hit[1]
            for i, g in enumerate(grads):
                arr[i].grad = g.data_ptr()
            hit[7] = gkey
        if hit is None or hit[0] != key:
            states = [self.state.get(p) for p in params]
            if any(not st for st in states) or any(st["step"].device.type != "cpu" for st in states):
                cache.pop(gi, None)
                return False
            if any(g.dtype != torch.float32 or not g.is_contiguous() or g.is_sparse for g in grads) or \
                    any(p.device.type != "cuda" or p.dtype != torch.float32 or not p.is_contiguous() for p in params):
                return False
            counts = {float(st["step"]) for st in states}
            if len(counts) != 1:
                return False
            # one step tensor object for the group (all counts are equal here): a step is then one
            # in-place add instead of a foreach over every parameter's CPU scalar
            shared = states[0]["step"]
            for st in states:
                st["step"] = shared
            entries = [(p, g, st["exp_avg"], st["exp_avg_sq"]) for p, g, st in zip(params, grads, states)]
            arr = (ops._lib.AdamTensor * len(entries))(*[
                ops._lib.AdamTensor(e[0].data_ptr(), e[1].data_ptr(), e[2].data_ptr(), e[3].data_ptr(), e[0].numel(),
                                    None) for e in entries])
            bumped = [t for e in entries for t in (e[0], e[2], e[3])]
            # the block keeps raw gradient pointers only: holding the gradient tensors would keep
            # last step's storages alive across zero_grad(set_to_none=True), so the next backward
            # could never get the same addresses and the key would miss every step
            hit = [key, arr, len(entries), shared, int(counts.pop()), bumped, params[0].device, gkey]
            cache[gi] = hit
            self._fast_builds = getattr(self, "_fast_builds", 0) + 1
        _key, arr, n, step_t, count, bumped, dev, _gkey = hit
        step_t.add_(1.0)
        hit[4] = count = count + 1
        beta1, beta2 = group["betas"]
        ops.check(ops._lib.load().rk_adam_step(arr, n, float(group["lr"]), beta1, beta2, group["eps"],
                                               group["weight_decay"], count,
                                               ops._lib.raw_stream(dev)), "rk_adam_step")
        torch.autograd.graph.increment_version(bumped)
        return True

    def load_state_dict(self, state_dict):
        self.__dict__.pop("_fast", None)  # new state tensors: rebuild the argument blocks
        return super().load_state_dict(state_dict)

    def state_dict(self):
        """Optimizer.state_dict with a step tensor of its own per parameter (the fast path shares
        one per group; another optimizer loading the dict must not see them aliased)."""
        sd = super().state_dict()
        for st in sd["state"].values():
            if "step" in st:
                st["step"] = st["step"].clone()
        return sd


_hooked_step = torch.optim.Optimizer.profile_hook_step(Adam._step)
