"""Deep Crossing on the rankops engine — drop-in for algorithm/DeepCrossing/deepcrossing.py.

`DeepCrossingModel(vocab_dir, residual_internal_dim=128, residual_network_num=1)` keeps the
reference constructor, state_dict keys (`embeddings.*`, `output_layer.*`; the residual units
have none, deepcrossing.py:106-137) and `forward(dense, category) -> (probability, logit)`
(deepcrossing.py:146-163).

Launches: rk_concat_gather -> x0 [B, 50]; per residual unit two rk_linear calls
(Linear+ReLU, then Linear + residual + ReLU), the last one also evaluating output_layer and
the sigmoid in its epilogue.  The residual units' Linear layers are drawn per call from the
CPU generator like the reference (deepcrossing.py:37-39) or frozen.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import ops, train
from . import common
from .common import InteractionWeights, check_eval, const, draw_residual_units, fused_mlp_fits, load_vocabulary, residual_spec, \
    table_rows


def residual_unit(input_tensor, internal_dim, index, weights=None):
    """Reference residual_unit (deepcrossing.py:25-42): ReLU(x + Linear2(ReLU(Linear1(x))))."""
    x = ops.as_f32(input_tensor, "input_tensor")
    B, d = x.shape
    if weights is None:
        weights = [t.to(x.device) for t in draw_residual_units(d, internal_dim, 1)[0]]
    w1, b1, w2, b2 = weights
    h = torch.empty(B, internal_dim, device=x.device, dtype=torch.float32)
    ops.linear(x, w1, h, epilogue=ops.make_epilogue(bias=b1, act="relu"))
    out = torch.empty(B, d, device=x.device, dtype=torch.float32)
    ops.linear(h, w2, out, epilogue=ops.make_epilogue(bias=b2, residual=x, ld_residual=x.stride(0), act="relu"))
    return out


class DeepCrossingModel(common.EngineModule):
    def __init__(self, vocab_dir, residual_internal_dim=128, residual_network_num=1, *, vocab_sizes=None,
                 interaction_weights="per_call"):
        super().__init__()
        fields = ("userid", "feedid", "device", "authorid", "bgm_song_id", "bgm_singer_id", "manual_tag_list")
        self.vocab_sizes = {f: table_rows(vocab_dir, f, vocab_sizes) for f in fields}
        self.num_dense_features = 16
        self.embeddings = nn.ModuleDict({
            "userid": nn.Embedding(self.vocab_sizes["userid"], 16),
            "device": nn.Embedding(self.vocab_sizes["device"], 2),
            "authorid": nn.Embedding(self.vocab_sizes["authorid"], 4),
            "bgm_song_id": nn.Embedding(self.vocab_sizes["bgm_song_id"], 4),
            "bgm_singer_id": nn.Embedding(self.vocab_sizes["bgm_singer_id"], 4),
            "manual_tag_list": nn.Embedding(self.vocab_sizes["manual_tag_list"], 4),
        })
        self.input_dim = self.num_dense_features + 16 + 2 + 4 + 4 + 4 + 4
        self.residual_internal_dim = residual_internal_dim
        self.residual_network_num = residual_network_num
        self.output_layer = nn.Linear(self.input_dim, 1)
        self.residual_weights = InteractionWeights(
            interaction_weights,
            lambda: residual_spec(self.input_dim, self.residual_internal_dim, self.residual_network_num))

    def _load_vocabulary(self, vocab_dir, filename):
        return load_vocabulary(vocab_dir, filename)

    def _mlp_layers(self, units):
        """rk_mlp_layer records of the residual units (packed images from common.PACKED)."""
        layers = []
        for w1, b1, w2, b2 in units:
            layers.append(ops.make_mlp_layer(w1, common.PACKED(w1), bias=b1, act="relu"))
            layers.append(ops.make_mlp_layer(w2, common.PACKED(w2), bias=b2, act="relu", residual=1))
        return layers

    def prepare(self, dense, category):
        """An eval forward bound to these input tensors (as DCNModel.prepare): returns `run()` that
        recomputes the forward from the current contents of the inputs with one
        rk_mlp_forward_gather launch (row gather + every residual unit + output_layer + sigmoid) and
        returns the same (prob, logit) tensors each time.  Binds the current weights: the residual
        units' and the output layer's packed images are pinned, so a later weight update is not seen
        by run() (prepare again after an update).  Frozen residual weights only (per-call mode redraws
        them every forward).  Index tensors must be int64 (bound by address, never copied)."""
        if self.training:
            raise RuntimeError("DeepCrossingModel.prepare: eval mode only (call .eval() first)")
        if self.residual_weights.mode != "frozen":
            raise RuntimeError("DeepCrossingModel.prepare: per-call residual weights are redrawn every forward; "
                               "use interaction_weights='frozen'")
        dense = ops.as_f32(dense, "dense")
        B, dev = dense.shape[0], dense.device
        segs = [ops.dense_segment(dense, self.num_dense_features, 0)]
        col, idxs = self.num_dense_features, []
        for name, emb in self.embeddings.items():
            idx = ops.bound_index(category[name], f"category[{name!r}]")
            idxs.append(idx)
            segs.append(ops.table_segment(emb.weight, idx, col))
            col += emb.embedding_dim
        units = self.residual_weights.get(dev)
        widths = [w for _ in units for w in (self.residual_internal_dim, self.input_dim)]
        if not (units and common.FUSED_MLP and fused_mlp_fits(self.input_dim, widths) and len(segs) <= 16
                and self.input_dim <= 256):
            raise RuntimeError("DeepCrossingModel.prepare: configuration outside rk_mlp_forward_gather's envelope")
        logit = torch.empty(B, 1, device=dev, dtype=torch.float32)
        prob = torch.empty(B, 1, device=dev, dtype=torch.float32)
        head = ops.make_epilogue(head_w=self.output_layer.weight, head_b=self.output_layer.bias, head_logit=logit,
                                 head_prob=prob)
        for w1, _, w2, _ in units:  # the images the launch binds are never rewritten in place under it
            common.PACKED.pin(w1)
            common.PACKED.pin(w2)
        packed = [common.PACKED(w) for w1, _, w2, _ in units for w in (w1, w2)]
        layers = self._mlp_layers(units)
        ops._lib.ensure_device(dev)
        larr = (ops._lib.MlpLayer * len(layers))(*layers)
        args = (ops._seg_array(segs), len(segs), self.input_dim, B, larr, len(layers), ops.ctypes.byref(head),
                ops._lib.stream_of(prob))
        fn, out = ops._lib.load().rk_mlp_forward_gather, (prob, logit)

        def run():
            ops.check(fn(*args), "rk_mlp_forward_gather")
            return out
        run.keep = (args, head, packed, units, segs, idxs, dense, category)
        return run

    def forward(self, dense, category):
        # no BatchNorm / Dropout: train mode computes the eval forward; with autograd recording it
        # runs under rankops.train._DeepCrossingTrain (HIP backward)
        dense = ops.as_f32(dense, "dense")
        B = dense.shape[0]
        dev = dense.device
        recording = self.training and torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
        if B == 0 and not recording:
            self.residual_weights.get(dev)  # per-call mode draws every forward (deepcrossing.py:25-42)
            return common.empty_rows(dev, 2)
        segs = [ops.dense_segment(dense, self.num_dense_features, 0)]
        col = self.num_dense_features
        for name, emb in self.embeddings.items():
            if name not in category:
                raise KeyError(f"DeepCrossingModel.forward: category feature {name!r} missing")
            idx = ops.as_index(category[name], f"category[{name!r}]")
            segs.append(ops.table_segment(emb.weight, idx, col))
            col += emb.embedding_dim
        if self.training and torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            idx = [ops.as_index(category[name], f"category[{name!r}]") for name in self.embeddings]
            return train.deepcrossing_train_forward(self, dense, idx, self.residual_weights.get(dev))
        logit = torch.empty(B, 1, device=dev, dtype=torch.float32)
        prob = torch.empty(B, 1, device=dev, dtype=torch.float32)
        head = dict(head_w=self.output_layer.weight, head_b=self.output_layer.bias, head_logit=logit,
                    head_prob=prob)
        units = self.residual_weights.get(dev)
        I = self.residual_internal_dim
        widths = [w for _ in units for w in (I, self.input_dim)]
        fused = units and common.FUSED_MLP and fused_mlp_fits(self.input_dim, widths)
        if fused and common.FUSED_GATHER_MLP and len(segs) <= 16 and self.input_dim <= 256:
            # the row gather, every residual unit, output_layer and sigmoid in one launch
            layers = self._mlp_layers(units)
            ops._lib.ensure_device(dev)
            ops.check(ops._lib.load().rk_mlp_forward_gather(ops._seg_array(segs), len(segs), self.input_dim, B,
                                                            (ops._lib.MlpLayer * len(layers))(*layers), len(layers),
                                                            ops.ctypes.byref(ops.make_epilogue(**head)),
                                                            ops._lib.stream_of(prob)), "rk_mlp_forward_gather")
            return prob, logit
        x = torch.empty(B, self.input_dim, device=dev, dtype=torch.float32)
        ops.concat_gather(segs, B, x)
        if fused:
            # all residual units + output_layer + sigmoid in one launch
            layers = []
            for w1, b1, w2, b2 in units:
                layers.append(ops.make_mlp_layer(w1, common.PACKED(w1), bias=b1, act="relu"))
                layers.append(ops.make_mlp_layer(w2, common.PACKED(w2), bias=b2, act="relu", residual=1))
            ops.mlp_forward(x, layers, ops.make_epilogue(**head))
            return prob, logit
        for i, (w1, b1, w2, b2) in enumerate(units):
            last = i == len(units) - 1
            h = torch.empty(B, I, device=dev, dtype=torch.float32)
            ops.linear(x, w1, h, epilogue=ops.make_epilogue(bias=b1, act="relu"))
            res = dict(bias=b2, residual=x, ld_residual=x.stride(0), act="relu")
            if last:
                ops.linear(h, w2, None, epilogue=ops.make_epilogue(**res, **head))
            else:
                y = torch.empty(B, self.input_dim, device=dev, dtype=torch.float32)
                ops.linear(h, w2, y, epilogue=ops.make_epilogue(**res))
                x = y
        if not units:
            ep = ops.make_epilogue(bias=self.output_layer.bias, head_w=const(dev, 1.0), head_b=const(dev, 0.0),
                                   head_logit=logit, head_prob=prob)
            ops.linear(x, self.output_layer.weight, None, epilogue=ep)
        return prob, logit
