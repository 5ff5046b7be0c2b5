"""DCN (Deep & Cross Network) on the rankops engine — drop-in for algorithm/DCN/dcn.py.

`DCNModel(vocab_dir, hidden_units=[512, 256, 128], num_cross_layer=1)` keeps the reference
constructor, parameter creation order (so a seeded construction gives the same weights),
`state_dict` keys (dcn.py:130-152: no cross-layer keys) and `forward(dense, category) ->
(probability, logit)` (dcn.py:161-180).  In train mode with autograd recording, the same
forward runs under `rankops.train._DCNTrain`, whose backward is HIP too (loss.backward() fills
every .grad).  The eval forward is one launch, rk_dcn_forward: per 16-row tile the gather of the
6 fields + dense (dcn.py:163-169) straight into the MLP's LDS input, the cross layers in registers
(dcn.py:25-50,171-173) with the cross half of output_layer, the dnn tail (dcn.py:175) and the head
(output_layer + sigmoid, dcn.py:177-180).  Shapes outside its envelope (more than 8 segments,
width > 256, hidden widths past the fused MLP's) run rk_dcn_cross + the rk_mlp_forward / rk_linear
tail instead.

The cross weights are drawn per call from the CPU generator like the reference
(`interaction_weights="per_call"`, dcn.py:37-45) or drawn once and kept on the device
(`"frozen"`).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import common, ops, train
from .common import EngineModule, InteractionWeights, Layer, draw_cross_layers, load_vocabulary, run_tail, table_rows


def cross_layer(x0: torch.Tensor, xl: torch.Tensor, index: int) -> torch.Tensor:
    """One reference cross layer (dcn.py:25-50): fresh xavier-normal w and zero b from the CPU
    generator, then x0 * (xl . w) + b + xl in the rk_dcn_cross kernel."""
    x0 = ops.as_f32(x0, "x0")
    xl = ops.as_f32(xl, "xl")
    B, d = x0.shape
    w, b = draw_cross_layers(d, 1)
    w, b = w.to(x0.device), b.to(x0.device)
    out = torch.empty(B, d, device=x0.device, dtype=torch.float32)
    ops.dcn_cross([ops.dense_segment(x0, d, 0)], B, d, w, b, 1, None, None, None, x0.device, xl_in=xl,
                  xl_out=out)
    return out


class DCNModel(EngineModule):
    def __init__(self, vocab_dir, hidden_units=[512, 256, 128], num_cross_layer=1, *, vocab_sizes=None,
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
        category_emb_dim = 16 + 2 + 4 + 4 + 4 + 4
        self.input_dim = self.num_dense_features + category_emb_dim
        self.num_cross_layer = num_cross_layer
        layers = []
        width = self.input_dim
        for h in hidden_units:
            layers += [nn.Linear(width, h), nn.ReLU()]
            width = h
        self.dnn = nn.Sequential(*layers)
        self.output_layer = nn.Linear(self.input_dim + hidden_units[-1], 1)
        self._tail = [Layer(m, act="relu") for m in self.dnn if isinstance(m, nn.Linear)]
        self.cross_weights = InteractionWeights(
            interaction_weights, lambda: draw_cross_layers(self.input_dim, self.num_cross_layer))

    def _load_vocabulary(self, vocab_dir, filename):
        return load_vocabulary(vocab_dir, filename)

    def forward(self, dense, category):
        # no BatchNorm / Dropout: the train-mode forward computes what the eval forward does; with
        # autograd recording it also keeps the activations for the HIP backward (rankops.train)
        dense = ops.as_f32(dense, "dense")
        B = dense.shape[0]
        dev = dense.device
        segs = [ops.dense_segment(dense, self.num_dense_features, 0)]
        col = self.num_dense_features
        idx_keep = []
        for name, emb in self.embeddings.items():
            if name not in category:
                raise KeyError(f"DCNModel.forward: category feature {name!r} missing")
            idx = ops.as_index(category[name], f"category[{name!r}]")
            idx_keep.append(idx)
            segs.append(ops.table_segment(emb.weight, idx, col))
            col += emb.embedding_dim
        cw, cb = self.cross_weights.get(dev)
        if self.training and torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            return train.dcn_train_forward(self, dense, idx_keep, cw, cb)
        logit = torch.empty(B, 1, device=dev, dtype=torch.float32)
        prob = torch.empty(B, 1, device=dev, dtype=torch.float32)
        if (common.FUSED_MLP and len(segs) <= 8 and self.input_dim <= 256
                and common.fused_mlp_fits(self.input_dim, [l.linear.out_features for l in self._tail])):
            # one launch: gather + cross stack + MLP tail + head (rk_dcn_forward)
            mls = [ops.make_mlp_layer(l.linear.weight, common.PACKED(l.linear.weight), **l.epilogue_kwargs())
                   for l in self._tail]
            head = _HeadView(self.output_layer, self.input_dim)
            ep = ops.make_epilogue(head_w=head.weight, head_b=head.bias, head_logit=logit, head_prob=prob)
            ops.dcn_forward(segs, B, self.input_dim, cw, cb, self.num_cross_layer, self.output_layer.weight, mls, ep,
                            dev)
            return prob, logit
        x0 = torch.empty(B, self.input_dim, device=dev, dtype=torch.float32)
        partial = torch.empty(B, device=dev, dtype=torch.float32)
        head_w = self.output_layer.weight
        ops.dcn_cross(segs, B, self.input_dim, cw, cb, self.num_cross_layer, head_w.data_ptr(), x0, partial, dev)
        head = _HeadView(self.output_layer, self.input_dim)
        run_tail(x0, self._tail, head, dict(head_partial=partial), logit, prob)
        return prob, logit


class _HeadView:
    """The dnn half of output_layer: weight columns [offset:], same bias (dcn.py:177-178)."""

    def __init__(self, linear: nn.Linear, offset: int):
        self.weight = linear.weight[:, offset:]
        self.bias = linear.bias
