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
from .common import (EngineModule, InteractionWeights, Layer, cross_spec, draw_cross_layers, load_vocabulary, run_tail,
                     table_rows)


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
            interaction_weights, lambda: cross_spec(self.input_dim, self.num_cross_layer))

    def _load_vocabulary(self, vocab_dir, filename):
        return load_vocabulary(vocab_dir, filename)

    def _eager_eval(self, dense, category):
        """The fused eval forward through the EagerCalls cache: on a hit one ctypes call with fresh
        output pointers (and the per-call H2 weights, if any) patched in; None when the fused
        path does not apply."""
        if not common.EAGER_CACHE:
            return None
        try:
            idx = [category[n] for n in self.embeddings]
        except (KeyError, TypeError):
            return None
        if not isinstance(dense, torch.Tensor) or dense.device.type != "cuda" or \
                not all(isinstance(t, torch.Tensor) for t in idx):
            return None  # lists / arrays take the normal path (as_index's descriptive errors)
        dev = dense.device
        stream = ops._lib.raw_stream(dev)
        calls = self.__dict__.setdefault("_eager", common.EagerCalls())
        key = calls.key(self, [dense] + idx, stream, (self.cross_weights.mode,))
        hit = calls.get(key)
        if hit is None and self._eager_build(dense, category, key, calls) is None:
            return None
        cw, cb = self.cross_weights.get(dev)  # per-call mode: the reference's draws, once per forward
        args, head, B, _keep = calls.get(key)
        logit = torch.empty(B, 1, device=dev, dtype=torch.float32)
        prob = torch.empty(B, 1, device=dev, dtype=torch.float32)
        head.head_logit = logit.data_ptr()
        head.head_prob = prob.data_ptr()
        args[4], args[5], args[-1] = cw.data_ptr(), cb.data_ptr(), stream
        ops.check(ops._lib.load().rk_dcn_forward(*args), "rk_dcn_forward")
        return prob, logit

    def _eager_build(self, dense, category, key, calls):
        dense = ops.as_f32(dense, "dense")
        B, dev = dense.shape[0], dense.device
        segs = [ops.dense_segment(dense, self.num_dense_features, 0)]
        col = self.num_dense_features
        for name, emb in self.embeddings.items():
            idx = category[name]
            if not isinstance(idx, torch.Tensor) or idx.dtype != torch.int64 or idx.device != dev:
                return None  # conversions make new tensors per call: the uncached path
            segs.append(ops.table_segment(emb.weight, ops.as_index(idx, f"category[{name!r}]"), col))
            col += emb.embedding_dim
        if not (common.FUSED_MLP and len(segs) <= 8 and self.input_dim <= 256
                and common.fused_mlp_fits(self.input_dim, [l.linear.out_features for l in self._tail])):
            return None
        packed = [common.PACKED(l.linear.weight) for l in self._tail]
        mls = [ops.make_mlp_layer(l.linear.weight, pk, **l.epilogue_kwargs()) for l, pk in zip(self._tail, packed)]
        head = _HeadView(self.output_layer, self.input_dim)
        ep = ops.make_epilogue(head_w=head.weight, head_b=head.bias)
        args = ops.dcn_forward_args(segs, B, self.input_dim, None, None, self.num_cross_layer,
                                    self.output_layer.weight, mls, ep, dev)
        # the packed images and the head view stay referenced by the entry: the argument block
        # holds their raw pointers (cross weights and outputs are patched in per call)
        return calls.put(key, (args, ep, B, (packed, head, segs)))

    def prepare(self, dense, category):
        """An eval forward bound to these input tensors (as DIN.prepare: the single-kernel analogue of
        capturing the forward in a hipGraph): returns `run()` that recomputes the whole forward from
        the current contents of the inputs with one rk_dcn_forward launch and returns the same
        (prob, logit) tensors each time.  Binds the current weights (frozen interaction weights only:
        per-call mode redraws them every forward)."""
        if self.training:
            raise RuntimeError("DCNModel.prepare: eval mode only (call .eval() first)")
        if self.cross_weights.mode != "frozen":
            raise RuntimeError("DCNModel.prepare: per-call interaction weights are redrawn every forward; "
                               "use interaction_weights='frozen'")
        calls = common.EagerCalls(1)
        dev = dense.device
        stream = ops._lib.raw_stream(dev)
        if self._eager_build(dense, category, 0, calls) is None:
            raise RuntimeError("DCNModel.prepare: configuration outside rk_dcn_forward's envelope")
        args, head, B, keep = calls.get(0)
        for l in self._tail:  # the images the plan binds are never rewritten in place under it
            common.PACKED.pin(l.linear.weight)
        cw, cb = self.cross_weights.get(dev)
        logit = torch.empty(B, 1, device=dev, dtype=torch.float32)
        prob = torch.empty(B, 1, device=dev, dtype=torch.float32)
        head.head_logit, head.head_prob = logit.data_ptr(), prob.data_ptr()
        args[4], args[5], args[-1] = cw.data_ptr(), cb.data_ptr(), stream
        fn, out = ops._lib.load().rk_dcn_forward, (prob, logit)

        def run():
            ops.check(fn(*args), "rk_dcn_forward")
            return out
        run.keep = (keep, head, cw, cb, dense, category)
        return run

    def forward(self, dense, category):
        if not self.training and ops.as_f32(dense, "dense").shape[0] == 0:
            self.cross_weights.get(dense.device)  # per-call mode draws every forward, as dcn.py:37-41 does
            return common.empty_rows(dense.device, 2)
        if not self.training:
            out = self._eager_eval(dense, category)
            if out is not None:
                return out
        # no BatchNorm / Dropout: the train-mode forward computes what the eval forward does; with
        # autograd recording it also keeps the activations for the HIP backward (rankops.train)
        dense = ops.as_f32(dense, "dense")
        B = dense.shape[0]
        dev = dense.device
        idx_keep = []
        for name in self.embeddings:
            if name not in category:
                raise KeyError(f"DCNModel.forward: category feature {name!r} missing")
            idx_keep.append(ops.as_index(category[name], f"category[{name!r}]"))
        cw, cb = self.cross_weights.get(dev)
        if self.training and torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            return train.dcn_train_forward(self, dense, idx_keep, cw, cb)  # marshals its own segments
        segs = [ops.dense_segment(dense, self.num_dense_features, 0)]
        col = self.num_dense_features
        for (name, emb), idx in zip(self.embeddings.items(), idx_keep):
            segs.append(ops.table_segment(emb.weight, idx, col))
            col += emb.embedding_dim
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
