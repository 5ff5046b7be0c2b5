"""DeepFM on the rankops engine — drop-in for algorithm/DeepFM/deepfm.py.

`DeepFM(vocab_dir, embedding_dim=8, hidden_units=None, dropout_rate=0.1, batch_norm=True)`
keeps the reference constructor, creation order and state_dict keys
(`first_order_embeddings.*`, `second_order_embeddings.*`, `deep_layers.N.*`,
`deep_output_layer.*`, `final_layer.*`; deepfm.py:73-112) and
`forward(category) -> (probability, total_logit, fm1, fm2, deep_logit)` (deepfm.py:121-151).

Beyond the reference's six wechat fields the constructor takes `vocab_sizes={field: rows-1}`
(any field names, dict order = field order) so the 30-field benchmark configuration runs
through the same class; with the default wechat vocabulary it is the reference model.

Launches: rk_fm_gather_packed (both embedding orders, fm1, fm2 and the deep input in one pass over
one packed [V, pad4(D+1)] table per field, built once per weight version by rk_fm_pack_table;
PACKED_TABLES = False gathers from the two nn.Embedding weights with rk_fm_gather), then
the deep layers on rk_linear with BatchNorm folded into the epilogue; the last one also
evaluates deep_output_layer, final_layer(3->1) and the sigmoid.  When the first deep layer runs as a
2D-tiled GEMM (common.tiled_layer: the 30-field benchmark configuration), the gather, fm1, fm2 and
that layer are one rk_fm_linear_packed launch (FUSED_FRONT): the deep input is staged in LDS and
never written to HBM, and the eval forward is two launches.  At configs[1]'s shape (30 fields x 32,
hidden [512, 256, 128]) the whole eval forward is one rk_deepfm_forward launch (FUSED_WHOLE): the
gather, the FM sums, the three deep layers on one weight stream and the head per 16-row tile.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import ops, train
from . import common
from .common import EngineModule, Layer, PackedFMTable, check_eval, load_vocabulary, run_tail, table_rows

WECHAT_FIELDS = ("userid", "feedid", "device", "authorid", "bgm_song_id", "bgm_singer_id")
# Eval gather from packed [V, pad4(D+1)] tables (one line pair per row instead of a row line plus
# a separate line for the 4-B first-order weight; costs one extra table copy in HBM).
PACKED_TABLES = True
# rk_fm_gather's field-major switch point (csrc/embedding.hip launch_fm_gather, RANKOPS_FM_FMAJ_MIN)
FIELD_MAJOR_MIN = 16384
# Gather + FM + first deep layer in one rk_fm_linear_packed launch when that layer is tiled.
FUSED_FRONT = True
# The whole eval forward in one rk_deepfm_forward launch where a plan is compiled for the shape
# (960 -> 512 -> 256 -> 128: configs[1]); otherwise FUSED_FRONT's two launches.
FUSED_WHOLE = True


class DeepFM(EngineModule):
    def __init__(self, vocab_dir, embedding_dim=8, hidden_units=None, dropout_rate=0.1, batch_norm=True, *,
                 vocab_sizes=None):
        super().__init__()
        if hidden_units is None:
            hidden_units = [512, 256, 128]
        if vocab_sizes is not None and any(f not in WECHAT_FIELDS for f in vocab_sizes):
            self.vocab_sizes = {f: int(n) + 1 for f, n in vocab_sizes.items()}
        else:
            self.vocab_sizes = {f: table_rows(vocab_dir, f, vocab_sizes) for f in WECHAT_FIELDS}
        self.num_categories = len(self.vocab_sizes)
        self.embedding_dim = embedding_dim
        self.first_order_embeddings = nn.ModuleDict(
            {col: nn.Embedding(n, 1) for col, n in self.vocab_sizes.items()})
        self.second_order_embeddings = nn.ModuleDict(
            {col: nn.Embedding(n, embedding_dim) for col, n in self.vocab_sizes.items()})
        self.deep_layers = nn.ModuleList()
        width = self.num_categories * embedding_dim
        self._tail = []
        for unit in hidden_units:
            lin = nn.Linear(width, unit)
            self.deep_layers.append(lin)
            bn = None
            if batch_norm:
                bn = nn.BatchNorm1d(unit)
                self.deep_layers.append(bn)
            self.deep_layers.append(nn.ReLU())
            if dropout_rate > 0:
                self.deep_layers.append(nn.Dropout(dropout_rate))
            self._tail.append(Layer(lin, pre_bn=bn, act="relu"))
            width = unit
        self.deep_output_layer = nn.Linear(width, 1)
        self.final_layer = nn.Linear(3, 1)
        self._dropout = train.DropoutStreams()
        self._fm_packs = {}  # field -> PackedFMTable (eval gather layout, not part of the state_dict)

    def _load_vocabulary(self, vocab_dir, filename):
        return load_vocabulary(vocab_dir, filename)

    def packed_table(self, name):
        """The packed [V, pad4(D+1)] eval table of field `name` (cached per weight version)."""
        pk = self._fm_packs.get(name)
        if pk is None:
            pk = self._fm_packs[name] = PackedFMTable()
        return pk(self.second_order_embeddings[name].weight, self.first_order_embeddings[name].weight)

    def _gather_plan(self, names, category, deep=True, packed=None):
        D = self.embedding_dim
        first = ops.as_index(category[names[0]], f"category[{names[0]!r}]")
        B, dev = first.shape[0], first.device
        fits = D % 4 == 0 and (D // 4) & (D // 4 - 1) == 0 and D <= 256
        if packed is None:
            # from FIELD_MAJOR_MIN samples the gather runs field-major (fm_gather_fmaj_kernel), where
            # the [V, D] + [V, 1] weights as they are beat the packed rows (one 128-B request per
            # row instead of two; the first-order lines are re-read on die): 109 vs 153 us at 65,536
            packed = PACKED_TABLES and B < FIELD_MAJOR_MIN
        packed = packed and fits
        second_segs, first_segs = [], []
        for f, name in enumerate(names):
            idx = ops.as_index(category[name], f"category[{name!r}]")
            if packed:
                if idx.stride(0) != 1:
                    idx = idx.contiguous()
                second_segs.append(ops.packed_segment(self.packed_table(name), idx, D, f * D))
                first_segs.append(idx)  # keeps a contiguous copy alive for the launch
            else:
                second_segs.append(ops.table_segment(self.second_order_embeddings[name].weight, idx, f * D))
                first_segs.append(ops.table_segment(self.first_order_embeddings[name].weight, idx, f))
        deep_in = torch.empty(B, len(names) * D, device=dev, dtype=torch.float32) if deep else None
        fm1 = torch.empty(B, 1, device=dev, dtype=torch.float32)
        fm2 = torch.empty(B, 1, device=dev, dtype=torch.float32)
        return (packed, second_segs, first_segs, D, B, deep_in, fm1, fm2)

    @staticmethod
    def _launch(plan):
        packed, second, first, D, B, deep_in, fm1, fm2 = plan
        if packed:
            ops.fm_gather_packed(second, D, B, deep_in, fm1, fm2)
        else:
            ops.fm_gather(second, first, D, B, deep_in, fm1, fm2)

    def _gather_fm(self, names, category):
        """rk_fm_gather_packed / rk_fm_gather: both embedding orders, fm1, fm2 and the deep input
        row in one pass (deepfm.py:122-140,142)."""
        plan = self._gather_plan(names, category)
        self._launch(plan)
        return plan[5], plan[6], plan[7]

    def gather_launcher(self, category, packed=None):
        """Zero-argument re-launch of this forward's FM gather kernel, for kernel-level timing
        (bench.py gather roofline).  packed=False: the two nn.Embedding weights as they are — the
        [V, D] second-order rows (128 B = one line at D = 32) and the [V, 1] first-order table."""
        names = [c for c in self.second_order_embeddings if c in category]
        plan = self._gather_plan(names, category, packed=packed)
        return lambda: self._launch(plan)

    def _eager_eval(self, category):
        """The eval forward through the EagerCalls cache (common.EagerCalls): the marshalled
        launches (rk_fm_linear_packed + rk_mlp_forward, or rk_fm_gather_packed + the tail) reused
        with fresh outputs patched in; rebuilt per call with EAGER_CACHE off.  None off that path."""
        try:
            idx = [category[n] for n in self.second_order_embeddings]
        except (KeyError, TypeError):
            return None
        if not all(isinstance(t, torch.Tensor) and t.dtype == torch.int64 for t in idx) or idx[0].device.type != "cuda":
            return None
        dev = idx[0].device
        stream = ops._lib.raw_stream(dev)
        if common.EAGER_CACHE:
            calls = self.__dict__.setdefault("_eager", common.EagerCalls())
            key = calls.key(self, idx, stream)
            hit = calls.get(key)
            if hit is None:
                hit = self._eager_build(category)
                if hit is None:
                    return None
                calls.put(key, hit)
        else:
            hit = self._eager_build(category)
            if hit is None:
                return None
        launches, fm_slots, ep, B, _keep = hit
        fm1 = torch.empty(B, 1, device=dev, dtype=torch.float32)
        fm2 = torch.empty(B, 1, device=dev, dtype=torch.float32)
        deep = torch.empty(B, 1, device=dev, dtype=torch.float32)
        total = torch.empty(B, 1, device=dev, dtype=torch.float32)
        prob = torch.empty(B, 1, device=dev, dtype=torch.float32)
        front = launches[0][1]
        front[fm_slots[0]], front[fm_slots[1]] = fm1.data_ptr(), fm2.data_ptr()
        ep.fm1, ep.fm2, ep.head_aux = fm1.data_ptr(), fm2.data_ptr(), deep.data_ptr()
        ep.head_logit, ep.head_prob = total.data_ptr(), prob.data_ptr()
        common.run_launches(launches, stream)
        return prob, total, fm1, fm2, deep

    def _eager_build(self, category):
        """(launches, fm1/fm2 argument slots of launches[0], head epilogue, B, keep-alive objects)."""
        names = list(self.second_order_embeddings)
        first = category[names[0]]
        B, dev, D = first.shape[0], first.device, self.embedding_dim
        head_kwargs = dict(final_w=self.final_layer.weight, final_b=self.final_layer.bias)
        widths = [l.linear.out_features for l in self._tail]
        if (FUSED_WHOLE and PACKED_TABLES and first.dim() == 1 and len(names) <= 32
                and ops.deepfm_whole_plan(len(names) * D, widths)):
            whole = self._whole_build(names, category, head_kwargs)
            if whole is not None:
                return whole
        l0, fused = self._tail[0], None
        if FUSED_FRONT and len(self._tail) >= 2 and len(names) <= 32 and first.dim() == 1:
            w0 = common.PACKED(l0.linear.weight)
            ml0 = ops.make_mlp_layer(l0.linear.weight, w0, **l0.epilogue_kwargs())
            fused = common.tiled_layer(len(names) * D, B, dev, ml0)
        plan = self._gather_plan(names, category, deep=not fused)
        packed, second, first, D, B, deep_in, fm1, fm2 = plan
        if not packed or any(t.data_ptr() != category[n].data_ptr() for t, n in zip(first, names)):
            return None  # unpacked tables, or contiguous copies of the indices: the uncached path
        ops._lib.ensure_device(dev)
        arr = ops._seg_array(second)
        if fused:  # rk_fm_linear_packed (gather, fm1, fm2, deep layer 0) + the rest of the tail
            y = torch.empty(B, l0.linear.out_features, device=dev, dtype=torch.float32)
            tail = common.tail_launches(y, self._tail[1:], self.deep_output_layer, head_kwargs)
            if tail is None:
                return None
            tl, ep, keep = tail
            front = ["rk_fm_linear_packed", [arr, len(second), D, B, ops.ctypes.byref(ml0), y.data_ptr(), y.stride(0),
                                             None, None, None]]
            # keep-alive: what the argument blocks point into (not the caller's index tensors: the
            # cache key's address / shape / stride check makes those pointers valid on a hit)
            return [front] + tl, (7, 8), ep, B, (keep, arr, self._images(names), w0, ml0, y)
        tail = common.tail_launches(deep_in, self._tail, self.deep_output_layer, head_kwargs)
        if tail is None:
            return None
        tl, ep, keep = tail
        gather = ["rk_fm_gather_packed", [arr, len(second), D, B, deep_in.data_ptr(), deep_in.stride(0), None, None,
                                          None]]
        return [gather] + tl, (6, 7), ep, B, (keep, arr, self._images(names), deep_in)

    def _images(self, names):
        """The device tensors a marshalled launch points into beyond its arguments: the packed FM
        tables and the folded BatchNorm affines.  A cache rebuild (a later .eval()/.train() or a
        weight change) replaces them, so a prepared run() must keep its own references."""
        return ([self.packed_table(n) for n in names],
                [l.epilogue_kwargs() for l in self._tail])

    def _whole_build(self, names, category, head_kwargs):
        """rk_deepfm_forward's launch (gather, FM, deep layers, head in one): the _eager_build tuple,
        or None off its path."""
        plan = self._gather_plan(names, category, deep=False)
        packed, second, first, D, B, _, fm1, fm2 = plan
        if not packed or any(t.data_ptr() != category[n].data_ptr() for t, n in zip(first, names)):
            return None
        dev = fm1.device
        ops._lib.ensure_device(dev)
        arr = ops._seg_array(second)
        weights = [common.PACKED(l.linear.weight) for l in self._tail]
        kws = [l.epilogue_kwargs() for l in self._tail]
        mls = [ops.make_mlp_layer(l.linear.weight, w, **kw) for l, w, kw in zip(self._tail, weights, kws)]
        la = (ops._lib.MlpLayer * len(mls))(*mls)
        ep = ops.make_epilogue(head_w=self.deep_output_layer.weight, head_b=self.deep_output_layer.bias,
                               **head_kwargs)
        launch = ["rk_deepfm_forward", [arr, len(second), D, B, la, len(mls), ops.ctypes.byref(ep), None, None, None]]
        return [launch], (7, 8), ep, B, (arr, self._images(names), weights, kws, mls, la)

    def prepare(self, category):
        """An eval forward bound to these input tensors (as DIN.prepare: the single-kernel analogue of
        capturing the forward in a hipGraph): returns `run()` that recomputes the whole forward from
        the current contents of the inputs with the cached launches (one rk_deepfm_forward at
        configs[1]'s shape) and returns the same (prob, total, fm1, fm2, deep) tensors each time.
        Binds the current weights: prepare again after changing them."""
        if self.training:
            raise RuntimeError("DeepFM.prepare: eval mode only (call .eval() first)")
        hit = self._eager_build(category)
        if hit is None:
            raise RuntimeError("DeepFM.prepare: configuration outside the cached eval path")
        launches, fm_slots, ep, B, keep = hit
        for l in self._tail:  # the images the plan binds are never rewritten in place under it
            common.PACKED.pin(l.linear.weight)
        dev = category[next(iter(self.second_order_embeddings))].device
        out = tuple(torch.empty(B, 1, device=dev, dtype=torch.float32) for _ in range(5))
        prob, total, fm1, fm2, deep = out
        front = launches[0][1]
        front[fm_slots[0]], front[fm_slots[1]] = fm1.data_ptr(), fm2.data_ptr()
        ep.fm1, ep.fm2, ep.head_aux = fm1.data_ptr(), fm2.data_ptr(), deep.data_ptr()
        ep.head_logit, ep.head_prob = total.data_ptr(), prob.data_ptr()
        stream = ops._lib.raw_stream(dev)
        lib = ops._lib.load()
        calls = []
        for name, args in launches:
            args[-1] = stream
            calls.append((name, getattr(lib, name), args))

        def run():
            for name, fn, args in calls:
                ops.check(fn(*args), name)
            return out
        run.keep = (keep, ep, category)
        return run

    def forward(self, category):
        first = category.get(next(iter(self.second_order_embeddings)), None) if isinstance(category, dict) else None
        if not self.training and isinstance(first, torch.Tensor) and first.shape[0] == 0:
            return common.empty_rows(ops.require_gpu(first, "category").device, 5)
        if not self.training:
            out = self._eager_eval(category)
            if out is not None:
                return out
        if self.training and not (torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())):
            check_eval(self)  # a train-mode forward without autograd is not implemented
        names = [c for c in self.second_order_embeddings if c in category]
        if len(names) != self.num_categories:
            missing = [c for c in self.second_order_embeddings if c not in category]
            raise KeyError(f"DeepFM.forward: category features missing: {missing}")
        if self.training:  # BatchNorm batch statistics, Dropout, HIP backward (rankops.train)
            idx = [ops.as_index(category[n], f"category[{n!r}]") for n in names]
            return train.deepfm_train_forward(self, names, idx)
        deep_in, fm1, fm2 = self._gather_fm(names, category)
        B, dev = deep_in.shape[0], deep_in.device
        deep = torch.empty(B, 1, device=dev, dtype=torch.float32)
        total = torch.empty(B, 1, device=dev, dtype=torch.float32)
        prob = torch.empty(B, 1, device=dev, dtype=torch.float32)
        head_kwargs = dict(fm1=fm1, fm2=fm2, final_w=self.final_layer.weight, final_b=self.final_layer.bias,
                           head_aux=deep)
        run_tail(deep_in, self._tail, self.deep_output_layer, head_kwargs, total, prob)
        return prob, total, fm1, fm2, deep
