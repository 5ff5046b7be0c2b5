"""FwFM (field-weighted factorization machine) on the rankops engine — drop-in for
algorithm/FwFM/fwfm.py.

`FwFM(field_dims, embed_dim)` keeps the reference constructor, parameter creation order (so a
seeded construction draws the same weights) and state_dict keys (`linear.<f>.weight`,
`embedding.<f>.weight`, `field_weight`, `bias`; fwfm.py:87-112), and
`forward(x) -> sigmoid(y).squeeze(1)` over `x = {'userid', 'feedid', 'device', 'authorid',
'bgm_song_id', 'bgm_singer_id'}` int64 index tensors (fwfm.py:114-139).  Tables have
`len(vocab)` rows (no +1, fwfm.py:235-242); the indices come from the dataset-level
LabelEncoder bucketing in `rankops.loader.label_encode` (fwfm.py:48-67).

The whole forward — 12 gathers, the 15 weighted pair dots, the linear term, bias and sigmoid — is
one rk_fwfm_forward launch.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import common, ops, train
from .common import EngineModule, check_eval

FWFM_FIELDS = ("userid", "feedid", "device", "authorid", "bgm_song_id", "bgm_singer_id")


class FwFM(EngineModule):
    def __init__(self, field_dims, embed_dim, *, field_names=FWFM_FIELDS):
        super().__init__()
        self.field_dims = field_dims
        self.num_fields = len(field_dims)
        self.embed_dim = embed_dim
        if len(field_names) != self.num_fields:
            raise ValueError(f"FwFM: {self.num_fields} field_dims but {len(field_names)} field names")
        self.field_names = tuple(field_names)
        self.linear = nn.ModuleList([nn.Embedding(n, 1) for n in field_dims])
        self.embedding = nn.ModuleList([nn.Embedding(n, embed_dim) for n in field_dims])
        for emb in self.embedding:
            nn.init.xavier_uniform_(emb.weight)
        self.num_pairs = self.num_fields * (self.num_fields - 1) // 2
        self.field_weight = nn.Parameter(torch.randn(self.num_pairs), requires_grad=True)
        self.bias = nn.Parameter(torch.zeros(1))

    def _eager_eval(self, x, return_logit):
        """The eval forward through the EagerCalls cache (common.EagerCalls): one rk_fwfm_forward
        call with fresh outputs patched in; None off that path."""
        if not common.EAGER_CACHE:
            return None
        try:
            idx = [x[n] for n in self.field_names]
        except (KeyError, TypeError):
            return None
        if not all(isinstance(t, torch.Tensor) and t.dtype == torch.int64 and t.dim() == 1 for t in idx) \
                or idx[0].device.type != "cuda" or any(t.shape != idx[0].shape for t in idx):
            return None
        dev = idx[0].device
        stream = ops._lib.raw_stream(dev)
        calls = self.__dict__.setdefault("_eager", common.EagerCalls())
        key = calls.key(self, idx, stream)
        hit = calls.get(key)
        if hit is None:
            emb = [ops.table_segment(self.embedding[f].weight, t, 0) for f, t in enumerate(idx)]
            lin = [ops.table_segment(self.linear[f].weight, t, 0) for f, t in enumerate(idx)]
            ops._lib.ensure_device(dev)
            ea, la = ops._seg_array(emb), ops._seg_array(lin)
            args = [ea, la, len(emb), self.embed_dim, idx[0].shape[0], ops.as_f32(self.field_weight, "field_weight")
                    .data_ptr(), ops.as_f32(self.bias, "bias").data_ptr(), None, None, None]
            hit = calls.put(key, (args, idx[0].shape[0], (ea, la)))
        args, B, _keep = hit
        prob = torch.empty(B, device=dev, dtype=torch.float32)
        logit = torch.empty(B, device=dev, dtype=torch.float32) if return_logit else None
        args[7] = logit.data_ptr() if return_logit else None
        args[8], args[9] = prob.data_ptr(), stream
        ops.check(ops._lib.load().rk_fwfm_forward(*args), "rk_fwfm_forward")
        return (prob, logit) if return_logit else prob

    def prepare(self, x):
        """An eval forward bound to these index tensors (as DCNModel.prepare): returns `run()` that
        recomputes (prob, logit) [B] from the indices' current contents with one rk_fwfm_forward
        launch, into the same tensors each time.  The launch reads the parameters in place.  Index
        tensors must be int64 (bound by address, never copied)."""
        if self.training:
            raise RuntimeError("FwFM.prepare: eval mode only (call .eval() first)")
        idxs = [ops.bound_index(x[name], f"x[{name!r}]") for name in self.field_names]
        B, dev = idxs[0].shape[0], idxs[0].device
        emb = ops._seg_array([ops.table_segment(self.embedding[f].weight, idx, 0) for f, idx in enumerate(idxs)])
        lin = ops._seg_array([ops.table_segment(self.linear[f].weight, idx, 0) for f, idx in enumerate(idxs)])
        prob = torch.empty(B, device=dev, dtype=torch.float32)
        logit = torch.empty(B, device=dev, dtype=torch.float32)
        fw, bias = ops.as_f32(self.field_weight, "field_weight"), ops.as_f32(self.bias, "bias")
        ops._lib.ensure_device(dev)
        args = (emb, lin, len(idxs), self.embed_dim, B, fw.data_ptr(), bias.data_ptr(), logit.data_ptr(),
                prob.data_ptr(), ops._lib.stream_of(prob))
        fn, out = ops._lib.load().rk_fwfm_forward, (prob, logit)

        def run():
            ops.check(fn(*args), "rk_fwfm_forward")
            return out
        run.keep = (args, idxs, fw, bias, x)
        return run

    def forward(self, x, *, return_logit=False):
        """x: {field: int64 [B]} -> probabilities [B] (and the logits [B] with return_logit).
        Under .train() with autograd on, the probabilities carry the HIP backward (rankops.train)."""
        first = x.get(self.field_names[0], None) if isinstance(x, dict) else None
        if not self.training and isinstance(first, torch.Tensor) and first.shape[0] == 0:
            prob, logit = common.empty_rows(ops.require_gpu(first, "x").device, 2, shape=(0,))
            return (prob, logit) if return_logit else prob
        if not self.training:
            out = self._eager_eval(x, return_logit)
            if out is not None:
                return out
        if self.training and not (torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())):
            check_eval(self)  # a train-mode forward without autograd is not implemented
        idx0 = ops.as_index(x[self.field_names[0]], f"x[{self.field_names[0]!r}]")
        B = idx0.shape[0]
        emb, lin, idxs = [], [], []
        for f, name in enumerate(self.field_names):
            idx = ops.as_index(x[name], f"x[{name!r}]")
            if idx.shape != (B,):
                raise ValueError(f"FwFM.forward: x[{name!r}] has shape {tuple(idx.shape)}, expected ({B},)")
            idxs.append(idx)
        if self.training:  # the train Function marshals its own segments
            return train.fwfm_train_forward(self, idxs, return_logit)
        for f, idx in enumerate(idxs):
            emb.append(ops.table_segment(self.embedding[f].weight, idx, 0))
            lin.append(ops.table_segment(self.linear[f].weight, idx, 0))
        prob = torch.empty(B, device=idx0.device, dtype=torch.float32)
        logit = torch.empty(B, device=idx0.device, dtype=torch.float32) if return_logit else None
        ops.fwfm_forward(emb, lin, self.embed_dim, B, ops.as_f32(self.field_weight, "field_weight"),
                         ops.as_f32(self.bias, "bias"), logit, prob)
        return (prob, logit) if return_logit else prob
