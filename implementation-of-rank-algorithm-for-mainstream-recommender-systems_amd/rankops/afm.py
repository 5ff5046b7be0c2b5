"""AFM (Attentional Factorization Machine) on the rankops engine — drop-in for
algorithm/AFM/afm.py.

`AFM(feature_columns, embedding_dim, attention_factor)` and `create_feature_columns(vocab_dir)`
keep the reference signatures, creation order and state_dict keys (`dense_layer.*`,
`embeddings.<col>.weight`, `attention.0/2.*`, `p.*`; afm.py:64-90, 121-156) and
`forward(dense_input, category_input) -> (prediction, total_logit)` (afm.py:92-119).

The whole forward — 7 gathers, 21 pairwise Hadamard products, the attention MLP, the softmax
over pairs, the projection and the dense linear term — is one rk_afm_forward launch.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from . import common, ops, train
from .common import DENSE_FEATURES, EngineModule, check_eval


def create_feature_columns(vocabulary_dir):
    """Feature-column config (afm.py:121-156): manual_tag_list reads manual_tag_id.txt; the
    vocabulary keeps non-empty stripped lines."""
    feature_columns = {
        'dense': list(DENSE_FEATURES),
        'category': ["userid", "feedid", "device", "authorid", "bgm_song_id", "bgm_singer_id", "manual_tag_list"],
        'sequence': [],
        'vocab': {},
    }
    label_columns = ["read_comment"]
    column_to_vocab = {"manual_tag_list": "manual_tag_id"}
    for col in feature_columns['category']:
        path = os.path.join(vocabulary_dir, f"{column_to_vocab.get(col, col)}.txt")
        if os.path.exists(path):
            with open(path, 'r') as f:
                feature_columns['vocab'][col] = [line.strip() for line in f if line.strip()]
        else:
            feature_columns['vocab'][col] = []
    return feature_columns, label_columns


class AFM(EngineModule):
    def __init__(self, feature_columns, embedding_dim, attention_factor):
        super().__init__()
        self.feature_columns = feature_columns
        self.embedding_dim = embedding_dim
        self.attention_factor = attention_factor
        self.dense_features = feature_columns['dense']
        self.num_dense = len(self.dense_features)
        self.dense_layer = nn.Linear(self.num_dense, 1)
        self.category_features = feature_columns['category']
        self.embeddings = nn.ModuleDict()
        for col in self.category_features:
            self.embeddings[col] = nn.Embedding(len(feature_columns['vocab'][col]) + 1, embedding_dim)
        self.num_fields = len(self.category_features)
        self.attention = nn.Sequential(
            nn.Linear(embedding_dim, attention_factor),
            nn.ReLU(),
            nn.Linear(attention_factor, 1),
        )
        self.p = nn.Linear(embedding_dim, 1)

    def forward(self, dense_input, category_input):
        if self.training and not (torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())):
            check_eval(self)  # a train-mode forward without autograd is not implemented
        dense_input = ops.as_f32(dense_input, "dense_input")
        B = dense_input.shape[0]
        dev = dense_input.device
        if B == 0 and not self.training:
            return common.empty_rows(dev, 2)
        fields, idxs = [], []
        for col in self.category_features:
            idx = ops.as_index(category_input[col], f"category_input[{col!r}]")
            fields.append(ops.table_segment(self.embeddings[col].weight, idx, 0))
            idxs.append(idx)
        if self.training:  # AFM has no BatchNorm / Dropout: the train forward is the eval math
            return train.afm_train_forward(self, dense_input.contiguous(), idxs)
        logit = torch.empty(B, 1, device=dev, dtype=torch.float32)
        pred = torch.empty(B, 1, device=dev, dtype=torch.float32)
        att1, att2 = self.attention[0], self.attention[2]
        ops.afm_forward(fields, self.embedding_dim, B, dense_input, self.dense_layer.weight, self.dense_layer.bias,
                        att1.weight, att1.bias, att2.weight, att2.bias, self.p.weight, self.p.bias, logit, pred)
        return pred, logit

    def prepare(self, dense_input, category_input):
        """An eval forward bound to these input tensors (as DCNModel.prepare: the single-kernel analogue
        of capturing the forward in a hipGraph): returns `run()` that recomputes the forward from the
        current contents of the inputs with one rk_afm_forward launch and returns the same
        (pred, logit) tensors each time.  The launch reads the parameters in place, so later weight
        updates are seen.  Index tensors must be int64 (bound by address, never copied)."""
        if self.training:
            raise RuntimeError("AFM.prepare: eval mode only (call .eval() first)")
        dense_input = ops.as_f32(dense_input, "dense_input")
        B, dev = dense_input.shape[0], dense_input.device
        idxs = [ops.bound_index(category_input[col], f"category_input[{col!r}]") for col in self.category_features]
        fields = [ops.table_segment(self.embeddings[col].weight, idx, 0)
                  for col, idx in zip(self.category_features, idxs)]
        logit = torch.empty(B, 1, device=dev, dtype=torch.float32)
        pred = torch.empty(B, 1, device=dev, dtype=torch.float32)
        att1, att2 = self.attention[0], self.attention[2]
        args = ops.afm_forward_args(fields, self.embedding_dim, B, dense_input, self.dense_layer.weight,
                                    self.dense_layer.bias, att1.weight, att1.bias, att2.weight, att2.bias,
                                    self.p.weight, self.p.bias, logit, pred)
        fn, out = ops._lib.load().rk_afm_forward, (pred, logit)

        def run():
            ops.check(fn(*args), "rk_afm_forward")
            return out
        run.keep = (args, fields, idxs, dense_input, category_input)
        return run
