"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py) — FwFM restatement.

`encode_column` restates WechatDataset's string cleaning + _encode_features for one feature
(algorithm/FwFM/fwfm.py:29-31, 48-67) in plain Python: values are str()-ed, the string 'None'
(what astype(str) makes of a null) is NaN, NaN is filled with the column's mode
(`series.mode(dropna=True).values[0]`: most frequent, ties -> smallest), values outside the
vocabulary are replaced by the mode, then LabelEncoder.transform with classes_ = the vocabulary
lines maps every value to the position of its last occurrence (sklearn's _map_to_integer dict)
and raises ValueError for a value not among the classes.  tests/test_fwfm.py pins it against
pandas + scikit-learn themselves (the reference's dependencies, installed here).

`forward` restates FwFM.forward (fwfm.py:114-139) in torch fp32 on a state_dict-keyed parameter
dict, accumulating in the reference's order.  Parity of the forward is unpinned (no reference
fixtures for FwFM; the reference may not be imported here).
"""
from __future__ import annotations

from collections import Counter

import torch

FIELDS = ("userid", "feedid", "device", "authorid", "bgm_song_id", "bgm_singer_id")


def load_vocab(path_or_lines):
    """fwfm.py:40-46: [line.strip() for line in f.readlines()] — empty lines kept; missing file -> []."""
    if isinstance(path_or_lines, (list, tuple)):
        return list(path_or_lines)
    try:
        with open(path_or_lines, "r") as f:
            return [line.strip() for line in f.readlines()]
    except FileNotFoundError:
        return []


def encode_column(values, vocab):
    """values: list of str / None -> list of int (or ValueError like the reference)."""
    vals = [None if (v is None or str(v) == "None") else str(v) for v in values]
    if not vocab:  # fwfm.py:66-67: fillna(0).astype(int)
        return [0 if v is None else int(v) for v in vals]
    counts = Counter(v for v in vals if v is not None)
    if counts:
        top = max(counts.values())
        mode = min(k for k, c in counts.items() if c == top)
    else:
        mode = "unknown"
    vocab_set = set(vocab)
    filled = [mode if (v is None or v not in vocab_set) else v for v in vals]
    table = {val: i for i, val in enumerate(vocab)}
    out = []
    for v in filled:
        if v not in table:
            raise ValueError(f"y contains previously unseen labels: {v!r}")
        out.append(table[v])
    return out


def forward(p: dict, x: dict, fields=FIELDS):
    """fwfm.py:114-139 -> (prob [B], logit [B])."""
    F = len(fields)
    vals = [x[f] for f in fields]
    linear_terms = [p[f"linear.{i}.weight"][vals[i]] for i in range(F)]
    linear_sum = sum(linear_terms)
    emb = [p[f"embedding.{i}.weight"][vals[i]] for i in range(F)]
    quadratic_sum = 0
    pair = 0
    for i in range(F):
        for j in range(i + 1, F):
            quadratic_sum += p["field_weight"][pair] * torch.sum(emb[i] * emb[j], dim=1, keepdim=True)
            pair += 1
    y = linear_sum + quadratic_sum + p["bias"]
    return torch.sigmoid(y).squeeze(1), y.squeeze(1)
