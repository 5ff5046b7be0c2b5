"""CPU restatement of the reference's input bucketing (hazard H1) — TEST INFRASTRUCTURE ONLY.

Pure-Python restatement of the reference's Dataset vocabulary handling and collate functions,
used by tests/ (and bench.py's CPU leg) to check the C++ loader (rankops.loader / rk_bucketize*)
bit-exactly.  Never imported by the product path.  Parity unpinned: the reference ships no tests
for this code and may not be executed here; this follows its lines:

  _load_vocabulary        dcn.py:84-89 (same in din.py:121-126, deepfm.py:46-51,
                          deepcrossing.py:76-81, bst.py:29-33); AFM's variant drops lines that
                          strip to '' (afm.py:31-36)
  vocab_indices           dcn.py:69 ({v: i for i, v in enumerate(vocab)})
  category / target       dcn.py:100-104, din.py:138-143,158-163, bst.py:135-140,
                          deepfm.py:61-66, afm.py:51-55, deepcrossing.py:95-100
  DIN history             din.py:145-157 (str -> split(','), per-item feedid lookup)
  din_collate_fn          din.py:175-213 (zero padding to the batch maximum)
  BST sequence            bst.py:142-150 ([value], capped at max_seq_length, zero padded)
  dense                   dcn.py:97 / bst.py:133 (torch.tensor([row.get(f, 0.0) ...], float32)),
                          din.py:134-136 (one float32 scalar per feature)
"""
from __future__ import annotations

import numpy as np

DENSE_FEATURES = (
    "videoplayseconds", "u_read_comment_7d_sum", "u_like_7d_sum", "u_click_avatar_7d_sum",
    "u_forward_7d_sum", "u_comment_7d_sum", "u_follow_7d_sum", "u_favorite_7d_sum",
    "i_read_comment_7d_sum", "i_like_7d_sum", "i_click_avatar_7d_sum", "i_forward_7d_sum",
    "i_comment_7d_sum", "i_follow_7d_sum", "i_favorite_7d_sum", "c_user_author_read_comment_7d_sum")

# vocabulary file of each category field in the WechatDataset classes (dcn.py:59-67)
VOCAB_FILES = {"userid": "userid.txt", "feedid": "feedid.txt", "device": "device.txt",
               "authorid": "authorid.txt", "bgm_song_id": "bgm_song_id.txt",
               "bgm_singer_id": "bgm_singer_id.txt", "manual_tag_list": "manual_tag_id.txt"}
DCN_CATEGORY = ("userid", "device", "authorid", "bgm_song_id", "bgm_singer_id", "manual_tag_list")
DEEPFM_CATEGORY = ("userid", "feedid", "device", "authorid", "bgm_song_id", "bgm_singer_id")
AFM_CATEGORY = ("userid", "feedid", "device", "authorid", "bgm_song_id", "bgm_singer_id", "manual_tag_list")
DIN_SEQ = "his_read_comment_7d_seq"


def load_vocabulary(path, skip_empty=False):
    """dcn.py:84-89 / afm.py:33-35."""
    with open(path, "r") as f:
        if skip_empty:
            return [line.strip() for line in f if line.strip()]
        return [line.strip() for line in f]


def vocab_indices(vocab):
    """dcn.py:69."""
    return {v: i for i, v in enumerate(vocab)}


def lookup(indices, value):
    """dcn.py:101-104: the value as stored in the row, 0 when absent (H1)."""
    if value in indices:
        return indices[value]
    return 0


def din_history(indices, value, null="raise"):
    """din.py:147-157: returns the per-row index list (its length is the row's length).  A null
    cell of a present column: row.get returns it and `for item in seq` raises TypeError
    (din.py:147-151); null="empty" reads it as [] (the engine's opt-in null_history="empty")."""
    if value is None and null == "raise":
        raise TypeError("'NoneType' object is not iterable (din.py:147-151)")
    seq = [] if value is None else value
    if isinstance(seq, str):
        seq = seq.split(',')
    out = []
    for item in seq:
        if item in indices:
            out.append(indices[item])
        else:
            out.append(0)
    return out


def din_collate(histories):
    """din.py:185-213: [B, max_len] zero padded + lengths."""
    max_len = 0
    for h in histories:
        max_len = max(max_len, len(h))
    out = np.zeros((len(histories), max_len), dtype=np.int64)
    for i, h in enumerate(histories):
        out[i, :len(h)] = h
    return out, np.array([len(h) for h in histories], dtype=np.int64)


def bst_sequence(indices, value, max_seq_length):
    """bst.py:142-150."""
    seq = value
    if not isinstance(seq, list):
        seq = [seq]
    length = min(len(seq), max_seq_length)
    out = np.zeros(max_seq_length, dtype=np.int64)
    for i in range(length):
        if seq[i] in indices:
            out[i] = indices[seq[i]]
    return out, length


def dense_row(row):
    """dcn.py:97: torch.tensor([row.get(f, 0.0) ...], dtype=float32) — float64 -> float32 rounding."""
    return np.array([row.get(f, 0.0) for f in DENSE_FEATURES], dtype=np.float64).astype(np.float32)


def batch(model, rows, vocabs, max_seq_length=50, null_history="raise"):
    """The collated batch the reference's DataLoader hands to `model.forward` for `rows` (list of
    dicts of raw values), as numpy arrays keyed like the forward's arguments.  `vocabs` maps a
    field to its vocab_indices dict (AFM: built with skip_empty and without manual_tag_list,
    afm.py:31-36 — its Dataset looks for manual_tag_list.txt, which does not exist)."""
    if model in ("dcn", "deepcrossing"):
        return {"dense": np.stack([dense_row(r) for r in rows]),
                "category": {c: np.array([lookup(vocabs[c], r.get(c)) for r in rows], dtype=np.int64)
                             for c in DCN_CATEGORY}}
    if model == "deepfm":
        return {"category": {c: np.array([lookup(vocabs[c], r.get(c)) for r in rows], dtype=np.int64)
                             for c in DEEPFM_CATEGORY}}
    if model == "afm":
        return {"dense_input": np.stack([dense_row(r) for r in rows]),
                "category_input": {c: np.array([lookup(vocabs[c], r.get(c)) if c in vocabs else 0
                                                for r in rows], dtype=np.int64) for c in AFM_CATEGORY}}
    if model == "din":
        hist, lens = din_collate([din_history(vocabs["feedid"], r.get(DIN_SEQ), null_history) for r in rows])
        return {"dense": {f: np.array([r.get(f, 0.0) for r in rows], dtype=np.float64).astype(np.float32)
                          for f in DENSE_FEATURES},
                "category": {c: np.array([lookup(vocabs[c], r.get(c)) for r in rows], dtype=np.int64)
                             for c in DCN_CATEGORY},
                "sequence": {DIN_SEQ: hist, DIN_SEQ + "_length": lens},
                "target": {"feedid": np.array([lookup(vocabs["feedid"], r.get("feedid")) for r in rows],
                                              dtype=np.int64)}}
    if model == "bst":
        seqs = [bst_sequence(vocabs["feedid"], r.get("feedid", []), max_seq_length) for r in rows]
        return {"dense": np.stack([dense_row(r) for r in rows]),
                "category": {c: np.array([lookup(vocabs[c], r.get(c)) for r in rows], dtype=np.int64)
                             for c in DCN_CATEGORY},
                "seq_feedid": np.stack([s for s, _ in seqs]),
                "seq_length": np.array([n for _, n in seqs], dtype=np.int64)}
    raise ValueError(model)
