"""GPU end-to-end of the host input path: raw rows -> rankops.BatchAssembler (C++ bucketing, one
pinned buffer, one H2D copy) -> the model forward.  The device tensors equal the reference
Dataset + collate restatement (oracle/bucketing.py) bit for bit, so the forward equals the
forward on the oracle-bucketed batch exactly."""
import os

import numpy as np
import pyarrow as pa
import pytest
import torch

import helpers as H
import rankops
from oracle import bucketing as ob
from test_loader import (ARGS, EDGE_VOCABS, HISTORIES, _compare, _oracle_vocab, _probe_values, _synthetic_rows,
                         _synthetic_vocab_file, _table)


@pytest.fixture(scope="module")
def vocab(tmp_path_factory):
    d = tmp_path_factory.mktemp("vocab_gpu")
    words = {}
    for f, n in H.SMALL_VOCAB.items():
        stem = ob.VOCAB_FILES[f][:-4]
        path, w = _synthetic_vocab_file(d, stem, n)
        words[f] = [x.replace(stem, f) for x in w]
        with open(path, "w") as fh:
            fh.write("".join(x + "\n" for x in words[f]))
    return str(d), words


def _to_torch(x, device):
    if isinstance(x, dict):
        return {k: _to_torch(v, device) for k, v in x.items()}
    return torch.from_numpy(np.ascontiguousarray(x)).to(device)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(EDGE_VOCABS))
def test_device_lookup_edge_vocabularies(tmp_path, name):
    """rk_bucketize_device probes the exported host table: same rows as the dict for every
    vocabulary-file edge case (sentinel first line so row 0 is unambiguous)."""
    path, words, idx = _oracle_vocab(tmp_path, name, b"sentinel\n" + EDGE_VOCABS[name], False)
    v = rankops.Vocabulary(path)
    probes = _probe_values(words)
    want = np.array([ob.lookup(idx, p) for p in probes], dtype=np.int64)
    np.testing.assert_array_equal(v.lookup_device(probes).cpu().numpy(), want)


@pytest.mark.gpu
def test_device_lookup_column_layouts(tmp_path):
    path, words = _synthetic_vocab_file(tmp_path, "feedid", 5000)
    idx = ob.vocab_indices(ob.load_vocabulary(path))
    v = rankops.Vocabulary(path)
    rng = np.random.default_rng(3)
    vals = [words[i] if i < len(words) else (None if i % 3 == 0 else f"feedid_x{i}")
            for i in rng.integers(0, len(words) + 500, size=20000)]
    want = np.array([ob.lookup(idx, x) for x in vals], dtype=np.int64)
    arr = pa.array(vals, type=pa.string())
    for col, w in ((arr, want), (pa.array(vals, type=pa.large_string()), want),
                   (arr.slice(777, 9000), want[777:9777]), (arr.slice(13, 5), want[13:18]),
                   (pa.chunked_array([arr.slice(0, 5), arr.slice(5)]), want),
                   (pa.array(np.arange(100)), np.zeros(100, np.int64))):
        np.testing.assert_array_equal(v.lookup_device(col).cpu().numpy(), w)


@pytest.mark.gpu
def test_device_history_sequences(tmp_path):
    """Wave-per-row separator scan: '', leading/trailing/double commas, nulls, a 300-item row,
    a 2000-item row (more than the 512 item starts one LDS pass holds) and T truncation."""
    path, words, idx = _oracle_vocab(tmp_path, "h", b"s\na\nb\nc\n\nzz\n", False)
    v = rankops.Vocabulary(path)
    rows = HISTORIES * 3 + [",".join(["a", "b", "zz", ""] * 500), "c," * 1999 + "a"]
    with pytest.raises(TypeError):
        v.lookup_sequences_device(pa.array(rows))
    want_seq, want_len = ob.din_collate([ob.din_history(idx, r, "empty") for r in rows])
    got_seq, got_len = v.lookup_sequences_device(pa.array(rows), null_history="empty")
    np.testing.assert_array_equal(got_len.cpu().numpy(), want_len)
    np.testing.assert_array_equal(got_seq.cpu().numpy(), want_seq)
    for T in (0, 1, 5, 600):
        s, n = v.lookup_sequences_device(pa.array(rows).slice(2), T=T, null_history="empty")
        np.testing.assert_array_equal(s.cpu().numpy(), want_seq[2:, :T] if T <= want_seq.shape[1] else
                                      np.pad(want_seq[2:], ((0, 0), (0, T - want_seq.shape[1]))))
        np.testing.assert_array_equal(n.cpu().numpy(), np.minimum(want_len[2:], T))


@pytest.mark.gpu
@pytest.mark.parametrize("bucketing", ["device", "host"])
@pytest.mark.parametrize("model", ["din", "bst", "dcn", "deepfm", "afm"])
def test_assembled_batch_feeds_forward(model, bucketing, vocab):
    vocab_dir, words = vocab
    rows = _synthetic_rows(words, 700, seed=11, with_nulls=True)
    skip = model == "afm"
    vocabs = rankops.wechat_vocabularies(vocab_dir, skip_empty_lines=skip)
    ovocabs = {f: ob.vocab_indices(ob.load_vocabulary(os.path.join(vocab_dir, ob.VOCAB_FILES[f]), skip))
               for f in ob.VOCAB_FILES}
    if model == "afm":
        ovocabs.pop("manual_tag_list")
    want = ob.batch(model, rows, ovocabs, max_seq_length=50, null_history="empty")
    asm = rankops.BatchAssembler(model, vocabs, device="cuda", bucketing=bucketing, null_history="empty")
    got = asm(_table(rows))
    for name, g in zip(ARGS[model], got):
        if isinstance(g, dict):
            assert all(t.device.type == "cuda" for t in g.values())
        else:
            assert g.device.type == "cuda"
        _compare(g, want[name])

    if model == "afm":  # AFM's forward takes a feature-column dict; the batch check above is the test
        return
    cfg = {"dcn": {}, "deepfm": {"fields": {f: H.SMALL_VOCAB[f] for f in ob.DEEPFM_CATEGORY}},
           "din": {"interaction_weights": "frozen"},
           "bst": {"dim": 128, "max_len": 50}}[model]
    m = H.build(model, cfg).cuda()
    ref_args = [_to_torch(want[n], "cuda") for n in ARGS[model]]
    with torch.no_grad():
        torch.manual_seed(1)
        a = m(*got)
        torch.manual_seed(1)
        b = m(*ref_args)
    for x, y in zip(H.as_tuple(a), H.as_tuple(b)):
        if isinstance(x, torch.Tensor):
            assert torch.equal(x, y) or torch.equal(torch.isnan(x), torch.isnan(y)) and torch.equal(
                torch.nan_to_num(x), torch.nan_to_num(y))
    assert rankops.error_flags() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("bucketing", ["device", "host"])
def test_double_buffered_batches_stay_independent(vocab, bucketing):
    """Consecutive batches reuse the two pinned buffers; earlier results must not change."""
    vocab_dir, words = vocab
    vocabs = rankops.wechat_vocabularies(vocab_dir)
    asm = rankops.BatchAssembler("din", vocabs, device="cuda", bucketing=bucketing, null_history="empty")
    outs = []
    for s in range(5):
        rows = _synthetic_rows(words, 300 + 17 * s, seed=100 + s)
        outs.append((rows, asm(_table(rows))))
    torch.cuda.synchronize()
    ovocabs = {f: ob.vocab_indices(ob.load_vocabulary(os.path.join(vocab_dir, ob.VOCAB_FILES[f])))
               for f in ob.VOCAB_FILES}
    for rows, got in outs:
        want = ob.batch("din", rows, ovocabs, null_history="empty")
        for name, g in zip(ARGS["din"], got):
            _compare(g, want[name])
