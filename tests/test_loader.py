"""CPU tests of the host input path (rankops.loader over include/rankops_io.h) against the
pure-Python restatement of the reference's bucketing (oracle/bucketing.py): bit-exact int64
rows for every vocabulary-file edge case, Arrow column layout, DIN history and per-model batch.
The reference's own vocabulary files are not copied into this repository; the vocabularies here
are synthetic, in the same `<field>_<id>` format, at SMALL and wechat row counts."""
import os

import numpy as np
import pyarrow as pa
import pytest

import helpers as H
import rankops
from oracle import bucketing as ob

EDGE_VOCABS = {
    "plain": b"a\nb\nc\n",
    "duplicates": b"x\ny\nx\nz\ny\n",                     # last occurrence wins
    "empties": b"\n  \n\tz \n\nq\n",                      # '' and stripped keys
    "crlf_cr": b"p\r\nq\rr\n\rs",                          # universal newlines, no final newline
    "unicode_space": "　w \n v \n\x1cu\x1f\n\u0085t \n k \n m \n"
                     .encode("utf-8"),
    "not_space": "​zw\n﻿bom\n᠎mv\n".encode("utf-8"),  # ZWSP, BOM, U+180E are kept
    "non_ascii": "用户_1\nfeedé\n".encode("utf-8"),
    "empty_file": b"",
    "only_newlines": b"\n\n\r\n",
    "wechat_like": b"userid_8\nuserid_12\nuserid_13\n",
}


def _oracle_vocab(tmp_path, name, data, skip):
    p = tmp_path / f"{name}.txt"
    p.write_bytes(data)
    words = ob.load_vocabulary(str(p), skip_empty=skip)
    return str(p), words, ob.vocab_indices(words)


def _probe_values(words):
    probes = list(dict.fromkeys(words)) + ["", " ", "a ", "nope", "userid_9", None, "x\n", "　w"]
    return probes


@pytest.mark.parametrize("sentinel", [False, True])
@pytest.mark.parametrize("skip", [False, True])
@pytest.mark.parametrize("name", sorted(EDGE_VOCABS))
def test_vocabulary_file_edge_cases(tmp_path, name, skip, sentinel):
    # row 0 is also the unknown-value row, so every case also runs with a plain first line
    data = (b"sentinel\n" if sentinel else b"") + EDGE_VOCABS[name]
    path, words, idx = _oracle_vocab(tmp_path, name, data, skip)
    v = rankops.Vocabulary(path, skip_empty_lines=skip)
    assert len(v) == len(words)
    probes = _probe_values(words)
    got = v.lookup(probes)
    want = np.array([ob.lookup(idx, p) for p in probes], dtype=np.int64)
    np.testing.assert_array_equal(got, want)
    # the in-memory parse is the same parse
    v2 = rankops.Vocabulary(text=data, skip_empty_lines=skip)
    assert len(v2) == len(words)
    np.testing.assert_array_equal(v2.lookup(probes), want)


def _synthetic_vocab_file(tmp_path, field, n, seed=0):
    rng = np.random.default_rng(seed + n)
    ids = rng.permutation(4 * n)[:n]
    p = tmp_path / f"{field}.txt"
    p.write_text("".join(f"{field}_{i}\n" for i in ids))
    return str(p), [f"{field}_{i}" for i in ids]


def test_column_layouts(tmp_path):
    path, words = _synthetic_vocab_file(tmp_path, "feedid", 5000)
    idx = ob.vocab_indices(ob.load_vocabulary(path))
    v = rankops.Vocabulary(path)
    rng = np.random.default_rng(3)
    vals = [words[i] if i < len(words) else (None if i % 3 == 0 else f"feedid_x{i}")
            for i in rng.integers(0, len(words) + 500, size=20000)]
    want = np.array([ob.lookup(idx, x) for x in vals], dtype=np.int64)
    arr = pa.array(vals, type=pa.string())
    np.testing.assert_array_equal(v.lookup(arr), want)
    np.testing.assert_array_equal(v.lookup(pa.array(vals, type=pa.large_string())), want)
    np.testing.assert_array_equal(v.lookup(arr.slice(777, 9000)), want[777:9777])          # offset slice
    np.testing.assert_array_equal(v.lookup(pa.chunked_array([arr.slice(0, 5), arr.slice(5)])), want)
    np.testing.assert_array_equal(v.lookup(arr.dictionary_encode()), want)
    np.testing.assert_array_equal(v.lookup(vals), want)                                    # Python list
    import pandas as pd
    np.testing.assert_array_equal(v.lookup(pd.Series(vals)), want)
    # int-typed values never equal the str keys of the reference's dicts -> 0
    np.testing.assert_array_equal(v.lookup(pa.array(np.arange(100))), np.zeros(100, np.int64))
    for threads in (1, 3, 16):
        np.testing.assert_array_equal(v.lookup(arr, threads=threads), want)


HISTORIES = ["", "a", "a,b", "a,,b", ",", "a,", ",a", None, "b,b,b,b", "zz,a,unknown,c",
             ",".join(["c"] * 300), " a", "a ,b"]


def test_din_history_sequences(tmp_path):
    path, words, idx = _oracle_vocab(tmp_path, "h", b"a\nb\nc\n\nzz\n", False)
    v = rankops.Vocabulary(path)
    rows = HISTORIES * 3
    # a null history raises as the reference's Dataset does (din.py:147-151) ...
    with pytest.raises(TypeError):
        v.lookup_sequences(rows)
    with pytest.raises(TypeError):
        ob.din_history(idx, None)
    # ... or reads as an empty history on request
    want_seq, want_len = ob.din_collate([ob.din_history(idx, r, "empty") for r in rows])
    got_seq, got_len = v.lookup_sequences(rows, null_history="empty")
    np.testing.assert_array_equal(got_len, want_len)
    np.testing.assert_array_equal(got_seq, want_seq)
    # capped width (BST-style truncation keeps the first T items and caps the length)
    got5, len5 = v.lookup_sequences(rows, T=5, null_history="empty")
    np.testing.assert_array_equal(got5, want_seq[:, :5])
    np.testing.assert_array_equal(len5, np.minimum(want_len, 5))
    big = [",".join(np.random.default_rng(i).choice(["a", "b", "c", "zz", "q"], size=i % 70)) for i in range(50000)]
    want_seq, want_len = ob.din_collate([ob.din_history(idx, r) for r in big])
    got_seq, got_len = v.lookup_sequences(pa.array(big))
    np.testing.assert_array_equal(got_len, want_len)
    np.testing.assert_array_equal(got_seq, want_seq)


def _synthetic_rows(vocab_words, B, seed, with_nulls=True):
    """Raw wechat-like rows: known ids, unknown ids, nulls; histories of 0..60 items."""
    rng = np.random.default_rng(seed)
    rows = []
    feed = vocab_words["feedid"]
    for i in range(B):
        r = {}
        for f, words in vocab_words.items():
            u = rng.random()
            if with_nulls and u < 0.03:
                r[f] = None
            elif u < 0.1:
                r[f] = f"{f}_unknown_{i}"
            else:
                r[f] = words[rng.integers(0, len(words))]
        n = int(rng.integers(0, 61))
        items = [feed[j] if j < len(feed) else "feedid_unk" for j in rng.integers(0, len(feed) + 20, size=n)]
        r[ob.DIN_SEQ] = None if (with_nulls and i % 97 == 5) else ",".join(items)
        for j, f in enumerate(ob.DENSE_FEATURES):
            r[f] = float(np.log1p(rng.poisson(2.0)) + 1e-9 * rng.random()) if rng.random() > 0.02 else float("nan")
        rows.append(r)
    return rows


def test_null_history_raises_like_the_reference(small_vocab):
    """din.py:147-151: row.get(col, []) returns a present column's null and iterating it raises
    TypeError; the assembler does the same by default, and reads it as [] with null_history="empty"."""
    vocab_dir, words = small_vocab
    vocabs = rankops.wechat_vocabularies(vocab_dir)
    rows = _synthetic_rows(words, 200, seed=3)
    assert any(r[ob.DIN_SEQ] is None for r in rows)
    with pytest.raises(TypeError, match="din.py:147-151"):
        rankops.BatchAssembler("din", vocabs, device="cpu")(_table(rows))
    oracle_vocabs = {f: ob.vocab_indices(ob.load_vocabulary(os.path.join(vocab_dir, ob.VOCAB_FILES[f])))
                     for f in ob.VOCAB_FILES}
    with pytest.raises(TypeError):
        ob.batch("din", rows, oracle_vocabs)
    clean = _synthetic_rows(words, 200, seed=3, with_nulls=False)
    got = rankops.BatchAssembler("din", vocabs, device="cpu")(_table(clean))
    want = ob.batch("din", clean, oracle_vocabs)
    for name, g in zip(ARGS["din"], got):
        _compare(g, want[name])
    with pytest.raises(ValueError):
        rankops.BatchAssembler("din", vocabs, device="cpu", null_history="skip")


def _table(rows):
    cols = {}
    for k in rows[0]:
        vals = [r[k] for r in rows]
        cols[k] = pa.array(vals, type=pa.float64() if k in ob.DENSE_FEATURES else pa.string())
    return pa.table(cols)


@pytest.fixture(scope="module")
def small_vocab(tmp_path_factory):
    d = tmp_path_factory.mktemp("vocab")
    words = {}
    for f, n in H.SMALL_VOCAB.items():
        path, w = _synthetic_vocab_file(d, ob.VOCAB_FILES[f][:-4], n)
        words[f] = [x.replace(ob.VOCAB_FILES[f][:-4], f) for x in w]
        # field values carry the field name; the file for manual_tag_list is manual_tag_id.txt
        with open(path, "w") as fh:
            fh.write("".join(x + "\n" for x in words[f]))
    return str(d), words


def _compare(got, want):
    if isinstance(want, dict):
        assert set(got) == set(want)
        for k in want:
            _compare(got[k], want[k])
        return
    g = got.cpu().numpy() if hasattr(got, "cpu") else np.asarray(got)
    assert g.shape == want.shape, (g.shape, want.shape)
    if want.dtype == np.float32:
        np.testing.assert_array_equal(g.view(np.int32), want.view(np.int32))  # bit-exact incl. NaN
    else:
        np.testing.assert_array_equal(g, want)


ARGS = {"dcn": ("dense", "category"), "deepcrossing": ("dense", "category"), "deepfm": ("category",),
        "afm": ("dense_input", "category_input"), "bst": ("dense", "category", "seq_feedid", "seq_length"),
        "din": ("dense", "category", "sequence", "target")}


@pytest.mark.parametrize("model", sorted(ARGS))
def test_batch_assembler_matches_reference_dataset(model, small_vocab):
    vocab_dir, words = small_vocab
    rows = _synthetic_rows(words, 1500, seed=sorted(ARGS).index(model))
    skip = model == "afm"
    vocabs = rankops.wechat_vocabularies(vocab_dir, skip_empty_lines=skip)
    oracle_vocabs = {f: ob.vocab_indices(ob.load_vocabulary(os.path.join(vocab_dir, ob.VOCAB_FILES[f]), skip))
                     for f in ob.VOCAB_FILES}
    if model == "afm":  # AFM's Dataset looks for manual_tag_list.txt (afm.py:31-36): absent
        oracle_vocabs.pop("manual_tag_list")
    want = ob.batch(model, rows, oracle_vocabs, max_seq_length=50, null_history="empty")
    asm = rankops.BatchAssembler(model, vocabs, device="cpu", null_history="empty")
    got = asm(_table(rows))
    assert len(got) == len(ARGS[model])
    for name, g in zip(ARGS[model], got):
        _compare(g, want[name])
    # a dict of Python lists gives the same batch, and buffers are reused across calls
    got2 = asm({k: [r[k] for r in rows] for k in rows[0]})
    for name, g in zip(ARGS[model], got2):
        _compare(g, want[name])


def test_wechat_size_vocabulary(tmp_path):
    """feedid at the wechat row count (106,444): 200k lookups, bit-exact with the dict."""
    path, words = _synthetic_vocab_file(tmp_path, "feedid", H.WECHAT_VOCAB["feedid"])
    v = rankops.Vocabulary(path)
    assert len(v) == H.WECHAT_VOCAB["feedid"]
    idx = ob.vocab_indices(ob.load_vocabulary(path))
    rng = np.random.default_rng(9)
    vals = [words[i] if i < len(words) else f"feedid_{10**9 + i}" for i in rng.integers(0, len(words) + 5000, 200000)]
    np.testing.assert_array_equal(v.lookup(pa.array(vals)), np.array([ob.lookup(idx, x) for x in vals]))


def test_io_invalid_arguments():
    lib = rankops.load_library()
    assert lib.rk_vocab_load(b"/nonexistent/vocab.txt", 0) is None
    assert "cannot open" in rankops._lib.last_error()
    assert lib.rk_bucketize(None, None, None, 32, None, 0, 4, None, 1, 0) != 0
    v = rankops.Vocabulary(text=b"a\n")
    assert lib.rk_bucketize(v._h, None, None, 16, None, 0, 1, None, 1, 0) != 0  # bad offset width
    assert lib.rk_vocab_size(None) == -1
