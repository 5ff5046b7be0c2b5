"""Builds the H1 bucketing fixture from the reference's own vocabulary files.

Reads, as text, the only reference-held data on the hot path's input side:
/root/reference/dataset/wechat_algo_data1/vocabulary/*.txt (7 files, 187,870 lines).  Writes

  tests/golden/wechat/wechat_vocab.npz      the file bytes (uint8, verbatim) and, per file, the expected
                                     row of every line looked up as a value (line position; the
                                     files hold no duplicates, so this is arange)
  tests/golden/wechat/wechat_rows.parquet   2,000 raw rows in the ETL's output format
                                     (DataGenerator.py:342-379): ids drawn from the real
                                     vocabularies, plus OOV ids, nulls, empty strings, multi-tag
                                     manual_tag_list values (comma-joined, DataGenerator.py:365-368)
                                     and feedid histories of 0..60 items (incl. '' and null)
  tests/golden/wechat/wechat_batches.npz    the batch each script's Dataset + collate hands to
                                     forward() for those rows, per model (dcn, deepcrossing,
                                     deepfm, din, bst, afm), from the CPU restatement
                                     oracle/bucketing.py of dcn.py:59-69,84-89,94-111,
                                     din.py:121-222, bst.py:127-159, deepfm.py:46-70,
                                     afm.py:31-62 (AFM's Dataset looks for manual_tag_list.txt,
                                     which does not exist, so that field is always row 0)

The semantics the tests pin against this data: index = line position, OOV -> 0 (colliding with
line 0), multi-tag manual_tag_list -> 0, empty history '' -> [0] with length 1, null history ->
length 0 (the engine's opt-in null_history="empty"; by default a null history raises TypeError as
din.py:147-151 does), and AFM's manual_tag_list always 0.  Run in the build container only:

    python tests/golden/wechat/make_wechat_bucketing.py
"""
import os
import sys

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(HERE))))

from oracle import bucketing as ob  # noqa: E402

VOCAB_DIR = "/root/reference/dataset/wechat_algo_data1/vocabulary"
ROWS = 2000
MODELS = ("dcn", "deepcrossing", "deepfm", "din", "bst", "afm")


def _rows(words, rng):
    """Raw rows: 80% known ids, then OOV ids, nulls, '' and whitespace variants per field."""
    rows = []
    feed, tags = words["feedid"], words["manual_tag_list"]
    for i in range(ROWS):
        r = {}
        for f, w in words.items():
            u = rng.random()
            if f == "manual_tag_list" and u < 0.35:
                k = int(rng.integers(2, 5))  # multi-tag row: never in the single-tag vocabulary
                r[f] = ",".join(tags[j] for j in rng.integers(0, len(tags), k))
            elif u < 0.80:
                r[f] = w[int(rng.integers(0, len(w)))]
            elif u < 0.86:
                r[f] = f"{f}_{10**7 + i}"           # well-formed but unknown id
            elif u < 0.90:
                r[f] = None
            elif u < 0.93:
                r[f] = ""
            elif u < 0.96:
                r[f] = " " + w[int(rng.integers(0, len(w)))]  # values are not stripped (dcn.py:101)
            else:
                r[f] = w[0]                            # line 0: same row as an unknown id
        n = int(rng.integers(0, 61))
        items = [feed[j] if j < len(feed) else f"feedid_unk{j}" for j in rng.integers(0, len(feed) + 200, n)]
        if i % 50 == 3:
            r[ob.DIN_SEQ] = ""                         # empty history -> [0], length 1
        elif i % 97 == 5:
            r[ob.DIN_SEQ] = None                       # no history -> length 0
        else:
            r[ob.DIN_SEQ] = ",".join(items)
        for f in ob.DENSE_FEATURES:
            r[f] = float(np.log1p(rng.poisson(2.0)))   # DataGenerator.py:361-363
        rows.append(r)
    return rows


def main():
    files = sorted(set(ob.VOCAB_FILES.values()))
    raw, expect, words = {}, {}, {}
    for fn in files:
        with open(os.path.join(VOCAB_DIR, fn), "rb") as fh:
            raw[fn] = fh.read()
        lines = ob.load_vocabulary(os.path.join(VOCAB_DIR, fn))
        idx = ob.vocab_indices(lines)
        assert len(idx) == len(lines), f"{fn}: duplicate lines"
        expect[fn] = np.array([ob.lookup(idx, v) for v in lines], dtype=np.int64)
        assert np.array_equal(expect[fn], np.arange(len(lines)))
    for f, fn in ob.VOCAB_FILES.items():
        words[f] = ob.load_vocabulary(os.path.join(VOCAB_DIR, fn))
    np.savez_compressed(os.path.join(HERE, "wechat_vocab.npz"),
                        **{f"bytes/{fn}": np.frombuffer(raw[fn], dtype=np.uint8) for fn in files},
                        **{f"expect/{fn}": expect[fn] for fn in files})

    rng = np.random.default_rng(20240614)
    rows = _rows(words, rng)
    cols = {k: pa.array([r[k] for r in rows], type=pa.float64() if k in ob.DENSE_FEATURES else pa.string())
            for k in rows[0]}
    pq.write_table(pa.table(cols), os.path.join(HERE, "wechat_rows.parquet"), compression="zstd")

    out = {}
    for model in MODELS:
        skip = model == "afm"
        vocabs = {f: ob.vocab_indices(ob.load_vocabulary(os.path.join(VOCAB_DIR, fn), skip))
                  for f, fn in ob.VOCAB_FILES.items()}
        if model == "afm":
            vocabs.pop("manual_tag_list")
        b = ob.batch(model, rows, vocabs, max_seq_length=50, null_history="empty")

        def put(prefix, v):
            if isinstance(v, dict):
                for k, x in v.items():
                    put(f"{prefix}/{k}", x)
            else:
                out[prefix] = v
        put(model, b)
    np.savez_compressed(os.path.join(HERE, "wechat_batches.npz"), **out)
    multi = sum(1 for r in rows if r["manual_tag_list"] and "," in r["manual_tag_list"])
    print(f"vocab files {len(files)}, lines {sum(len(e) for e in expect.values())}; rows {ROWS} "
          f"({multi} multi-tag manual_tag_list)")


if __name__ == "__main__":
    main()
