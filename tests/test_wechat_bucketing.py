"""H1 bucketing pinned to the reference's own data: the seven wechat_algo_data1 vocabulary files
(tests/golden/wechat/wechat_vocab.npz, verbatim bytes; made by tests/golden/wechat/make_wechat_bucketing.py) and
2,000 raw ETL-format rows (wechat_rows.parquet) with the batches each script's Dataset + collate
produces for them (wechat_batches.npz).

Semantics checked bit for bit, host (rk_bucketize*) and device (rk_bucketize*_device):
  index = line position                 dcn.py:69, din.py:102 ({v: i for i, v in enumerate(vocab)})
  OOV / null / '' -> 0                  dcn.py:101-104, din.py:140-143
  multi-tag manual_tag_list -> 0        the ETL comma-joins tags (DataGenerator.py:365-368); the
                                        vocabulary holds single tags
  '' history -> [0] with length 1       din.py:147-157 (''.split(',') == [''])
  null history -> TypeError             din.py:147-151 (row.get(col, []) returns a present column's
                                        null, and iterating it raises); null_history="empty" reads it as
                                        length 0, the mode the fixture's DIN batch was made in (a row
                                        WITHOUT the column gets [] in the reference)
  AFM manual_tag_list always 0          afm.py:31-36 (its Dataset opens manual_tag_list.txt,
                                        which does not exist)
  table rows = len(vocab) + 1           dcn.py:119-125"""
import os

import numpy as np
import pyarrow.parquet as pq
import pytest
import torch

import rankops
from oracle import bucketing as ob
from test_loader import ARGS, _compare

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "wechat")
LINES = {"userid.txt": 19626, "feedid.txt": 106444, "device.txt": 2, "authorid.txt": 18789,
         "bgm_song_id.txt": 25159, "bgm_singer_id.txt": 17500, "manual_tag_id.txt": 350}


@pytest.fixture(scope="module")
def wechat(tmp_path_factory):
    d = tmp_path_factory.mktemp("wechat_vocabulary")
    z = np.load(os.path.join(GOLDEN, "wechat_vocab.npz"))
    expect = {}
    for fn in LINES:
        (d / fn).write_bytes(z[f"bytes/{fn}"].tobytes())
        expect[fn] = z[f"expect/{fn}"]
    rows = pq.read_table(os.path.join(GOLDEN, "wechat_rows.parquet"))
    b = np.load(os.path.join(GOLDEN, "wechat_batches.npz"))
    batches = {}
    for key in b.files:
        parts = key.split("/")
        node = batches.setdefault(parts[0], {})
        for p in parts[1:-1]:
            node = node.setdefault(p, {})
        node[parts[-1]] = b[key]
    return str(d), expect, rows, batches


def _lines(path):
    with open(path) as fh:
        return [line.strip() for line in fh]


def test_vocabulary_files_index_is_line_position(wechat):
    vocab_dir, expect, _, _ = wechat
    vocabs = rankops.wechat_vocabularies(vocab_dir)
    for field, fn in ob.VOCAB_FILES.items():
        words = _lines(os.path.join(vocab_dir, fn))
        assert len(words) == LINES[fn] == len(expect[fn])
        v = vocabs[field]
        assert len(v) == LINES[fn]
        np.testing.assert_array_equal(v.lookup(words), expect[fn])
        # the oracle restatement agrees with the fixture too (it generated it from the same lines)
        idx = ob.vocab_indices(ob.load_vocabulary(os.path.join(vocab_dir, fn)))
        assert [idx[w] for w in words[:100]] == list(range(min(100, len(words))))
        assert rankops.common.table_rows(vocab_dir, field) == LINES[fn] + 1


def test_unknown_multitag_and_whitespace_probes(wechat):
    vocab_dir, _, _, _ = wechat
    vocabs = rankops.wechat_vocabularies(vocab_dir)
    tags = _lines(os.path.join(vocab_dir, "manual_tag_id.txt"))
    mt = vocabs["manual_tag_list"]
    probes = [tags[5], f"{tags[5]},{tags[6]}", f"{tags[0]},{tags[1]},{tags[2]}", "", None, " " + tags[5],
              tags[5] + " ", "manual_tag_id_999999", tags[5].upper()]
    np.testing.assert_array_equal(mt.lookup(probes), [5, 0, 0, 0, 0, 0, 0, 0, 0])
    feed = _lines(os.path.join(vocab_dir, "feedid.txt"))
    probes = ["", None, feed[7], f"{feed[7]},{feed[9]}", f"{feed[7]},,feedid_x", f",{feed[3]}"]
    with pytest.raises(TypeError):
        vocabs["feedid"].lookup_sequences(probes)
    seqs, lens = vocabs["feedid"].lookup_sequences(probes, null_history="empty")
    np.testing.assert_array_equal(lens, [1, 0, 1, 2, 3, 2])
    np.testing.assert_array_equal(seqs, [[0, 0, 0], [0, 0, 0], [7, 0, 0], [7, 9, 0], [7, 0, 0], [0, 3, 0]])


@pytest.mark.parametrize("model", sorted(ARGS))
def test_reference_vocabulary_batches_host(wechat, model):
    vocab_dir, _, rows, batches = wechat
    vocabs = rankops.wechat_vocabularies(vocab_dir, skip_empty_lines=model == "afm")
    if model == "din":  # the fixture holds null histories: the reference raises on them (din.py:147-151)
        with pytest.raises(TypeError):
            rankops.BatchAssembler(model, vocabs, device="cpu")(rows)
    asm = rankops.BatchAssembler(model, vocabs, device="cpu", null_history="empty")
    got = asm(rows)
    for name, g in zip(ARGS[model], got):
        _compare(g, batches[model][name])
    if model == "afm":
        assert not np.any(batches["afm"]["category_input"]["manual_tag_list"])
    if model == "din":
        seq_len = batches["din"]["sequence"][ob.DIN_SEQ + "_length"]
        assert seq_len.min() == 0 and seq_len.max() <= 60
        empty = [i for i, v in enumerate(rows.column(ob.DIN_SEQ).to_pylist()) if v == ""]
        assert empty and all(seq_len[i] == 1 for i in empty)


@pytest.mark.gpu
@pytest.mark.parametrize("bucketing", ["device", "host"])
@pytest.mark.parametrize("model", sorted(ARGS))
def test_reference_vocabulary_batches_gpu(wechat, model, bucketing):
    vocab_dir, _, rows, batches = wechat
    vocabs = rankops.wechat_vocabularies(vocab_dir, skip_empty_lines=model == "afm")
    asm = rankops.BatchAssembler(model, vocabs, device="cuda", bucketing=bucketing, null_history="empty")
    got = asm(rows)
    torch.cuda.synchronize()
    for name, g in zip(ARGS[model], got):
        _compare(g, batches[model][name])


@pytest.mark.gpu
def test_reference_vocabulary_device_lookup(wechat):
    vocab_dir, expect, _, _ = wechat
    vocabs = rankops.wechat_vocabularies(vocab_dir)
    for field, fn in ob.VOCAB_FILES.items():
        words = _lines(os.path.join(vocab_dir, fn))
        np.testing.assert_array_equal(vocabs[field].lookup_device(words).cpu().numpy(), expect[fn])
