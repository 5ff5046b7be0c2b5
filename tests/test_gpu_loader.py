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
from test_loader import ARGS, _compare, _synthetic_rows, _synthetic_vocab_file, _table


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
@pytest.mark.parametrize("model", ["din", "bst", "dcn", "deepfm"])
def test_assembled_batch_feeds_forward(model, vocab):
    vocab_dir, words = vocab
    rows = _synthetic_rows(words, 700, seed=11, with_nulls=True)
    vocabs = rankops.wechat_vocabularies(vocab_dir)
    ovocabs = {f: ob.vocab_indices(ob.load_vocabulary(os.path.join(vocab_dir, ob.VOCAB_FILES[f])))
               for f in ob.VOCAB_FILES}
    want = ob.batch(model, rows, ovocabs, max_seq_length=50)
    asm = rankops.BatchAssembler(model, vocabs, device="cuda")
    got = asm(_table(rows))
    for name, g in zip(ARGS[model], got):
        if isinstance(g, dict):
            assert all(t.device.type == "cuda" for t in g.values())
        else:
            assert g.device.type == "cuda"
        _compare(g, want[name])

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
def test_double_buffered_batches_stay_independent(vocab):
    """Consecutive batches reuse the two pinned buffers; earlier results must not change."""
    vocab_dir, words = vocab
    vocabs = rankops.wechat_vocabularies(vocab_dir)
    asm = rankops.BatchAssembler("din", vocabs, device="cuda")
    outs = []
    for s in range(5):
        rows = _synthetic_rows(words, 300 + 17 * s, seed=100 + s)
        outs.append((rows, asm(_table(rows))))
    torch.cuda.synchronize()
    ovocabs = {f: ob.vocab_indices(ob.load_vocabulary(os.path.join(vocab_dir, ob.VOCAB_FILES[f])))
               for f in ob.VOCAB_FILES}
    for rows, got in outs:
        want = ob.batch("din", rows, ovocabs)
        for name, g in zip(ARGS["din"], got):
            _compare(g, want[name])
