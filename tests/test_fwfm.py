"""CPU tests of FwFM: the LabelEncoder bucketing restatement
(oracle/fwfm.py) pinned against pandas + scikit-learn themselves — the reference's own
dependencies, driven the way fwfm.py:29-31,48-67 drives them — then rankops.loader.label_encode
(C++ rk_label_encode) bit-exact against the oracle; the FwFM module's construction (parameter
order, shapes, state_dict keys, seeded values) against the reference's constructor
(fwfm.py:87-112).  Vocabularies are synthetic."""
import numpy as np
import pandas as pd
import pyarrow as pa
import pytest
import torch

import helpers as H  # noqa: F401
import rankops
from oracle import fwfm as of
from rankops.fwfm import FwFM
from rankops.loader import Vocabulary, label_encode

sk_pre = pytest.importorskip("sklearn.preprocessing")


def pandas_sklearn_encode(values, vocab):
    """The reference's pipeline for one feature, run on pandas + sklearn (fwfm.py:29-31, 48-67)."""
    with pd.option_context("future.no_silent_downcasting", True):
        series = pd.Series(values, dtype=object).astype(str).replace("None", np.nan)
    if not vocab:
        return series.fillna(0).astype(int).tolist()
    enc = sk_pre.LabelEncoder()
    enc.classes_ = np.array(vocab)
    modes = series.mode(dropna=True)
    mode_value = modes.values[0] if not modes.empty else "unknown"
    filled = series.fillna(mode_value)
    filled = np.where(filled.isin(set(vocab)), filled, mode_value)
    return enc.transform(filled).tolist()


VOCAB = ["f_3", "f_1", "", "f_3", "f_9", "unknown_not", "f_é"]
CASES = {
    "plain": ["f_1", "f_9", "f_3", "f_9"],
    "dup_last_wins": ["f_3", "f_3", "f_1"],
    "empty_string_value": ["", "", "f_1"],
    "nulls_fill_mode": [None, "f_9", "f_9", None, "f_1"],
    "none_string_is_nan": ["None", "f_1", "None", "None"],
    "oov_to_mode": ["zzz", "f_1", "f_1", "qq", "f_9"],
    "mode_tie_smallest": ["f_9", "f_1", "f_9", "f_1", "x"],
    "non_ascii": ["f_é", "f_é", "f_1"],
    "single": ["f_9"],
}
RAISE_CASES = {
    "mode_is_oov": ["zzz", "zzz", "f_1"],
    "all_nan_unknown_missing": [None, None, "None"],
    "tie_smallest_is_oov": ["a_oov", "f_1"],
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_encode_matches_pandas_sklearn(name):
    assert of.encode_column(CASES[name], VOCAB) == pandas_sklearn_encode(CASES[name], VOCAB)


@pytest.mark.parametrize("name", sorted(RAISE_CASES))
def test_oracle_encode_raises_like_sklearn(name):
    with pytest.raises(ValueError):
        pandas_sklearn_encode(RAISE_CASES[name], VOCAB)
    with pytest.raises(ValueError):
        of.encode_column(RAISE_CASES[name], VOCAB)


def test_oracle_all_nan_with_unknown_in_vocab():
    vocab = VOCAB + ["unknown"]
    vals = [None, "None"]
    assert of.encode_column(vals, vocab) == pandas_sklearn_encode(vals, vocab) == [7, 7]


def test_oracle_no_vocab_parses_ints():
    vals = ["12", " 3 ", "1_0", "-4", "+5", None]
    assert of.encode_column(vals, []) == pandas_sklearn_encode(vals, []) == [12, 3, 10, -4, 5, 0]


def _vocab(lines):
    return Vocabulary(text="".join(w + "\n" for w in lines).encode("utf-8"))


@pytest.mark.parametrize("name", sorted(CASES))
def test_label_encode_matches_oracle(name):
    got = label_encode(pa.array(CASES[name], type=pa.string()), _vocab(VOCAB))
    np.testing.assert_array_equal(got, of.encode_column(CASES[name], VOCAB))


@pytest.mark.parametrize("name", sorted(RAISE_CASES))
def test_label_encode_raises(name):
    with pytest.raises(ValueError, match="unseen labels"):
        label_encode(pa.array(RAISE_CASES[name], type=pa.string()), _vocab(VOCAB))


def test_label_encode_no_vocab_ints_and_errors():
    vals = ["12", " 3 ", "1_0", "-4", "+5", None, "9223372036854775807", "-9223372036854775808"]
    np.testing.assert_array_equal(label_encode(pa.array(vals), None), of.encode_column(vals, []))
    np.testing.assert_array_equal(label_encode(pa.array(vals), _vocab([])), of.encode_column(vals, []))
    for bad in ["1.0", "nan", "", "0x1", "1__0", "_1", "9223372036854775808"]:
        with pytest.raises(ValueError, match="invalid literal"):
            label_encode(pa.array(["1", bad]), None)


def test_label_encode_integer_column():
    """An integer column is str()-ed first (astype(str)); vocabulary lines are decimal strings."""
    vocab = ["10", "20", "30"]
    vals = [20, 30, 30, 99]
    np.testing.assert_array_equal(label_encode(pa.array(vals, type=pa.int64()), _vocab(vocab)),
                                  pandas_sklearn_encode(vals, vocab))


def test_label_encode_layouts():
    """large_string, sliced arrays with a validity offset, chunked columns, pandas input."""
    rng = np.random.default_rng(0)
    vals = [None if r < 0.1 else (f"oov_{r}" if r > 0.95 else f"f_{int(r * 40)}") for r in rng.random(3000)]
    vocab = [f"f_{i}" for i in range(40)] + ["f_3"]
    want = of.encode_column(vals[7:2900], vocab)
    v = _vocab(vocab)
    for arr in (pa.array(vals, type=pa.string()), pa.array(vals, type=pa.large_string())):
        np.testing.assert_array_equal(label_encode(arr.slice(7, 2893), v), want)
    chunked = pa.chunked_array([pa.array(vals[7:1000]), pa.array(vals[1000:2900])])
    np.testing.assert_array_equal(label_encode(chunked, v), want)
    np.testing.assert_array_equal(label_encode(pd.Series(vals[7:2900]), v), want)


@pytest.mark.parametrize("threads", [1, 3, 16])
def test_label_encode_wechat_size(threads):
    """A feedid-sized vocabulary (106,444 lines) over 200k rows with nulls, OOV values and a
    clear mode, split over several threads."""
    rng = np.random.default_rng(1)
    n_vocab = H.WECHAT_VOCAB["feedid"]
    vocab = [f"feedid_{i}" for i in rng.permutation(2 * n_vocab)[:n_vocab]]
    ids = rng.integers(0, n_vocab, 200_000)
    vals = [vocab[i] for i in ids]
    for i in rng.integers(0, len(vals), 5000):
        vals[i] = None
    for i in rng.integers(0, len(vals), 5000):
        vals[i] = f"feedid_oov_{i % 50}"
    for i in range(300):
        vals[i * 7] = vocab[123]  # the mode
    got = label_encode(pa.array(vals), _vocab(vocab), threads=threads)
    np.testing.assert_array_equal(got, of.encode_column(vals, vocab))


def test_label_encode_empty_column():
    assert label_encode(pa.array([], type=pa.string()), _vocab(VOCAB)).shape == (0,)


def test_fwfm_construction_matches_reference():
    """Same parameter creation order as fwfm.py:89-112: seeded, the drawn values coincide."""
    dims = [5, 7, 2, 4, 3, 6]
    torch.manual_seed(0)
    m = FwFM(dims, 8)
    torch.manual_seed(0)
    lin = [torch.nn.Embedding(n, 1) for n in dims]
    emb = [torch.nn.Embedding(n, 8) for n in dims]
    for e in emb:
        torch.nn.init.xavier_uniform_(e.weight)
    fw = torch.randn(15)
    sd = m.state_dict()
    # nn.Module lists its own parameters before its children's
    assert list(sd) == (["field_weight", "bias"] + [f"linear.{i}.weight" for i in range(6)]
                        + [f"embedding.{i}.weight" for i in range(6)])
    for i in range(6):
        assert torch.equal(sd[f"linear.{i}.weight"], lin[i].weight.detach())
        assert torch.equal(sd[f"embedding.{i}.weight"], emb[i].weight.detach())
    assert torch.equal(sd["field_weight"], fw)
    assert torch.equal(sd["bias"], torch.zeros(1))
    assert m.num_pairs == 15


def test_fwfm_requires_gpu_and_autograd_in_train():
    m = FwFM([3, 3, 3, 3, 3, 3], 8)
    x = {f: torch.zeros(4, dtype=torch.long) for f in of.FIELDS}
    with torch.no_grad(), pytest.raises(NotImplementedError):  # train mode without autograd
        m(x)
    with pytest.raises(RuntimeError, match="ROCm GPU"):  # train mode: the HIP backward path, GPU only
        m(x)
    m.eval()
    with pytest.raises(RuntimeError, match="ROCm GPU"):  # CPU tensors: the engine has no CPU path
        m(x)


def test_fwfm_oracle_forward_is_the_reference_formula():
    """The oracle's forward against an independent float64 evaluation of the FwFM formula."""
    torch.manual_seed(3)
    dims = [5, 7, 2, 4, 3, 6]
    m = FwFM(dims, 8)
    p = {k: v.detach() for k, v in m.state_dict().items()}
    x = {f: torch.randint(0, n, (32,)) for f, n in zip(of.FIELDS, dims)}
    prob, logit = of.forward(p, x)
    e = [p[f"embedding.{i}.weight"].double()[x[f]] for i, f in enumerate(of.FIELDS)]
    y = sum(p[f"linear.{i}.weight"].double()[x[f]][:, 0] for i, f in enumerate(of.FIELDS)) + p["bias"].double()
    k = 0
    for i in range(6):
        for j in range(i + 1, 6):
            y = y + p["field_weight"].double()[k] * (e[i] * e[j]).sum(1)
            k += 1
    torch.testing.assert_close(logit.double(), y, rtol=0, atol=1e-5)
    torch.testing.assert_close(prob.double(), torch.sigmoid(y), rtol=0, atol=1e-6)
