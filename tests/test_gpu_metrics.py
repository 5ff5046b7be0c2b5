"""GPU evaluation metrics (rankops.metrics over rk_eval_batch / rk_auc) against the reference's
own metric code path: sklearn.metrics.roc_auc_score / accuracy_score (scikit-learn, the
reference's dependency, installed here) and torch's BCEWithLogitsLoss, as evaluate() uses them
(dcn.py:214-239)."""
import numpy as np
import pytest
import torch

import rankops

sk = pytest.importorskip("sklearn.metrics")


def _cases():
    rng = np.random.default_rng(0)
    yield "random", rng.random(10000).astype(np.float32), (rng.random(10000) < 0.3).astype(np.float32)
    # heavy ties: scores on a coarse grid
    yield "ties", (rng.integers(0, 7, 5000) / 7).astype(np.float32), (rng.random(5000) < 0.5).astype(np.float32)
    yield "all_tied", np.full(100, 0.25, np.float32), (np.arange(100) % 3 == 0).astype(np.float32)
    yield "perfect", np.linspace(0, 1, 64, dtype=np.float32), (np.arange(64) >= 32).astype(np.float32)
    yield "inverted", np.linspace(1, 0, 64, dtype=np.float32), (np.arange(64) >= 32).astype(np.float32)
    s = rng.normal(size=3000).astype(np.float32)
    s[:10] = -0.0
    s[10:20] = 0.0
    s[20:25] = np.inf
    s[25:30] = -np.inf
    yield "signed_zero_inf", s, (rng.random(3000) < 0.5).astype(np.float32)
    yield "two", np.array([0.1, 0.9], np.float32), np.array([0.0, 1.0], np.float32)
    yield "large", rng.random(3_000_000).astype(np.float32), (rng.random(3_000_000) < 0.05).astype(np.float32)


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(_cases()), ids=lambda c: c[0])
def test_roc_auc_matches_sklearn(case):
    _, s, y = case
    got = float(rankops.roc_auc(torch.from_numpy(s).cuda(), torch.from_numpy(y).cuda()))
    # sklearn rejects +-inf; the AUC depends only on the order, so rank-preserving finite stand-ins
    fin = np.finfo(np.float32)
    want = sk.roc_auc_score(y, np.nan_to_num(s, posinf=fin.max, neginf=fin.min))
    assert abs(got - want) < 1e-12, (got, want)


@pytest.mark.gpu
def test_roc_auc_degenerate_is_nan():
    """sklearn raises for one class / NaN scores; the device AUC reports NaN."""
    s = torch.rand(50, device="cuda")
    assert np.isnan(float(rankops.roc_auc(s, torch.ones(50, device="cuda"))))
    s[3] = float("nan")
    assert np.isnan(float(rankops.roc_auc(s, (torch.arange(50, device="cuda") % 2).float())))


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["dcn", "din"])
def test_eval_accumulator_matches_reference_evaluate(model):
    """The evaluate() bookkeeping over ragged batches: mean of per-batch loss (BCEWithLogitsLoss on
    logits for dcn, BCELoss on probabilities + l2_reg for din), accuracy_score(labels,
    np.round(preds)) (0.5 rounds to 0), roc_auc_score."""
    rng = np.random.default_rng(1)
    crit = torch.nn.BCEWithLogitsLoss() if model == "dcn" else torch.nn.BCELoss()
    acc = rankops.EvalAccumulator.for_model(model, "cuda")
    total, labels, preds, nb = 0.0, [], [], 0
    for B in (4096, 4096, 1000, 7):
        logit = torch.from_numpy(rng.normal(scale=2.0, size=B).astype(np.float32))
        logit[:3] = 0.0  # sigmoid = 0.5 exactly: np.round -> 0
        label = torch.from_numpy((rng.random(B) < 0.4).astype(np.float32))
        prob = torch.sigmoid(logit)
        l2 = torch.tensor(0.0123 * (nb + 1)) if model == "din" else 0.0
        total += (crit(logit if model == "dcn" else prob, label) + l2).item()
        labels.extend(label.numpy())
        preds.extend(prob.numpy())
        nb += 1
        acc.add(prob.cuda(), label.cuda(), logits=logit.cuda(),
                extra=l2.cuda() if isinstance(l2, torch.Tensor) else l2)
    loss, accuracy, auc = acc.result()
    assert abs(loss - total / nb) < 1e-5
    assert accuracy == sk.accuracy_score(labels, np.round(preds))
    assert abs(auc - sk.roc_auc_score(labels, preds)) < 1e-12


@pytest.mark.gpu
def test_eval_accumulator_saturated_bce():
    """BCELoss clamps log(0) at -100 like torch."""
    acc = rankops.EvalAccumulator("cuda", loss="bce")
    p = torch.tensor([0.0, 1.0, 0.0, 1.0, 0.3])
    y = torch.tensor([1.0, 0.0, 0.0, 1.0, 1.0])
    acc.add(p.cuda(), y.cuda())
    loss, accuracy, auc = acc.result()
    assert abs(loss - torch.nn.BCELoss()(p, y).item()) < 1e-4
    assert accuracy == pytest.approx(2 / 5)


@pytest.mark.gpu
def test_eval_accumulator_invalid():
    with pytest.raises(ValueError):
        rankops.EvalAccumulator("cuda", loss="mse")
    acc = rankops.EvalAccumulator("cuda")
    with pytest.raises(ValueError):  # BCEWithLogitsLoss without logits
        acc.add(torch.rand(4, device="cuda"), torch.ones(4, device="cuda"))
    with pytest.raises(ValueError):
        acc.result()
