"""CPU: the evaluate() metric restatement (oracle/metrics.py) pinned against the reference's own
metric code path — sklearn.metrics (the reference's dependency, installed here) and torch's
BCEWithLogitsLoss / BCELoss — on random, tie-heavy and edge-case inputs."""
import numpy as np
import pytest
import torch

from oracle import metrics as om

sk = pytest.importorskip("sklearn.metrics")


def _cases():
    rng = np.random.default_rng(0)
    yield "random", rng.random(20000).astype(np.float32), (rng.random(20000) < 0.3).astype(np.float32)
    yield "ties", (rng.integers(0, 7, 5000) / 7).astype(np.float32), (rng.random(5000) < 0.5).astype(np.float32)
    yield "all_tied", np.full(100, 0.25, np.float32), (np.arange(100) % 3 == 0).astype(np.float32)
    yield "perfect", np.linspace(0, 1, 64, dtype=np.float32), (np.arange(64) >= 32).astype(np.float32)
    yield "inverted", np.linspace(1, 0, 64, dtype=np.float32), (np.arange(64) >= 32).astype(np.float32)
    s = rng.normal(size=3000).astype(np.float32)
    s[:10], s[10:20] = -0.0, 0.0
    yield "signed_zero", s, (rng.random(3000) < 0.5).astype(np.float32)
    yield "two", np.array([0.1, 0.9], np.float32), np.array([0.0, 1.0], np.float32)


@pytest.mark.parametrize("case", list(_cases()), ids=lambda c: c[0])
def test_oracle_auc_matches_sklearn(case):
    _, s, y = case
    assert abs(om.roc_auc(s, y) - sk.roc_auc_score(y, s)) < 1e-12


def test_oracle_auc_degenerate_is_nan():
    assert np.isnan(om.roc_auc(np.random.rand(10), np.ones(10)))
    s = np.random.rand(10)
    s[2] = np.nan
    assert np.isnan(om.roc_auc(s, np.arange(10) % 2))


def test_oracle_losses_match_torch():
    rng = np.random.default_rng(3)
    x = rng.normal(scale=3, size=4096).astype(np.float32)
    y = (rng.random(4096) < 0.4).astype(np.float32)
    p = torch.sigmoid(torch.from_numpy(x))
    want = torch.nn.BCEWithLogitsLoss()(torch.from_numpy(x), torch.from_numpy(y)).item()
    assert abs(om.bce_with_logits_mean(x, y) - want) < 1e-6
    want = torch.nn.BCELoss()(p, torch.from_numpy(y)).item()
    assert abs(om.bce_mean(p.numpy(), y) - want) < 1e-5
    # saturated probabilities: torch clamps the logs at -100
    p = torch.tensor([0.0, 1.0, 0.0, 1.0])
    yy = torch.tensor([1.0, 0.0, 0.0, 1.0])
    assert abs(om.bce_mean(p.numpy(), yy.numpy()) - torch.nn.BCELoss()(p, yy).item()) < 1e-4


def test_oracle_accuracy_rounds_half_to_even():
    """np.round(0.5) == 0: a probability of exactly 0.5 predicts the negative class."""
    assert om.accuracy([0, 1, 1], [0.5, 0.5, 0.51]) == pytest.approx(2 / 3)
    assert om.accuracy([0, 1, 1], [0.5, 0.5, 0.51]) == sk.accuracy_score([0, 1, 1], np.round([0.5, 0.5, 0.51]))


def test_oracle_evaluate_matches_reference_loop():
    """evaluate(): mean over batches of the batch loss (+ DIN l2 term), accuracy / AUC over all rows."""
    rng = np.random.default_rng(4)
    batches = []
    for B in (512, 512, 100):
        x = rng.normal(size=B).astype(np.float32)
        batches.append((x, 1 / (1 + np.exp(-x.astype(np.float64))), (rng.random(B) < 0.5).astype(np.float32), 0.01))
    loss, acc, auc = om.evaluate(batches, loss="bce")
    crit = torch.nn.BCELoss()
    want = np.mean([crit(torch.tensor(p), torch.tensor(y, dtype=torch.float64)).item() + e for _, p, y, e in batches])
    assert abs(loss - want) < 1e-6
    ys = np.concatenate([b[2] for b in batches])
    ps = np.concatenate([b[1] for b in batches]).astype(np.float32)
    assert acc == sk.accuracy_score(ys, np.round(ps))
    assert abs(auc - sk.roc_auc_score(ys, ps)) < 1e-12
