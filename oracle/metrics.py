"""TEST INFRASTRUCTURE ONLY — CPU restatement of the reference's evaluate() metrics.

Follows the reference's `evaluate()` (algorithm/DCN/dcn.py:214-239; the same loop in din.py:
365-393, bst.py:290-315, deepfm.py:187-210, afm.py:194-216, deepcrossing.py:201-224):
    avg_loss = sum over batches of BCEWithLogitsLoss(logits.squeeze(), label) / len(loader)
    accuracy = sklearn accuracy_score(labels, np.round(preds))
    auc      = sklearn roc_auc_score(labels, preds)
The AUC is restated as the Mann-Whitney U statistic with ties credited 1/2, which is the
trapezoidal area sklearn's roc_curve + auc produce; tests/test_metrics.py pins this restatement
against sklearn itself (scikit-learn is the reference's own dependency and is installed here).
Only tests/ and bench.py's CPU leg import this module.
"""
import numpy as np


def bce_with_logits_mean(logits, labels) -> float:
    """torch.nn.BCEWithLogitsLoss() (mean reduction): max(x,0) - x*y + log1p(exp(-|x|))."""
    x = np.asarray(logits, np.float64).reshape(-1)
    y = np.asarray(labels, np.float64).reshape(-1)
    return float(np.mean(np.maximum(x, 0) - x * y + np.log1p(np.exp(-np.abs(x)))))


def bce_mean(probs, labels) -> float:
    """torch.nn.BCELoss() (mean reduction), logs clamped at -100 as torch does."""
    p = np.asarray(probs, np.float64).reshape(-1)
    y = np.asarray(labels, np.float64).reshape(-1)
    with np.errstate(divide="ignore"):
        return float(np.mean(-(y * np.maximum(np.log(p), -100) + (1 - y) * np.maximum(np.log1p(-p), -100))))


def accuracy(labels, probs) -> float:
    """accuracy_score(labels, np.round(preds)); np.round is round-half-to-even."""
    return float(np.mean(np.round(np.asarray(probs, np.float32)) == np.asarray(labels, np.float32)))


def roc_auc(scores, labels) -> float:
    """Exact AUC = (sum over positives of #negatives below + 1/2 #negatives tied) / (P N).
    NaN for a NaN score or a single class (sklearn raises there)."""
    s = np.asarray(scores, np.float32).reshape(-1).astype(np.float64)
    pos = np.asarray(labels, np.float32).reshape(-1) > 0.5
    P, N = int(pos.sum()), int((~pos).sum())
    if P == 0 or N == 0 or np.isnan(s).any():
        return float("nan")
    order = np.argsort(s, kind="stable")
    s, pos = s[order], pos[order]
    starts = np.flatnonzero(np.r_[True, s[1:] != s[:-1]])
    gpos = np.add.reduceat(pos.astype(np.int64), starts)
    gneg = np.add.reduceat((~pos).astype(np.int64), starts)
    neg_before = np.cumsum(gneg) - gneg
    two_u = int(np.sum(gpos * (2 * neg_before + gneg)))
    return two_u / (2.0 * P * N)


def evaluate(batches, loss="bce_with_logits"):
    """batches: iterable of (logits, probs, labels, extra) -> (avg_loss, accuracy, auc); loss is
    "bce_with_logits" (dcn/bst/deepcrossing) or "bce" (din/deepfm/afm/fwfm); extra is the
    per-batch term added to the loss (DIN's l2_reg, din.py:380) or 0."""
    losses, probs, labels = [], [], []
    for x, p, y, extra in batches:
        losses.append((bce_with_logits_mean(x, y) if loss == "bce_with_logits" else bce_mean(p, y)) + float(extra))
        probs.append(np.asarray(p, np.float32).reshape(-1))
        labels.append(np.asarray(y, np.float32).reshape(-1))
    p, y = np.concatenate(probs), np.concatenate(labels)
    return sum(losses) / len(losses), accuracy(y, p), roc_auc(p, y)
