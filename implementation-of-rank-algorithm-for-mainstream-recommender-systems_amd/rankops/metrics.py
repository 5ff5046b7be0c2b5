"""Evaluation metrics on the device.

The reference's `evaluate()` (dcn.py:214-239; identical in din.py, bst.py, deepfm.py, afm.py,
deepcrossing.py) copies every batch's probabilities and labels to the host
(`.cpu().numpy()`), then computes `avg_loss = sum(batch BCEWithLogitsLoss) / len(loader)`,
`accuracy_score(labels, np.round(preds))` and sklearn's `roc_auc_score(labels, preds)`.
Here the batches stay in HBM: `rk_eval_batch` accumulates the loss and the correct count per
batch, the predictions are appended to a device buffer, and `rk_auc` computes the exact AUC
(Mann-Whitney U with ties credited 1/2 — the trapezoid sklearn integrates) from a radix sort
and integer counts.  One host synchronisation per evaluation, at `result()`.

    acc = EvalAccumulator.for_model("dcn", device)
    for batch in loader:
        prob, logit = model(...)
        acc.add(prob, label, logits=logit)
    avg_loss, accuracy, auc = acc.result()

The loss is the one each script's criterion computes: BCEWithLogitsLoss on the logits for
dcn/bst/deepcrossing (dcn.py:274,229), BCELoss on the probabilities for din/deepfm/afm/fwfm
(din.py:434,379), DIN adding its per-batch l2_reg (din.py:380) — pass it as `extra`.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


def roc_auc(scores: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """Exact ROC AUC (sklearn.metrics.roc_auc_score for labels in {0, 1}) as a 0-d float64 device
    tensor; NaN when a score is NaN or only one class is present (sklearn raises)."""
    lib = _lib.load()
    s = scores.detach().reshape(-1).to(torch.float32).contiguous()
    y = labels.detach().reshape(-1).to(torch.float32).contiguous()
    if s.device.type != "cuda" or y.device != s.device:
        raise RuntimeError("rankops.roc_auc: scores and labels must be on the same ROCm device")
    if s.numel() != y.numel():
        raise ValueError(f"rankops.roc_auc: {s.numel()} scores vs {y.numel()} labels")
    n = s.numel()
    nb = ctypes.c_int64()
    _lib.check(lib.rk_auc_workspace_size(n, ctypes.byref(nb)), "rk_auc_workspace_size")
    ws = torch.empty(nb.value, dtype=torch.uint8, device=s.device)
    out = torch.empty((), dtype=torch.float64, device=s.device)
    _lib.check(lib.rk_auc(s.data_ptr(), y.data_ptr(), n, ws.data_ptr(), nb.value, out.data_ptr(),
                          _lib.stream_of(s)), "rk_auc")
    return out


LOSS_KINDS = {"bce_with_logits": 0, "bce": 1}
MODEL_LOSS = {"dcn": "bce_with_logits", "bst": "bce_with_logits", "deepcrossing": "bce_with_logits",
              "din": "bce", "deepfm": "bce", "afm": "bce", "fwfm": "bce"}


class EvalAccumulator:
    """Device-side replacement for the evaluate() bookkeeping: loss / accuracy / AUC over all
    batches with no per-batch host copy."""

    @classmethod
    def for_model(cls, model: str, device="cuda"):
        return cls(device, loss=MODEL_LOSS[model.lower()])

    def __init__(self, device="cuda", loss="bce_with_logits"):
        if loss not in LOSS_KINDS:
            raise ValueError(f"EvalAccumulator: loss must be one of {sorted(LOSS_KINDS)}, got {loss!r}")
        self.loss_kind = LOSS_KINDS[loss]
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self._acc = torch.zeros(3, dtype=torch.float64, device=self.device)  # [loss sum | uint64 | uint64]
        self._probs = []
        self._labels = []
        self._n = 0

    def add(self, probs: torch.Tensor, labels: torch.Tensor, logits: torch.Tensor = None, extra=None):
        """One batch: probabilities, labels, the logits (needed for BCEWithLogitsLoss) and an
        optional per-batch scalar added to the batch loss (DIN's l2_reg)."""
        lib = _lib.load()
        p = probs.detach().reshape(-1).to(torch.float32).contiguous()
        y = labels.detach().reshape(-1).to(torch.float32).contiguous()
        if p.device != self.device or y.device != self.device:
            raise RuntimeError(f"EvalAccumulator.add: tensors must be on {self.device}")
        if p.numel() != y.numel() or p.numel() == 0:
            raise ValueError("EvalAccumulator.add: probs and labels must have the same non-zero size")
        x = None
        if self.loss_kind == 0:
            if logits is None:
                raise ValueError("EvalAccumulator.add: BCEWithLogitsLoss needs the logits")
            x = logits.detach().reshape(-1).to(torch.float32).contiguous()
            if x.numel() != p.numel() or x.device != self.device:
                raise ValueError("EvalAccumulator.add: logits must match probs")
        e = None
        if extra is not None and not (isinstance(extra, (int, float)) and extra == 0):
            e = torch.as_tensor(extra, dtype=torch.float32, device=self.device).detach().reshape(1).contiguous()
        _lib.check(lib.rk_eval_batch(x.data_ptr() if x is not None else None, p.data_ptr(), y.data_ptr(), p.numel(),
                                     self.loss_kind, e.data_ptr() if e is not None else None, self._acc.data_ptr(),
                                     _lib.stream_of(p)), "rk_eval_batch")
        self._keep = (x, e)  # alive until the kernel has read them (stream order)
        self._probs.append(p)
        self._labels.append(y)
        self._n += p.numel()

    def result(self):
        """(avg_loss, accuracy, auc) as Python floats, like evaluate()'s return values."""
        if not self._n:
            raise ValueError("EvalAccumulator: no batches")
        auc = roc_auc(torch.cat(self._probs), torch.cat(self._labels))
        acc = self._acc.cpu()
        counts = acc.view(torch.int64)
        loss_sum, correct, batches = float(acc[0]), int(counts[1]), int(counts[2])
        return loss_sum / batches, correct / self._n, float(auc)
