"""Single-machine evaluation metrics (reference src/util/evaluation.h:8-63).

``auc``: sort by prediction, area = sum over negatives of the positives ranked
below them, normalised, reported as ``max(a, 1-a)`` like the reference.
``accuracy``: label>0 & pred>threshold or label<0 & pred<=threshold, reported as
``max(acc, 1-acc)``. ``logloss`` is added (the trainers report it as the
objective). Works on numpy arrays or torch tensors (GPU tensors stay on the GPU:
the sort and the cumulative sums are device ops). Training-time AUC on the GPU
uses the histogram path in ops/linear.py instead of a sort.
"""
from __future__ import annotations

import numpy as np


def _np(x):
    if hasattr(x, "detach"):
        return x.detach().cpu().double().numpy()
    return np.asarray(x, dtype=np.float64)


def auc(label, predict) -> float:
    if hasattr(predict, "is_cuda") and predict.is_cuda:
        import torch

        order = torch.argsort(predict.double(), stable=True)
        pos = (label.reshape(-1)[order] > 0).double()
        cum_tp = torch.cumsum(pos, 0)
        area = float(((1 - pos) * cum_tp).sum())
        n, tp = pos.numel(), float(pos.sum())
    else:
        y, p = _np(label).reshape(-1), _np(predict).reshape(-1)
        pos = (y[np.argsort(p, kind="stable")] > 0).astype(np.float64)
        area = float(((1 - pos) * np.cumsum(pos)).sum())
        n, tp = pos.size, float(pos.sum())
    if tp == 0 or tp == n:
        return 1.0
    a = area / (tp * (n - tp))
    return 1 - a if a < 0.5 else a


def accuracy(label, predict, threshold: float = 0.0) -> float:
    y, p = _np(label).reshape(-1), _np(predict).reshape(-1)
    correct = ((y > 0) & (p > threshold)) | ((y < 0) & (p <= threshold))
    acc = float(correct.mean()) if y.size else 1.0
    return acc if acc > 0.5 else 1 - acc


def logloss(label, margin) -> float:
    """Mean log(1 + exp(-y m)) for labels in {-1, +1} (or {0, 1})."""
    y, m = _np(label).reshape(-1), _np(margin).reshape(-1)
    y = np.where(y > 0, 1.0, -1.0)
    return float(np.mean(np.logaddexp(0.0, -y * m))) if y.size else 0.0
