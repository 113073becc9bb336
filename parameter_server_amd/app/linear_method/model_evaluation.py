"""Offline model evaluation (scheduler only).

Reference ModelEvaluation (src/app/linear_method/model_evaluation.h:9-74): load
every ``key\\tw`` model file matching ``model_input.file`` (regex) into a hash map,
stream the validation data in 100k-row batches, compute Xw by hash lookup, and
log AUC and accuracy. Here the model lookup is a sorted-key join (vectorised).
"""
from __future__ import annotations

import sys

import numpy as np
import torch

from ...data import StreamReader, search_files
from ...ops.linear import exact_auc
from ...system.customer import App
from ...utils.checkpoint import read_text_models


def evaluate_model(model: dict, files, fmt, batch=100000):
    keys = np.array(sorted(model), dtype=np.uint64)
    w = np.array([model[int(k)] for k in keys], dtype=np.float64)
    scores, labels = [], []
    for b in StreamReader(files, fmt, batch, ignore_slot=True):
        pos = np.searchsorted(keys, b.keys)
        pos_c = np.minimum(pos, max(keys.size - 1, 0))
        hit = keys.size > 0
        wv = np.where(hit & (keys[pos_c] == b.keys), w[pos_c], 0.0) if keys.size else np.zeros(b.nnz)
        if b.vals is not None:
            wv = wv * b.vals
        rows = np.repeat(np.arange(b.rows), np.diff(b.row_ptr))
        xw = np.bincount(rows, weights=wv, minlength=b.rows)
        scores.append(xw)
        labels.append(b.labels)
    s = torch.from_numpy(np.concatenate(scores)) if scores else torch.zeros(0)
    y = torch.from_numpy(np.concatenate(labels)) if labels else torch.zeros(0)
    yy = torch.where(y > 0, 1.0, -1.0).double()
    acc = float(((yy * s) > 0).double().mean()) if s.numel() else float("nan")
    return {"auc": exact_auc(s, y) if s.numel() else float("nan"), "accuracy": acc,
            "examples": int(s.numel())}


class ModelEvaluation(App):
    def __init__(self, lm, name="app"):
        super().__init__(name, lm)
        self.lm = lm
        self.result = None

    def run(self):
        model = read_text_models(self.lm.model_input.file[0])
        print(f"loaded {len(model)} model entries", file=sys.stderr)
        files = search_files(self.lm.validation_data)
        self.result = evaluate_model(model, files, self.lm.validation_data.text)
        print(f"evaluation: auc {self.result['auc']:.6f} accuracy {self.result['accuracy']:.6f} "
              f"examples {self.result['examples']}", file=sys.stderr)
