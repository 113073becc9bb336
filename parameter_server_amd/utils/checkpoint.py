"""Model checkpoints.

Text layout (reference parity): ``<prefix>_<NodeID>`` holding one ``key\\tweight``
line per non-zero, non-NaN weight (src/parameter/kv_store.h:63-73,
src/learner/bcd.h:251-272); the directory is created if missing. Consumed by
ModelEvaluation (src/app/linear_method/model_evaluation.h:22-33).
Binary snapshot (new, for resume): safetensors of keys + optimizer state.
"""
from __future__ import annotations

import glob
import os
import re

import numpy as np
import torch


def write_text_model(path: str, keys, w) -> int:
    """``keys``: uint64 (or int64 bit pattern) tensor / array; ``w``: float tensor / array."""
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    k = keys.cpu().numpy() if isinstance(keys, torch.Tensor) else np.asarray(keys)
    v = w.cpu().numpy() if isinstance(w, torch.Tensor) else np.asarray(w)
    if v.dtype not in (np.float32, np.float64):
        v = v.astype(np.float32)
    keep = (v != 0) & ~np.isnan(v)
    k = k[keep].view(np.uint64) if k.dtype.itemsize == 8 else k[keep].astype(np.uint64)
    v = v[keep]
    order = np.argsort(k, kind="stable")
    with open(path, "w") as f:
        for kk, vv in zip(k[order], v[order]):
            f.write(f"{int(kk)}\t{float(vv):.9g}\n")
    return int(keep.sum())


def read_text_models(pattern: str) -> dict[int, float]:
    """Load every ``key\\tweight`` file matching a regex / glob (model_evaluation.h:22-33)."""
    files = sorted(glob.glob(pattern))
    if not files:
        d = os.path.dirname(pattern) or "."
        rx = re.compile(os.path.basename(pattern))
        files = sorted(os.path.join(d, f) for f in os.listdir(d) if rx.fullmatch(f) or rx.match(f))
    model: dict[int, float] = {}
    for fn in files:
        with open(fn) as f:
            for line in f:
                line = line.strip()
                if not line:
                    continue
                k, v = line.split("\t")
                model[int(k)] = float(v)
    return model


def save_snapshot(path: str, state: dict) -> None:
    from safetensors.torch import save_file

    tensors = {k: v.contiguous() for k, v in state.items() if isinstance(v, torch.Tensor)}
    meta = {k: str(v) for k, v in state.items() if not isinstance(v, torch.Tensor)}
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    save_file(tensors, path, metadata=meta)


def load_snapshot(path: str) -> dict:
    from safetensors import safe_open

    out = {}
    with safe_open(path, framework="pt") as f:
        for k in f.keys():
            out[k] = f.get_tensor(k)
        for k, v in (f.metadata() or {}).items():
            out[k] = int(v) if v.lstrip("-").isdigit() else v
    return out
