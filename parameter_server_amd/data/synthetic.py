"""Deterministic synthetic datasets for batch (Darlin) training and tests.

* ``sparse_classification`` — multi-group sparse data with a planted sparse
  logistic model (power-law key popularity per group, optional real values).
* ``sparse_groups`` — CTR-log-shaped data: many groups, a few present per example.
* ``criteo_slots`` — Criteo-shaped slots from the streaming generator
  (``ops.synthetic.criteo_batch``): 39 groups with one key per example each.
* ``write_text`` — dump as PS text (``label; grp k[:v] ...``) / LIBSVM files so the
  runtime apps can read them through the normal parsers.
"""
from __future__ import annotations

import numpy as np

from .slot_reader import SlotData


def sparse_classification(rows: int, groups=(1, 2, 3), keys_per_group: int = 1000,
                          nnz_per_row=(1, 3, 5), binary: bool = True, seed: int = 0,
                          w_density: float = 0.1, alpha: float = 1.2, noise: float = 0.5,
                          key_offset: int = 0) -> SlotData:
    rng = np.random.default_rng(seed)
    labels_margin = np.zeros(rows)
    sd = SlotData(labels=np.zeros(rows, np.float32))
    for gi, g in enumerate(groups):
        k = nnz_per_row[gi % len(nnz_per_row)]
        # power-law popularity: rank r drawn with p ~ 1/(r+1)^alpha
        p = 1.0 / np.arange(1, keys_per_group + 1) ** alpha
        p /= p.sum()
        ids = rng.choice(keys_per_group, size=(rows, k), p=p)
        keys = np.sort(ids, axis=1).reshape(-1).astype(np.uint64) * np.uint64(7) \
            + np.uint64(key_offset + g * 1_000_003)
        wg = np.where(rng.random(keys_per_group) < w_density, rng.normal(0, 2, keys_per_group), 0)
        vals = None if binary else rng.uniform(0.2, 1.5, rows * k).astype(np.float32)
        contrib = wg[ids.reshape(-1)] * (1.0 if vals is None else vals)
        labels_margin += contrib.reshape(rows, k).sum(1)
        off = np.arange(rows + 1, dtype=np.int64) * k
        sd.groups[g] = (off, keys, vals)
    pr = 1 / (1 + np.exp(-(labels_margin + rng.normal(0, noise, rows))))
    sd.labels = np.where(rng.random(rows) < pr, 1.0, -1.0).astype(np.float32)
    return sd


def sparse_groups(rows: int, groups: int = 120, present: int = 8, keys_per_group: int = 20000,
                  nnz_per_group: int = 2, seed: int = 0, w_density: float = 0.05,
                  alpha: float = 1.1, noise: float = 0.5) -> SlotData:
    """ADFEA / CTR-log-shaped slots: many feature groups, each example carrying keys of
    only ``present`` of them (``nnz_per_group`` distinct keys each, power-law
    popularity), as in the reference's batch CTR workload (group ids into the hundreds,
    e.g. prior groups 127 / 120 of example/linear/ctr/batch_l1lr.conf). Unlike the
    one-hot Criteo slots, two blocks of different groups share few examples, which is
    what lets Darlin's bounded block delay (tau blocks in flight against stale margins)
    converge."""
    from math import gcd

    rng = np.random.default_rng(seed)
    present = min(present, groups)
    # the example's groups: base + j * step (mod groups) with step coprime to groups
    steps = np.array([s for s in range(1, groups) if gcd(s, groups) == 1] or [1])
    base = rng.integers(0, groups, rows)
    step = steps[rng.integers(0, steps.size, rows)]
    member = (base[:, None] + np.arange(present)[None, :] * step[:, None]) % groups
    g_of = member.reshape(-1)
    r_of = np.repeat(np.arange(rows), present)
    order = np.lexsort((r_of, g_of))
    g_of, r_of = g_of[order], r_of[order]
    starts = np.searchsorted(g_of, np.arange(groups + 1))
    margin = np.zeros(rows)
    p = 1.0 / np.arange(1, keys_per_group + 1) ** alpha
    p /= p.sum()
    K = keys_per_group + nnz_per_group
    sd = SlotData(labels=np.zeros(rows, np.float32))
    for g in range(groups):
        rws = r_of[starts[g]:starts[g + 1]]  # sorted example ids holding group g
        cnt = np.zeros(rows, np.int64)
        cnt[rws] = nnz_per_group
        off = np.zeros(rows + 1, np.int64)
        np.cumsum(cnt, out=off[1:])
        ids = rng.choice(keys_per_group, size=(rws.size, nnz_per_group), p=p)
        ids.sort(axis=1)  # distinct, sorted keys within an example (the reference's rows)
        for c in range(1, nnz_per_group):
            ids[:, c] = np.maximum(ids[:, c], ids[:, c - 1] + 1)
        wg = np.where(rng.random(K) < w_density, rng.normal(0, 2, K), 0)
        margin[rws] += wg[ids].sum(1)
        keys = ids.reshape(-1).astype(np.uint64) * np.uint64(7) + np.uint64((g + 1) * 1_000_003)
        sd.groups[g + 1] = (off, keys, None)
    pr = 1 / (1 + np.exp(-(margin + rng.normal(0, noise, rows))))
    sd.labels = np.where(rng.random(rows) < pr, 1.0, -1.0).astype(np.float32)
    return sd


def criteo_slots(rows: int, *, seed: int = 0, row0: int = 0, num_features: int = 10 ** 9,
                 alpha: float = 1.1, device="cpu", on_device: bool = False) -> SlotData:
    """Criteo-shaped slot data: group s+1 holds slot s (one key per example).
    ``on_device``: keep the groups as device tensors (keys int64 = raw uint64 bits) for
    the GPU Darlin preprocessing, instead of host numpy arrays."""
    from ..ops.synthetic import NUM_SLOTS, criteo_batch

    keys, labels = criteo_batch(rows, seed=seed, row0=row0, num_features=num_features,
                                alpha=alpha, device=device)
    if on_device:
        import torch

        kd = keys.view(rows, NUM_SLOTS)
        sd = SlotData(labels=labels.cpu().numpy().astype(np.float32))
        off = torch.arange(rows + 1, dtype=torch.int64, device=keys.device)
        for s in range(NUM_SLOTS):
            sd.groups[s + 1] = (off, kd[:, s].contiguous(), None)
        return sd
    k = keys.view(rows, NUM_SLOTS).cpu().numpy().view(np.uint64)
    sd = SlotData(labels=labels.cpu().numpy().astype(np.float32))
    off = np.arange(rows + 1, dtype=np.int64)
    for s in range(NUM_SLOTS):
        sd.groups[s + 1] = (off, np.ascontiguousarray(k[:, s]), None)
    return sd


def write_text(sd: SlotData, path: str, fmt: str = "SPARSE_BINARY"):
    """PS text format (reference text_parser.cc:200-250): ``label; g k[:v] k ...; ...``
    or LIBSVM ``label k:v ...`` (groups merged)."""
    gids = sorted(sd.groups)
    with open(path, "w") as f:
        for i in range(sd.rows):
            y = 1 if sd.labels[i] > 0 else 0 if fmt != "LIBSVM" else -1
            parts = [str(y)]
            if fmt == "LIBSVM":
                items = []
                for g in gids:
                    off, keys, vals = sd.groups[g]
                    for j in range(off[i], off[i + 1]):
                        items.append((int(keys[j]), 1.0 if vals is None else float(vals[j])))
                items.sort()
                f.write(" ".join([str(y if y > 0 else -1)] + [f"{k}:{v:g}" for k, v in items]) + "\n")
                continue
            for g in gids:
                off, keys, vals = sd.groups[g]
                if off[i + 1] == off[i]:
                    continue
                if vals is None:
                    toks = [str(int(k)) for k in keys[off[i]:off[i + 1]]]
                else:
                    toks = [f"{int(k)}:{float(v):g}" for k, v in
                            zip(keys[off[i]:off[i + 1]], vals[off[i]:off[i + 1]])]
                parts.append(f"{g} " + " ".join(toks))
            f.write("; ".join(parts) + "\n")
