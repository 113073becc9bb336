"""Synthetic Criteo-shaped minibatches (13 integer + 26 categorical slots).

Integer slots are log2-bucketised heavy-tailed counts; categorical slots draw
power-law ids over per-slot cardinalities and everything is hashed into
[0, num_features). Labels come from a planted sparse logistic model so the
training loss actually decreases. Deterministic in (seed, global row index):
the GPU kernel (``criteo_gen``) and this CPU path produce the same keys.
"""
from __future__ import annotations

import math

import torch

from .native import hipops, is_gpu

# Criteo Terabyte (24 days) per-slot cardinalities of the 26 categorical features
# (~0.88e9 distinct values in total): with 10^9 hashed features this is the
# "10^9-feature" regime of BASELINE.json.
CRITEO_1TB_CARDS = [227605432, 39060, 17295, 7424, 20265, 3, 7122, 1543, 63, 130229467,
                    3067956, 405282, 10, 2209, 11938, 155, 4, 976, 14, 292775614, 40790948,
                    187188510, 590152, 12973, 108, 36]
# Criteo Kaggle (display advertising challenge) cardinalities (~33.8M distinct).
CRITEO_KAGGLE_CARDS = [1460, 583, 10131227, 2202608, 305, 24, 12517, 633, 3, 93145, 5683,
                       8351593, 3194, 27, 14992, 5461306, 10, 5652, 2173, 4, 7046547, 18, 15,
                       286181, 105, 142572]
NUM_SLOTS = 39

_cards_set = {}


def gauss_table() -> list[float]:
    """Planted-weight quantiles 0.6 * Phi^-1((i + 0.5) / 256), f32 (shared by the GPU
    kernel, which holds them in constant memory, and the CPU reference)."""
    import statistics

    nd = statistics.NormalDist(0.0, 0.6)
    import numpy as np

    return [float(np.float32(nd.inv_cdf((i + 0.5) / 256))) for i in range(256)]


def _set_cards(device, cards):
    # per-call fast path: the same cards object on the same device (the tuple / str
    # key below costs ~8 us of host time, once per generated minibatch)
    hit = _cards_set.get(device)
    if hit is not None and hit[0] is cards:
        return
    key = (str(device), tuple(cards))
    if _cards_set.get(str(device)) != key:
        hipops().criteo_set_tables([int(c) for c in cards], gauss_table())
        _cards_set[str(device)] = key
    _cards_set[device] = (cards, key)


def criteo_batch(B: int, *, seed: int, row0: int, num_features: int, alpha: float = 1.1,
                 cards=CRITEO_1TB_CARDS, device="cpu", keys=None, labels=None, row0_dev=None,
                 row_scale: int = 1, row0_out=None):
    """Returns (keys int64 [B*39] row-major, labels float32 [B] in {-1,+1}).
    GPU only: ``row0_dev`` (int64[1] device) adds ``row0_dev * row_scale`` to ``row0``
    at kernel time, so a captured graph generates fresh rows on every replay;
    ``row0_out`` (int64[1] device, another word) receives ``row0_dev + 1``: two captured
    launches alternating the two words (A -> B, then B -> A) advance the cursor with no
    separate increment launch per replay."""
    device = torch.device(device)
    keys = torch.empty(B * NUM_SLOTS, dtype=torch.int64, device=device) if keys is None else keys
    labels = torch.empty(B, dtype=torch.float32, device=device) if labels is None else labels
    if device.type == "cuda":
        _set_cards(device, cards)
        hipops().criteo_gen(seed & ((1 << 64) - 1), row0, B, num_features, alpha, keys, labels,
                            row0_dev, row_scale, row0_out)
        return keys, labels
    k, l = _criteo_cpu(B, seed, row0, num_features, alpha, cards)
    keys.copy_(k)
    labels.copy_(l)
    return keys, labels


# ----------------------------------------------------------------------------- CPU path
def _mix32(x):
    """gen_mix32 of linear.hip on numpy uint32 arrays (wrapping arithmetic)."""
    import numpy as np

    x = x.astype(np.uint32)
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


def _fmix64(k):
    import numpy as np

    k = k.astype(np.uint64)
    k ^= k >> np.uint64(33)
    k *= np.uint64(0xFF51AFD7ED558CCD)
    k ^= k >> np.uint64(33)
    k *= np.uint64(0xC4CEB9FE1A85EC53)
    k ^= k >> np.uint64(33)
    return k


def _criteo_cpu(B, seed, row0, num_features, alpha, cards):
    """Vectorised reference of criteo_gen_kernel (linear.hip): same streams, hashes and
    tables. numpy's f32 log2 / exp2 may differ from the hardware v_log / v_exp in the
    last ulp, which moves a large power-law id (and so its key) for a few rows."""
    import numpy as np

    with np.errstate(over="ignore"):
        u32 = np.uint32
        gr = np.uint64(row0) + np.arange(B, dtype=np.uint64)
        lo, hi = gr.astype(np.uint32), (gr >> np.uint64(32)).astype(np.uint32)
        s_lo, s_hi = u32(seed & 0xFFFFFFFF), u32((seed >> 32) & 0xFFFFFFFF)
        sj = [_mix32(np.array([s_lo], dtype=np.uint32)
                     ^ _mix32(np.array([s_hi + u32(0x9E3779B9) * u32(j + 1)], dtype=np.uint32)))[0]
              for j in range(40)]

        def u01(j):
            x = _mix32(lo ^ _mix32(hi ^ sj[j]))
            return ((x >> u32(8)) + u32(1)).astype(np.float32) * np.float32(1.0 / 16777216.0)

        gauss = np.array(gauss_table(), dtype=np.float32)
        oma = np.float32(1.0 - np.float32(alpha))
        inv_oma = np.float32(np.float32(1.0) / oma)
        keys = np.empty((B, NUM_SLOTS), dtype=np.uint64)
        logit = np.full(B, np.float32(-1.2), dtype=np.float32)
        wide = num_features > (1 << 32)
        for j in range(NUM_SLOTS):
            u = u01(j)
            if j < 13:
                idv = (u * np.float32(34.62468098)).astype(np.uint32)
            else:
                cm1 = np.float32(np.power(np.float32(cards[j - 13]), oma, dtype=np.float32)
                                 - np.float32(1.0))
                x = np.exp2(inv_oma * np.log2(cm1 * u + np.float32(1.0), dtype=np.float32),
                            dtype=np.float32)
                v = x.astype(np.uint32)
                idv = np.where(v >= 1, v - u32(1), u32(0)).astype(np.uint32)
            if not wide:
                h = _mix32(idv + u32(0x9E3779B9) * u32(j + 1)).astype(np.uint64)
                key = (h * np.uint64(num_features)) >> np.uint64(32)
            else:
                key = _fmix64((np.uint64(j + 1) << np.uint64(48)) ^ idv.astype(np.uint64))
                key = key % np.uint64(num_features)
            keys[:, j] = key
            hp = _mix32(key.astype(np.uint32) ^ _mix32((key >> np.uint64(32)).astype(np.uint32)
                                                      ^ u32(0x5BD1E995)))
            logit += np.where((hp & u32(0xFF)) < 51, gauss[hp >> u32(24)], np.float32(0.0))
        p = np.float32(1.0) / (np.float32(1.0) + np.exp(-logit, dtype=np.float32))
        labels = np.where(u01(39) < p, np.float32(1.0), np.float32(-1.0)).astype(np.float32)
    return (torch.from_numpy(keys.reshape(-1).view(np.int64).copy()),
            torch.from_numpy(labels))
