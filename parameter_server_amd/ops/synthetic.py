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


def _set_cards(device, cards):
    key = (str(device), tuple(cards))
    if _cards_set.get(str(device)) != key:
        hipops().criteo_set_cards([int(c) for c in cards])
        _cards_set[str(device)] = key


def criteo_batch(B: int, *, seed: int, row0: int, num_features: int, alpha: float = 1.1,
                 cards=CRITEO_1TB_CARDS, device="cpu", keys=None, labels=None, row0_dev=None,
                 row_scale: int = 1):
    """Returns (keys int64 [B*39] row-major, labels float32 [B] in {-1,+1}).
    GPU only: ``row0_dev`` (int64[1] device) adds ``row0_dev * row_scale`` to ``row0``
    at kernel time, so a captured graph generates fresh rows on every replay."""
    device = torch.device(device)
    keys = torch.empty(B * NUM_SLOTS, dtype=torch.int64, device=device) if keys is None else keys
    labels = torch.empty(B, dtype=torch.float32, device=device) if labels is None else labels
    if device.type == "cuda":
        _set_cards(device, cards)
        hipops().criteo_gen(seed & ((1 << 64) - 1), row0, B, num_features, alpha, keys, labels,
                            row0_dev, row_scale)
        return keys, labels
    k, l = _criteo_cpu(B, seed, row0, num_features, alpha, cards)
    keys.copy_(k)
    labels.copy_(l)
    return keys, labels


# ----------------------------------------------------------------------------- CPU path
M64 = (1 << 64) - 1


def _rng64(seed, idx):
    z = (seed + 0x9E3779B97F4A7C15 * (idx + 1)) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def _u01(r):
    return ((r >> 40) + 1.0) * (1.0 / 16777216.0)


def _fmix64(k):
    k ^= k >> 33
    k = (k * 0xFF51AFD7ED558CCD) & M64
    k ^= k >> 33
    k = (k * 0xC4CEB9FE1A85EC53) & M64
    k ^= k >> 33
    return k


def _planted_w(key, seed):
    r = _rng64(seed ^ 0x5BD1E995, key)
    if (r & 0xFF) >= 51:
        return 0.0
    u1 = _u01(_rng64(seed, key * 2 + 7))
    u2 = _u01(r)
    return 0.6 * math.sqrt(-2 * math.log(u1)) * math.cos(6.283185307 * u2)


def _criteo_cpu(B, seed, row0, num_features, alpha, cards):
    """Scalar reference generator (small B only: tests). float32 rounding of the
    power-law inverse CDF can differ from the GPU in the last ulp for a few rows."""
    import numpy as np

    keys = np.empty(B * NUM_SLOTS, dtype=np.uint64)
    labels = np.empty(B, dtype=np.float32)
    f32 = np.float32
    for r in range(B):
        gr = row0 + r
        logit = -1.2
        for j in range(NUM_SLOTS):
            u = f32(_u01(_rng64((seed + j * 0x632BE59BD9B4E019) & M64, gr)))
            if j < 13:
                # floor(2 log2(1 + (e^(12u) - 1))) = floor(u * 24 log2 e), in f32 as the kernel
                idv = int(f32(u) * f32(34.62468098))
            else:
                C = f32(cards[j - 13])
                oma = f32(1.0 - alpha)
                x = np.power(f32((np.power(C, oma, dtype=f32) - f32(1.0)) * u + f32(1.0)),
                             f32(1.0) / oma, dtype=f32)
                v = int(x)
                idv = v - 1 if v >= 1 else 0
            key = _fmix64(((j + 1) << 48) ^ idv) % num_features
            keys[r * NUM_SLOTS + j] = key
            logit += _planted_w(key, seed & M64)
        p = 1.0 / (1.0 + math.exp(-logit))
        u = _u01(_rng64((seed ^ 0xABCDEF) & M64, gr))
        labels[r] = 1.0 if u < p else -1.0
    return torch.from_numpy(keys.view(np.int64).copy()), torch.from_numpy(labels)
