"""Fixed-point gradient compression (FixingFloat filter, K16).

Reference: src/filter/fixing_float.h:44-95 — per value array, [min, max] (derived
when unset, max + 1e-6), map to ``nbytes`` fixed point over 2^(8n)-2 levels with a
random rounding bit. Here rounding up happens with probability equal to the
fractional part (unbiased stochastic rounding), counter-based RNG per element.
"""
from __future__ import annotations

import torch

from .native import hipops, is_gpu


def minmax(x: torch.Tensor) -> torch.Tensor:
    mm = torch.empty(2, dtype=torch.float32, device=x.device)
    if is_gpu(x):
        hipops().ff_minmax(x.contiguous(), mm)
    else:
        finite = x[~torch.isnan(x)]
        lo = float(finite.min()) if finite.numel() else 0.0
        hi = float(finite.max()) if finite.numel() else 0.0
        mm[0] = lo
        mm[1] = hi + 1e-6
    return mm


def encode(x: torch.Tensor, nbytes: int, mm: torch.Tensor | None = None, seed: int = 0):
    """Returns (code uint8 [n*nbytes], mm float32[2])."""
    assert 1 <= nbytes <= 7
    x = x.contiguous().float()
    mm = minmax(x) if mm is None else mm.to(x.device).float()
    out = torch.empty(x.numel() * nbytes, dtype=torch.uint8, device=x.device)
    if is_gpu(x):
        hipops().ff_encode(x, mm, nbytes, seed & ((1 << 64) - 1), out)
        return out, mm
    lo, hi = float(mm[0]), float(mm[1])
    ratio = float((1 << (8 * nbytes)) - 2)
    v = x.double().clamp(lo, hi)
    t = (v - lo) / (hi - lo) * ratio
    g = torch.Generator().manual_seed(seed)
    u = torch.rand(t.shape, generator=g, dtype=torch.float64)
    r = (torch.floor(t) + ((t - torch.floor(t)) > u).double()).long()
    for j in range(nbytes):
        out[j::nbytes] = ((r >> (8 * j)) & 0xFF).to(torch.uint8)
    return out, mm


def decode(code: torch.Tensor, nbytes: int, mm: torch.Tensor, n: int | None = None):
    n = code.numel() // nbytes if n is None else n
    out = torch.empty(n, dtype=torch.float32, device=code.device)
    if is_gpu(code):
        hipops().ff_decode(code.contiguous(), mm.to(code.device).float(), nbytes, out)
        return out
    lo, hi = float(mm[0]), float(mm[1])
    ratio = float((1 << (8 * nbytes)) - 2)
    r = torch.zeros(n, dtype=torch.int64)
    c = code.long()
    for j in range(nbytes):
        r |= c[j::nbytes] << (8 * j)
    out.copy_((r.double() / ratio * (hi - lo) + lo).float())
    return out


def key_signature(keys: torch.Tensor) -> int:
    """Position-dependent 64-bit signature of a key array (device-side, K15)."""
    if is_gpu(keys):
        sig = torch.zeros(1, dtype=torch.int64, device=keys.device)
        hipops().key_signature(keys.contiguous(), sig)
        return int(sig.item()) & ((1 << 64) - 1)
    from .native import core

    acc = 0
    M = (1 << 64) - 1
    f = core().fmix64
    for i, k in enumerate(keys.tolist()):
        acc = (acc + f((k & M) ^ f((i + 0x9E3779B97F4A7C15) & M))) & M
    return acc
