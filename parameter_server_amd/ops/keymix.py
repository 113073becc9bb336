"""Bijective key mixing on [0, 2^bits) (device: ``mix_keys`` kernel; host: C++).

Deduplicating, sorting and range-partitioning *mixed* keys is equivalent to doing
so on raw keys (the map is a bijection), but shards stay balanced even for
small consecutive integer ids (LIBSVM / rcv1), which the reference's raw-key
range partition (src/system/postmaster.cc:17-31) sends entirely to server 0.
"""
from __future__ import annotations

import torch

from .native import core, hipops, is_gpu, ptr


def key_bits_for(num_features: int | None) -> int:
    """Bits needed for keys in [0, num_features); 64 for unbounded uint64 keys."""
    if not num_features or num_features <= 0 or num_features > (1 << 63):
        return 64
    return max(2, int(num_features - 1).bit_length())


def mix(keys: torch.Tensor, bits: int, inverse: bool = False) -> torch.Tensor:
    keys = keys.contiguous()
    assert keys.dtype == torch.int64
    out = torch.empty_like(keys)
    if keys.numel() == 0:
        return out
    if is_gpu(keys):
        hipops().mix_keys(keys, bits, out, inverse)
    else:
        core().mix_keys(ptr(keys), ptr(out), keys.numel(), bits, inverse)
    return out


def unmix(h: torch.Tensor, bits: int) -> torch.Tensor:
    return mix(h, bits, inverse=True)


def to_unsigned_order(x: torch.Tensor) -> torch.Tensor:
    """Map uint64-in-int64 to int64 whose signed order equals the unsigned order."""
    return x ^ torch.tensor(-(1 << 63), dtype=torch.int64, device=x.device)


def random_keys_in_range(lo: int, hi: int, n: int, generator=None, device="cpu") -> torch.Tensor:
    """``n`` uniform random (mixed) keys of the unsigned range [lo, hi) as int64 bit
    patterns (the table's key format). Ranges past 2^63 (64-bit key spaces, e.g. the
    upper shards of raw-u64 keys) are drawn as high and low 32-bit halves with
    wrap-around int64 arithmetic instead of ``torch.randint``, which stops at 2^63."""
    lo, hi = int(lo), int(hi)
    span = hi - lo
    if span <= 0:
        raise ValueError(f"empty key range [{lo}, {hi})")
    if hi <= (1 << 63):
        return torch.randint(lo, hi, (n,), generator=generator, device=device, dtype=torch.int64)
    # span > 2^32 here: offset = (h << 32) + l with h < span >> 32, l < 2^32 -> offset < span
    h = torch.randint(0, span >> 32, (n,), generator=generator, device=device, dtype=torch.int64)
    low = torch.randint(0, 1 << 32, (n,), generator=generator, device=device, dtype=torch.int64)
    base = lo - (1 << 64) if lo >= (1 << 63) else lo
    return (h << 32) + low + base
