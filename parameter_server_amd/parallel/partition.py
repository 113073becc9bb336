"""Key-range partitioning of the (mixed) key space over server shards.

Reference: ``Postmaster::partitionServerKeyRange`` gives server s the range
``Range::all().evenDivide(num_servers, s)`` over raw uint64 keys
(src/system/postmaster.cc:17-31, src/util/range.h:89-107). Here the same even
split is applied to the *mixed* key space [0, 2^bits) (a bijection of the raw
space), which keeps shards balanced for any key distribution.
"""
from __future__ import annotations

import torch


def even_divide(begin: int, end: int, n: int, i: int) -> tuple[int, int]:
    """[begin,end) split into n nearly equal parts; part i (reference Range::evenDivide)."""
    size = end - begin
    return begin + size * i // n, begin + size * (i + 1) // n


def to_i64(u: int) -> int:
    u &= (1 << 64) - 1
    return u - (1 << 64) if u >= (1 << 63) else u


class KeyPartition:
    """G contiguous ranges of [0, 2^bits); shard s owns [bounds[s], bounds[s+1])."""

    def __init__(self, bits: int, num_shards: int):
        self.bits = bits
        self.G = int(num_shards)
        total = 1 << bits
        self.bounds_u = [even_divide(0, total, self.G, s)[0] for s in range(self.G)] + [total]
        # int64 view for device kernels; the last bound (2^bits) is never compared
        self.bounds = torch.tensor([to_i64(min(b, (1 << 64) - 1)) for b in self.bounds_u],
                                   dtype=torch.int64)
        self._dev = {}

    def range_of(self, shard: int) -> tuple[int, int]:
        return self.bounds_u[shard], self.bounds_u[shard + 1]

    def bounds_on(self, device) -> torch.Tensor:
        key = str(device)
        if key not in self._dev:
            self._dev[key] = self.bounds.to(device)
        return self._dev[key]

    def owner_of(self, h: torch.Tensor) -> torch.Tensor:
        """Owner shard of each mixed key (unsorted input)."""
        if self.G == 1:
            return torch.zeros(h.numel(), dtype=torch.int32, device=h.device)
        if h.is_cuda:
            from ..ops.native import hipops

            out = torch.empty(h.numel(), dtype=torch.int32, device=h.device)
            hipops().owner_of(h.contiguous(), self.bounds_on(h.device), out)
            return out
        hb = h ^ torch.tensor(-(1 << 63), dtype=torch.int64) if self.bits == 64 else h
        bb = self.bounds[:-1]
        if self.bits == 64:
            bb = bb ^ torch.tensor(-(1 << 63), dtype=torch.int64)
        return (torch.searchsorted(bb, hb, right=True) - 1).to(torch.int32)

    def split_sorted(self, uniq: torch.Tensor, n_uniq: torch.Tensor | None = None) -> torch.Tensor:
        """Offsets [G+1] of each owner's run in a sorted unique key array (K14)."""
        dev = uniq.device
        if self.G == 1:
            n = int(n_uniq.item()) if n_uniq is not None else uniq.numel()
            return torch.tensor([0, n], dtype=torch.int64)
        if uniq.is_cuda:
            from ..ops.native import hipops

            off = torch.empty(self.G + 1, dtype=torch.int64, device=dev)
            hipops().owner_split(uniq, n_uniq, self.bounds_on(dev), off)
            return off
        n = int(n_uniq.item()) if n_uniq is not None else uniq.numel()
        u = uniq[:n]
        bb = self.bounds[1:-1]
        if self.bits == 64:
            u = u ^ torch.tensor(-(1 << 63), dtype=torch.int64)
            bb = bb ^ torch.tensor(-(1 << 63), dtype=torch.int64)
        mid = torch.searchsorted(u, bb, right=False)
        return torch.cat([torch.zeros(1, dtype=torch.int64), mid, torch.tensor([n])])
