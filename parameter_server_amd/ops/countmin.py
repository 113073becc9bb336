"""CountMin sketch with saturating uint8 cells (tail-feature filter, K6).

Reference: ``CountMin<K, uint8>`` (src/util/countmin.h:8-48) wrapped by
``FreqencyFilter`` (src/parameter/frequency_filter.h:9-45): insert per-key counts,
keep keys whose estimated count > freq. Cells saturate at v_max = 254.

``key_bits`` set (the GPU trainers): the sketch is partitioned into 2^lgR regions of
``rsize`` cells and a key's k cells lie in region ``key >> (key_bits - lgR)``
(csrc/hip/countmin.cuh), inside one 64-cell block of it (blocked CountMin: a key's cells
share one cache line). The flat localiser's bucket workgroups own whole key ranges and so
whole regions: each inserts its keys and queries them behind a workgroup barrier, in the
same launch. The cells per key are the reference's k; the collision rate is that of a
blocked sketch of the same size (slightly above the global layout's for the same n);
``key_bits=None`` keeps the reference's global layout (the CPU runtime apps on raw keys).
"""
from __future__ import annotations

import torch

from .native import core, hipops, is_gpu, ptr

VMAX = 254
LG_REGIONS = 11  # >= log2 of the flat localiser's largest fine-bucket count (2048)

_M32 = 0xFFFFFFFF


def sketch_hash_torch(keys: torch.Tensor) -> torch.Tensor:
    """The 64->32 sketch hash (countmin.cuh sketch_hash) on an int64 tensor -> int64 in
    [0, 2^32)."""
    m = 0xC6A4A793
    h = (0xBC9F1D34 ^ ((8 * m) & _M32)) & _M32
    lo = keys & _M32
    hi = (keys >> 32) & _M32
    h = torch.full_like(keys, h)
    for part in (lo, hi):
        h = (h + part) & _M32
        h = (h * m) & _M32
        h = h ^ (h >> 16)
    return h


class CountMinSketch:
    def __init__(self, n: int, k: int = 2, device="cpu", vmax: int = VMAX,
                 key_bits: int | None = None, lg_regions: int = LG_REGIONS):
        n = max(64, int(n))
        self.k = min(30, max(1, int(k)))
        self.vmax = int(vmax)
        self.device = torch.device(device)
        self.key_bits = key_bits
        if key_bits is None:
            n = (n + 3) // 4 * 4  # whole 32-bit words on the device
            self.lgR, self.rshift, self.rsize = 0, 64, n
        else:
            self.lgR = min(int(lg_regions), int(key_bits))
            self.rshift = int(key_bits) - self.lgR
            r = 1 << self.lgR
            # whole 64-cell blocks: regions never share a cache line
            self.rsize = max(64, ((n + r - 1) // r + 63) // 64 * 64)
            n = self.rsize << self.lgR
        self.n = n
        self.cells = torch.zeros(n, dtype=torch.uint8, device=self.device)

    @property
    def partitioned(self) -> bool:
        return self.rshift < 64

    def args(self, freq: int = 0) -> tuple:
        """(cells as int32 words, rsize, rshift, k, vmax, freq): what the fused localiser
        filter takes."""
        return (self.cells.view(torch.int32), self.rsize, self.rshift, self.k, self.vmax, int(freq))

    def clear(self):
        self.cells.zero_()

    def _kw(self) -> dict:
        return dict(rsize=self.rsize, rshift=self.rshift,
                    key_bits=self.key_bits if self.key_bits is not None else 64)

    def _cells_of(self, keys: torch.Tensor) -> torch.Tensor:
        """[n, k] cell indices of keys (CPU reference of countmin.cuh)."""
        keys = keys.to(torch.int64)
        h = sketch_hash_torch(keys)
        delta = ((h >> 17) | (h << 15)) & _M32
        cols = []
        if not self.partitioned:
            for _ in range(self.k):
                cols.append(h % self.rsize)
                h = (h + delta) & _M32
            return torch.stack(cols, 1)
        # blocked: the key's block of its region, offsets o_j = (h2 + j * d2) mod 64
        base = (keys >> self.rshift) * self.rsize + (h % (self.rsize // 64)) * 64
        o = delta & 63
        d2 = ((delta >> 6) & 63) | 1
        for _ in range(self.k):
            cols.append(base + o)
            o = (o + d2) & 63
        return torch.stack(cols, 1)

    def insert(self, keys: torch.Tensor, counts: torch.Tensor | None = None, n_dev=None):
        keys = keys.contiguous()
        if counts is not None:
            counts = counts.contiguous()
        if is_gpu(keys):
            hipops().cm_insert(self.cells.view(torch.int32), self.k, self.vmax, keys, counts, n_dev,
                               **self._kw())
        elif self.partitioned:
            if n_dev is not None:
                n = int(n_dev.reshape(-1)[0])
                keys = keys[:n]
                counts = None if counts is None else counts[:n]
            c = (torch.ones(keys.numel(), dtype=torch.int64) if counts is None
                 else counts.to(torch.int64))
            # a chain of saturating adds of non-negative counts = the clamped sum
            cells = self._cells_of(keys)
            acc = self.cells.to(torch.int64)
            for j in range(self.k):
                acc.index_add_(0, cells[:, j], c)
            self.cells.copy_(acc.clamp(max=self.vmax).to(torch.uint8))
        else:
            core().cm_insert(ptr(self.cells), self.n, self.k, self.vmax, ptr(keys), ptr(counts),
                             keys.numel())

    def insert_segments(self, keys: torch.Tensor, seg_start: torch.Tensor, n_dev=None):
        """Insert unique keys with counts = their occurrence run lengths
        ``seg_start[i+1] - seg_start[i]`` (saturated to a byte); ``n_dev``: device count
        (no host sync: graph-capturable)."""
        if is_gpu(keys):
            hipops().cm_insert_seg(self.cells.view(torch.int32), self.k, self.vmax,
                                   keys.contiguous(), seg_start.contiguous(), n_dev, **self._kw())
            return
        n = keys.numel() if n_dev is None else int(n_dev.reshape(-1)[0])
        cnt = (seg_start[1:n + 1] - seg_start[:n]).clamp(max=255).to(torch.uint8)
        self.insert(keys[:n], cnt)

    def query(self, keys: torch.Tensor, freq: int = 0, n_dev=None):
        """(keep int32 [n] = count > freq, count uint8 [n])."""
        keys = keys.contiguous()
        keep = torch.empty(keys.numel(), dtype=torch.int32, device=keys.device)
        cnt = torch.empty(keys.numel(), dtype=torch.uint8, device=keys.device)
        if is_gpu(keys):
            hipops().cm_query(self.cells.view(torch.int32), self.k, self.vmax, keys, n_dev, freq,
                              keep, cnt, **self._kw())
        elif self.partitioned:
            v = self.cells[self._cells_of(keys)].to(torch.int32).min(1).values
            v = v.clamp(max=self.vmax)
            cnt.copy_(v.to(torch.uint8))
            keep.copy_((v > freq).to(torch.int32))
        else:
            core().cm_query(ptr(self.cells), self.n, self.k, self.vmax, ptr(keys), keys.numel(),
                            freq, ptr(keep), ptr(cnt))
        return keep, cnt
