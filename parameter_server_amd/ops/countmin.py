"""CountMin sketch with saturating uint8 cells (tail-feature filter, K6).

Reference: ``CountMin<K, uint8>`` (src/util/countmin.h:8-48) wrapped by
``FreqencyFilter`` (src/parameter/frequency_filter.h:9-45): insert per-key counts,
keep keys whose estimated count > freq. Cells saturate at v_max = 254.
"""
from __future__ import annotations

import torch

from .native import core, hipops, is_gpu, ptr

VMAX = 254


class CountMinSketch:
    def __init__(self, n: int, k: int = 2, device="cpu", vmax: int = VMAX):
        n = max(64, int(n))
        n = (n + 3) // 4 * 4  # whole 32-bit words on the device
        self.n = n
        self.k = min(30, max(1, int(k)))
        self.vmax = int(vmax)
        self.device = torch.device(device)
        self.cells = torch.zeros(n, dtype=torch.uint8, device=self.device)

    def clear(self):
        self.cells.zero_()

    def insert(self, keys: torch.Tensor, counts: torch.Tensor | None = None, n_dev=None):
        keys = keys.contiguous()
        if counts is not None:
            counts = counts.contiguous()
        if is_gpu(keys):
            hipops().cm_insert(self.cells.view(torch.int32), self.k, self.vmax, keys, counts, n_dev)
        else:
            core().cm_insert(ptr(self.cells), self.n, self.k, self.vmax, ptr(keys), ptr(counts),
                             keys.numel())

    def insert_segments(self, keys: torch.Tensor, seg_start: torch.Tensor, n_dev=None):
        """Insert unique keys with counts = their occurrence run lengths
        ``seg_start[i+1] - seg_start[i]`` (saturated to a byte); ``n_dev``: device count
        (no host sync: graph-capturable)."""
        if is_gpu(keys):
            hipops().cm_insert_seg(self.cells.view(torch.int32), self.k, self.vmax,
                                   keys.contiguous(), seg_start.contiguous(), n_dev)
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
                              keep, cnt)
        else:
            core().cm_query(ptr(self.cells), self.n, self.k, self.vmax, ptr(keys), keys.numel(),
                            freq, ptr(keep), ptr(cnt))
        return keep, cnt
