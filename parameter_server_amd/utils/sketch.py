"""Bit sketches: Bitmap, BloomFilter, BlockBloomFilter.

Reference: src/util/bitmap.h (uint16-word bitmap with set/clear/test/fill/nnz),
src/util/bloom_filter.h and block_bloom_filter.h (k-probe Bloom filters over the
Sketch hash, src/util/sketch.h:20-31, probes spaced by the hash rotated right
17 bits; the block variant keeps all probes of a key inside one 64-byte bin).
The CountMin sketch used by the frequency filter lives in ops/countmin.py (host
C++ and a HIP kernel). Bulk insert/query here run in the host C++ runtime
(csrc/core/setops.cc) over whole key arrays; the bit layout is the reference's
(bit ``p`` is byte ``p/8`` bit ``p%8``), so filters built by either agree.
"""
from __future__ import annotations

import numpy as np

from ..ops.native import core


def _keys(keys) -> np.ndarray:
    if hasattr(keys, "cpu"):
        keys = keys.cpu().numpy()
    k = np.ascontiguousarray(np.asarray(keys).astype(np.uint64, copy=False))
    return k.reshape(-1)


class Bitmap:
    """Fixed-size bitmap; vectorised set / clear / test over index arrays."""

    def __init__(self, size: int = 0, value: bool = False):
        self.resize(size, value)

    def resize(self, size: int, value: bool = False) -> None:
        self._size = int(size)
        self._words = np.zeros((self._size >> 6) + 1, dtype=np.uint64)
        self.fill(value)

    def fill(self, value: bool) -> None:
        self._words[:] = np.uint64(~0 & 0xFFFFFFFFFFFFFFFF) if value else np.uint64(0)

    def clear(self, i=None) -> None:
        if i is None:
            self._words[:] = 0
            return
        i = np.asarray(i, dtype=np.uint64)
        np.bitwise_and.at(self._words, (i >> np.uint64(6)).astype(np.int64),
                          ~(np.uint64(1) << (i & np.uint64(63))))

    def set(self, i) -> None:
        i = np.asarray(i, dtype=np.uint64)
        np.bitwise_or.at(self._words, (i >> np.uint64(6)).astype(np.int64),
                         np.uint64(1) << (i & np.uint64(63)))

    def test(self, i):
        i = np.asarray(i, dtype=np.uint64)
        w = self._words[(i >> np.uint64(6)).astype(np.int64)]
        r = ((w >> (i & np.uint64(63))) & np.uint64(1)).astype(bool)
        return bool(r) if r.ndim == 0 else r

    __getitem__ = test

    def nnz(self, start: int = 0, end: int | None = None) -> int:
        end = self._size if end is None else end
        if end <= start:
            return 0
        bits = np.unpackbits(self._words.view(np.uint8), bitorder="little")
        return int(bits[start:end].sum())

    def size(self) -> int:
        return self._size

    def mem_size(self) -> int:
        return self._words.nbytes

    def to_bool(self) -> np.ndarray:
        return np.unpackbits(self._words.view(np.uint8), bitorder="little")[:self._size].astype(bool)


class BloomFilter:
    """m-bit, k-probe Bloom filter (reference bloom_filter.h)."""

    def __init__(self, m: int, k: int):
        self.resize(m, k)

    def resize(self, m: int, k: int) -> None:
        self.m = max(1, int(m))
        self.k = min(64, max(1, int(k)))
        self.bits = np.zeros(self.m // 8 + 1, dtype=np.uint8)

    def insert(self, keys) -> None:
        ks = _keys(keys)
        core().bloom_insert(self.bits.ctypes.data, self.m, self.k, ks.ctypes.data, ks.size)

    def query(self, keys):
        ks = _keys(keys)
        out = np.empty(ks.size, dtype=np.uint8)
        core().bloom_query(self.bits.ctypes.data, self.m, self.k, ks.ctypes.data, ks.size,
                           out.ctypes.data)
        return out.astype(bool)

    def __contains__(self, key) -> bool:
        return bool(self.query([key])[0])

    count = query


class BlockBloomFilter(BloomFilter):
    """Cache-blocked variant: every probe of a key hits one 64-byte bin
    (reference block_bloom_filter.h; m is rounded up to >= 1024 bits)."""

    BIN_BYTES = 64

    def resize(self, m: int, k: int) -> None:
        self.m = max(int(m), 1024)
        self.k = min(64, max(1, int(k)))
        self.nbin = self.m // 8 // self.BIN_BYTES + 1
        self.bits = np.zeros(self.nbin * self.BIN_BYTES, dtype=np.uint8)

    def reset(self) -> None:
        self.bits[:] = 0

    def insert(self, keys) -> None:
        ks = _keys(keys)
        core().block_bloom_insert(self.bits.ctypes.data, self.nbin, self.BIN_BYTES, self.k,
                                  ks.ctypes.data, ks.size)

    def query(self, keys):
        ks = _keys(keys)
        out = np.empty(ks.size, dtype=np.uint8)
        core().block_bloom_query(self.bits.ctypes.data, self.nbin, self.BIN_BYTES, self.k,
                                 ks.ctypes.data, ks.size, out.ctypes.data)
        return out.astype(bool)

    count = query
