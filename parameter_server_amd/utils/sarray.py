"""Sorted-key array algebra (reference SArray + parallel_ordered_match.h).

The reference's ``SArray<K>`` carries ``setUnion`` / ``setIntersection`` /
``findRange`` / ``segment`` (src/util/shared_array_inl.h:133-176), and
``parallelOrderedMatch`` / ``parallelUnion`` (src/util/parallel_ordered_match.h)
merge-join sorted key lists with an operator on the matching values; the KV
vectors and Darlin's key exchange sit on these. A framework "SArray" is a
torch tensor / numpy array (zero-copy views already cover ``segment``); this
module supplies the algebra:

* CPU numpy/torch arrays with uint64 keys -> the threaded C++ merge join in
  ``csrc/core/setops.cc`` (``_pscore``), one dst piece per thread;
* GPU tensors -> ``torch.searchsorted`` (a device kernel) + an indexed op, no
  host round trip;
* anything else -> a numpy searchsorted fallback with identical semantics.

Values are ``k`` per key (flat ``[n*k]`` or ``[n, k]``); ops: ASSIGN, PLUS,
MINUS, OR.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..ops.native import core, is_gpu

_OPS = {"ASSIGN": 0, "PLUS": 1, "OR": 2, "MINUS": 3}
_VT = {np.dtype(np.float32): 0, np.dtype(np.float64): 1, np.dtype(np.int32): 2,
       np.dtype(np.int64): 3, np.dtype(np.uint8): 4}


def _threads() -> int:
    return int(os.environ.get("PSAMD_NUM_THREADS", min(8, os.cpu_count() or 1)))


def find_range(keys, lo, hi) -> tuple[int, int]:
    """Positions [a, b) of the sorted ``keys`` inside the key range [lo, hi)
    (reference SArray::findRange, shared_array_inl.h:169)."""
    if is_gpu(keys):
        b = torch.tensor([lo, hi], dtype=keys.dtype, device=keys.device)
        r = torch.searchsorted(keys, b).tolist()
        return r[0], r[1]
    k = np.asarray(keys)
    return (int(np.searchsorted(k, k.dtype.type(lo))),
            int(np.searchsorted(k, k.dtype.type(hi))) if hi is not None else k.size)


def _np_u64(a):
    a = np.asarray(a)
    return a if a.dtype == np.uint64 and a.flags.c_contiguous else None


def set_union(a, b):
    """Sorted union of two sorted, duplicate-free key arrays."""
    if is_gpu(a) or is_gpu(b):
        return torch.unique(torch.cat([a, b]))
    ua, ub = _np_u64(a), _np_u64(b)
    if ua is None or ub is None:
        return np.union1d(a, b)
    out = np.empty(ua.size + ub.size, dtype=np.uint64)
    n = core().set_union(ua.ctypes.data, ua.size, ub.ctypes.data, ub.size, out.ctypes.data)
    return out[:n]


def set_intersection(a, b):
    if is_gpu(a) or is_gpu(b):
        pos = torch.searchsorted(b, a).clamp_max(max(b.numel() - 1, 0))
        return a[b[pos] == a] if b.numel() else a[:0]
    ua, ub = _np_u64(a), _np_u64(b)
    if ua is None or ub is None:
        return np.intersect1d(a, b, assume_unique=True)
    out = np.empty(min(ua.size, ub.size), dtype=np.uint64)
    n = core().set_intersection(ua.ctypes.data, ua.size, ub.ctypes.data, ub.size, out.ctypes.data)
    return out[:n]


def _apply_torch(dv, idx, sv, op):
    if op == "ASSIGN":
        dv[idx] = sv
    elif op == "PLUS":
        dv.index_add_(0, idx, sv)
    elif op == "MINUS":
        dv.index_add_(0, idx, -sv)
    elif op == "OR":
        dv[idx] |= sv
    else:
        raise ValueError(op)


def ordered_match(src_key, src_val, dst_key, k: int = 1, op: str = "ASSIGN", dst_val=None):
    """For keys present in both sorted arrays apply ``dst_val[j] (op)= src_val[i]``
    (reference parallelOrderedMatch). Returns ``(dst_val, n_matched)``; a missing
    ``dst_val`` is created zero-filled like the reference does."""
    if op not in _OPS:
        raise ValueError(op)
    if is_gpu(dst_key):
        n = dst_key.numel()
        sv = torch.as_tensor(src_val, device=dst_key.device).reshape(-1, k)
        if dst_val is None:
            dst_val = torch.zeros(n * k, dtype=sv.dtype, device=dst_key.device)
        if src_key.numel() == 0 or n == 0:
            return dst_val, 0
        pos = torch.searchsorted(dst_key, src_key).clamp_max(n - 1)
        hit = dst_key[pos] == src_key
        _apply_torch(dst_val.view(-1, k), pos[hit], sv[hit], op)
        return dst_val, int(hit.sum())
    src_key = np.asarray(src_key)
    dst_key = np.asarray(dst_key)
    sv = np.ascontiguousarray(src_val)
    n = dst_key.size
    if dst_val is None:
        dst_val = np.zeros(n * k, dtype=sv.dtype)
    if src_key.size == 0 or n == 0:
        return dst_val, 0
    if sv.size != src_key.size * k or np.asarray(dst_val).size != n * k:
        raise ValueError("ordered_match: value arrays must hold k values per key")
    sk, dk = _np_u64(src_key), _np_u64(dst_key)
    dv = dst_val
    vt = _VT.get(sv.dtype)
    if (sk is not None and dk is not None and vt is not None and isinstance(dv, np.ndarray)
            and dv.dtype == sv.dtype and dv.flags.c_contiguous):
        m = core().ordered_match(sk.ctypes.data, sk.size, sv.ctypes.data, dk.ctypes.data, dk.size,
                                 dv.ctypes.data, k, vt, _OPS[op], _threads())
        return dst_val, int(m)
    # generic fallback (other key / value dtypes)
    pos = np.minimum(np.searchsorted(dst_key, src_key), n - 1)
    hit = dst_key[pos] == src_key
    s = sv.reshape(-1, k)[hit]
    d = np.asarray(dst_val).reshape(-1, k)
    idx = pos[hit]
    if op == "ASSIGN":
        d[idx] = s
    elif op == "PLUS":
        np.add.at(d, idx, s)
    elif op == "MINUS":
        np.subtract.at(d, idx, s)
    else:
        d[idx] |= s
    return dst_val, int(hit.sum())


def parallel_union(k1, v1, k2, v2, k: int = 1, op: str = "PLUS"):
    """Sorted key union with values combined by ``op`` (reference parallelUnion,
    parallel_ordered_match.h:88-112)."""
    keys = set_union(k1, k2)
    dt = (v1 if v1 is not None and len(v1) else v2).dtype
    if is_gpu(keys):
        vals = torch.zeros(keys.numel() * k, dtype=dt, device=keys.device)
    else:
        vals = np.zeros(len(keys) * k, dtype=dt)
    if len(k1):
        vals, n1 = ordered_match(k1, v1, keys, k, op, vals)
        assert n1 == len(k1)
    if len(k2):
        vals, n2 = ordered_match(k2, v2, keys, k, op, vals)
        assert n2 == len(k2)
    return keys, vals
