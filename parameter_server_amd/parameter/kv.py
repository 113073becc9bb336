"""Concrete shared parameters: KVVector, KVBufferedVector, KVStore, KVMap.

Reference semantics:
* ``KVVector<K,V>`` (src/parameter/kv_vector.h:13-100): per ``key_channel`` a
  sorted key array + value array (k values per key). ``set_value``: union-merge
  for ``gather`` / tail-filter messages, else ordered-match ADD into existing
  values; ``get_value``: ordered-match gather.
* ``KVBufferedVector`` (kv_buffered_vector.h): pushes at time t are summed across
  senders into a buffer read once with ``received(t)``.
* ``KVStore<K,V,E,S>`` (kv_store.h:28-80): hash-map store whose entries apply the
  optimizer on push and return the weight on pull; ``write_to_file`` writes
  ``key\\tw`` for non-zero weights. Backed here by the same 32-byte-slot table the
  GPU uses (``ops.KVTable``), with the C++ host kernels.
* ``KVMap`` (kv_map.h): unordered map with an element-wise operator on push.
"""
from __future__ import annotations

import threading

import numpy as np
import torch

from ..ops.kv_table import KVTable, UpdateRule
from ..system.message import KEY_MAX
from ..utils import sarray
from .shared_parameter import SharedParameter, comp_ass_op


def ordered_match(src_key, src_val, dst_key, k: int = 1, op: str = "ASSIGN", dst_val=None):
    """Merge-join of sorted key arrays (reference parallelOrderedMatch,
    src/util/parallel_ordered_match.h:5-86); native threaded join on CPU
    (utils/sarray.py -> csrc/core/setops.cc). Returns (dst_val, number matched)."""
    return sarray.ordered_match(src_key, src_val, dst_key, k, op, dst_val)


def ordered_union(k1, v1, k2, v2, k: int = 1):
    """Sorted union with values summed on common keys (parallelUnion)."""
    return sarray.parallel_union(np.asarray(k1), np.asarray(v1), np.asarray(k2), np.asarray(v2), k)


class KVVector(SharedParameter):
    def __init__(self, name: str, k: int = 1, dtype=np.float32, key_dtype=np.uint64, parent=None,
                 po=None):
        super().__init__(name, parent, po)
        self.k = k
        self.dtype = np.dtype(dtype)
        self.key_dtype = np.dtype(key_dtype)
        self.keys: dict[int, np.ndarray] = {}
        self.vals: dict[int, np.ndarray] = {}
        self.mu = threading.RLock()

    def key(self, chl: int = 0) -> np.ndarray:
        with self.mu:
            return self.keys.setdefault(chl, np.zeros(0, self.key_dtype))

    def value(self, chl: int = 0) -> np.ndarray:
        with self.mu:
            return self.vals.setdefault(chl, np.zeros(0, self.dtype))

    def set_key(self, chl: int, key):
        with self.mu:
            self.keys[chl] = np.asarray(key, dtype=self.key_dtype)

    def set_val(self, chl: int, val):
        with self.mu:
            self.vals[chl] = np.asarray(val, dtype=self.dtype)

    def clear(self, chl: int = 0):
        with self.mu:
            self.keys.pop(chl, None)
            self.vals.pop(chl, None)

    def set_value(self, msg):
        rk = msg.key
        if rk is None or rk.size == 0:
            return
        chl = msg.task.get("key_channel", 0)
        call = msg.task.get("shared_para", {})
        with self.mu:
            mk, mv = self.key(chl), self.value(chl)
            if "tail_filter" in call or call.get("gather"):
                if not msg.value:
                    self.keys[chl] = np.union1d(mk, rk.astype(self.key_dtype))
                else:
                    nk, nv = ordered_union(mk, mv, rk.astype(self.key_dtype),
                                           msg.value[0].astype(self.dtype), self.k)
                    self.keys[chl], self.vals[chl] = nk, nv
                return
            if mv.size != mk.size * self.k:
                mv = np.zeros(mk.size * self.k, self.dtype)
            mv, n = ordered_match(rk, msg.value[0].astype(self.dtype), mk, self.k, "PLUS", mv)
            self.vals[chl] = mv
            if n != rk.size:
                raise RuntimeError(f"{self.name}: {rk.size - n} pushed keys are unknown")

    def get_value(self, msg):
        rk = msg.key
        if rk is None or rk.size == 0:
            return
        chl = msg.task.get("key_channel", 0)
        with self.mu:
            val, _ = ordered_match(self.key(chl), self.value(chl), rk.astype(self.key_dtype), self.k)
        msg.clear_value()
        msg.add_value(val)


class KVBufferedVector(KVVector):
    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.recved: dict[int, tuple] = {}

    def received(self, t: int):
        """(index range into key(chl), [summed value arrays]) pushed at time t."""
        with self.mu:
            if t not in self.recved:
                raise KeyError(f"{self.my_node_id()} hasn't received data at time {t}")
            return self.recved.pop(t)

    def set_value(self, msg):
        rk = msg.key
        if rk is None or rk.size == 0:
            return
        chl = msg.task.get("key_channel", 0)
        with self.mu:
            mk = self.key(chl)
            if not msg.value:
                self.keys[chl] = np.union1d(mk, rk.astype(self.key_dtype))
                self.vals[chl] = np.zeros(0, self.dtype)
                return
            t = msg.task["time"]
            lo, hi = msg.task.get("key_range", [0, KEY_MAX])
            ukey = mk.astype(np.uint64)
            a = int(np.searchsorted(ukey, np.uint64(lo)))
            b = int(np.searchsorted(ukey, np.uint64(hi))) if hi < KEY_MAX else ukey.size
            seg = mk[a:b]
            rng, bufs = self.recved.setdefault(t, ((a, b), []))
            for i, v in enumerate(msg.value):
                v = v.astype(self.dtype)
                kk = v.size // rk.size
                if i >= len(bufs):
                    bufs.append(np.zeros(seg.size * kk, self.dtype))
                _, n = ordered_match(rk, v, seg, kk, "PLUS", bufs[i])
                if n != rk.size:
                    raise RuntimeError("pushed keys not in the key set")


class KVStore(SharedParameter):
    """Server-side optimizer store (one table per node, C++ host kernels)."""

    def __init__(self, name: str, rule: UpdateRule, capacity: int = 1 << 20, parent=None, po=None,
                 reporter=None):
        super().__init__(name, parent, po)
        self.rule = rule
        self.table = KVTable(capacity, "cpu")
        self.mu = threading.Lock()
        self.stats = torch.zeros(3, dtype=torch.float64)
        self.nnz = 0
        self.reporter = reporter

    def _keys(self, key: np.ndarray) -> torch.Tensor:
        return torch.from_numpy(key.astype(np.uint64, copy=False).view(np.int64).copy())

    def get_value(self, msg):
        with self.mu:
            _, w = self.table.resolve(self._keys(msg.key), insert=True)
        msg.clear_value()
        msg.add_value(w.numpy())

    def set_value(self, msg):
        if msg.key is None or msg.key.size == 0:
            return
        g = torch.from_numpy(msg.value[0].astype(np.float32, copy=False).copy())
        with self.mu:
            slot, _ = self.table.resolve(self._keys(msg.key), insert=True, with_w=False)
            self.stats.zero_()
            self.table.update(slot, g, self.rule, self.stats)
            self.nnz += int(self.stats[0])
            if self.reporter:
                self.reporter(self.nnz, float(self.stats[1]), float(self.stats[2]))

    def write_to_file(self, path: str):
        from ..utils.checkpoint import write_text_model

        k, w, _, _ = self.table.occupied()
        return write_text_model(path, k, w)


class KVMap(SharedParameter):
    def __init__(self, name: str, op: str = "PLUS", parent=None, po=None):
        super().__init__(name, parent, po)
        self.data: dict[int, float] = {}
        self.op = op

    def get_value(self, msg):
        msg.clear_value()
        msg.add_value(np.array([self.data.get(int(k), 0.0) for k in msg.key], dtype=np.float32))

    def set_value(self, msg):
        op = msg.task.get("shared_para", {}).get("op", self.op)
        for k, v in zip(msg.key.tolist(), msg.value[0].tolist()):
            cur = np.array([self.data.get(k, 0.0)], dtype=np.float64)
            comp_ass_op(op, cur, np.array([v], dtype=np.float64))
            self.data[k] = float(cur[0])
