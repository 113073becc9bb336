"""Message filters applied on every send / receive (src/filter/).

The sender encodes in configuration order just before queueing; the receiver
decodes in reverse order (reference RNode::encodeFilter / decodeFilter,
src/system/remote_node.cc:177-191). Filter runtime state travels inside the
task's filter entries. One filter instance per (peer, type).

On the GPU data plane the same ideas are realised differently (see
models/sparse_lr.py): key caching = the owner keeps the slot indices resolved
by the pull and the push sends only values; fixing-float = ``ff_encode`` /
``ff_decode`` kernels around the RCCL exchange; no compression on xGMI.
"""
from __future__ import annotations

import threading

import numpy as np

from ..ops.native import core


class Filter:
    def encode(self, msg):
        pass

    def decode(self, msg):
        pass


class KeyCachingFilter(Filter):
    """Do not resend an identical key list (src/filter/key_caching.h:6-76).
    Signature = crc32c of the first <= 2048 key bytes + size; cache key =
    (key_channel, key_range). ``clear_cache_if_done`` drops the entry after a PUSH
    request or any reply."""

    MAX_SIG_LEN = 2048

    def __init__(self):
        self.cache = {}
        self.mu = threading.Lock()

    @staticmethod
    def _sig(key: np.ndarray) -> int:
        b = key.view(np.uint8)[: KeyCachingFilter.MAX_SIG_LEN]
        return core().crc32c(b.tobytes())

    @staticmethod
    def _done(task) -> bool:
        return (not task.get("request")) or task.get("shared_para", {}).get("cmd") == "PUSH"

    def _ck(self, msg):
        return (msg.task.get("key_channel", 0), tuple(msg.task.get("key_range", [0, (1 << 64) - 1])))

    def encode(self, msg):
        conf = msg.find_filter("KEY_CACHING")
        if conf is None:
            return
        if msg.key is None:
            conf.pop("signature", None)
            return
        sig = self._sig(msg.key)
        conf["signature"] = sig
        ck = self._ck(msg)
        with self.mu:
            hit = self.cache.get(ck)
            if hit is not None and hit[0] == sig and hit[1].size == msg.key.size:
                msg.key = None
                msg.task["has_key"] = False
                conf["key_size"] = int(hit[1].size)
            else:
                self.cache[ck] = (sig, msg.key)
            if conf.get("clear_cache_if_done") and self._done(msg.task):
                self.cache.pop(ck, None)

    def decode(self, msg):
        conf = msg.find_filter("KEY_CACHING")
        if conf is None or "signature" not in conf:
            return
        sig = conf["signature"]
        ck = self._ck(msg)
        with self.mu:
            if msg.key is not None:
                if self._sig(msg.key) != sig:
                    raise RuntimeError("key caching: signature mismatch")
                self.cache[ck] = (sig, msg.key)
            else:
                hit = self.cache.get(ck)
                if hit is None or hit[0] != sig:
                    raise RuntimeError(f"key caching: cache miss for {ck}")
                msg.key = hit[1]
                msg.task["has_key"] = True
            if conf.get("clear_cache_if_done") and self._done(msg.task):
                self.cache.pop(ck, None)


class CompressingFilter(Filter):
    """Compress the key and each value frame (src/filter/compressing.h:6-39). The
    reference uses snappy; zlib level 1 (C++, _pscore) here."""

    def encode(self, msg):
        conf = msg.find_filter("COMPRESSING")
        if conf is None or conf.get("done"):
            return
        C = core()
        sizes = []
        if msg.key is not None:
            raw = msg.key.tobytes()
            sizes.append(len(raw))
            conf["key_dtype"] = msg.key.dtype.str
            msg.key = np.frombuffer(C.zlib_compress(raw, 1), dtype=np.uint8)
        vals = []
        conf["value_dtype"] = []
        for v in msg.value:
            raw = v.tobytes()
            sizes.append(len(raw))
            conf["value_dtype"].append(v.dtype.str)
            vals.append(np.frombuffer(C.zlib_compress(raw, 1), dtype=np.uint8))
        msg.value = vals
        conf["uncompressed_size"] = sizes
        conf["done"] = True

    def decode(self, msg):
        conf = msg.find_filter("COMPRESSING")
        if conf is None or not conf.get("done"):
            return
        C = core()
        sizes = list(conf["uncompressed_size"])
        if msg.key is not None and "key_dtype" in conf:
            n = sizes.pop(0)
            msg.key = np.frombuffer(C.zlib_decompress(msg.key.tobytes(), n), dtype=np.dtype(conf["key_dtype"])).copy()
        msg.value = [np.frombuffer(C.zlib_decompress(v.tobytes(), n), dtype=np.dtype(dt)).copy()
                     for v, n, dt in zip(msg.value, sizes, conf["value_dtype"])]
        conf["done"] = False


class FixingFloatFilter(Filter):
    """Fixed-point compression of float value arrays (src/filter/fixing_float.h)."""

    def encode(self, msg):
        import torch

        from ..ops import fixing_float as ff

        conf = msg.find_filter("FIXING_FLOAT")
        if conf is None:
            return
        fps = conf.setdefault("fixed_point", [])
        k = 0
        out = []
        for v in msg.value:
            if v.dtype in (np.float32, np.float64):
                if k >= len(fps):
                    fps.append({"num_bytes": 3})
                fp = fps[k]
                k += 1
                nb = int(fp.get("num_bytes", 3))
                x = torch.from_numpy(v.astype(np.float32))
                mm = None
                if "min_value" in fp and "max_value" in fp:
                    mm = torch.tensor([fp["min_value"], fp["max_value"]], dtype=torch.float32)
                code, mm = ff.encode(x, nb, mm)
                fp["min_value"], fp["max_value"] = float(mm[0]), float(mm[1])
                fp["orig_dtype"] = v.dtype.str
                out.append(code.numpy())
            else:
                out.append(v)
        msg.value = out

    def decode(self, msg):
        import torch

        from ..ops import fixing_float as ff

        conf = msg.find_filter("FIXING_FLOAT")
        if conf is None:
            return
        fps = conf.get("fixed_point", [])
        k = 0
        out = []
        for v in msg.value:
            if k < len(fps) and "orig_dtype" in fps[k] and v.dtype == np.uint8:
                fp = fps[k]
                k += 1
                nb = int(fp["num_bytes"])
                mm = torch.tensor([fp["min_value"], fp["max_value"]], dtype=torch.float32)
                x = ff.decode(torch.from_numpy(v.copy()), nb, mm).numpy()
                out.append(x.astype(np.dtype(fp["orig_dtype"])))
            else:
                out.append(v)
        msg.value = out


class SparseFilter(Filter):
    """Mark filtered entries with NaN (all-ones bit pattern); test with v != v
    (src/filter/sparse_filter.h). Darlin's KKT filter uses it."""

    @staticmethod
    def mark(v: np.ndarray, mask: np.ndarray):
        v[mask] = np.nan

    @staticmethod
    def marked(v: np.ndarray) -> np.ndarray:
        return v != v


_REG = {"KEY_CACHING": KeyCachingFilter, "COMPRESSING": CompressingFilter,
        "FIXING_FLOAT": FixingFloatFilter, "SPARSE": SparseFilter}


def create_filter(ftype: str) -> Filter:
    if ftype not in _REG:
        raise ValueError(f"unknown filter {ftype}")
    return _REG[ftype]()
