"""Per-feature-group (slot) batch loader for Darlin BCD with a local disk cache.

Reference ``SlotReader`` (src/data/slot_reader.cc:31-197): parses every file of
the worker's shard (thread pool), splits examples by slot, writes each slot of
each file to ``<cache><file>.{colidx,rowsiz,value}`` plus an ``.info`` summary,
reuses the cache when the ``.info`` file exists, and serves ``index(slot)``
(keys), ``offset(slot)`` (CSR row pointer over ALL examples) and
``value(slot)``; slot 0 is the label.

Here files are parsed by the C++ runtime (``_pscore.parse_text``), the cache is
``.npy`` arrays (loaded with ``allow_pickle=False``) plus a JSON ``.info``, and
slot info follows the reference ``InfoParser`` (src/data/info_parser.cc:10-48):
``max_key`` is exclusive (max + 1), label slot 0 has range [0, 1).
"""
from __future__ import annotations

import json
import os
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field

import numpy as np

from . import merge_example_info, parse_text, read_file


@dataclass
class SlotData:
    """Examples of one worker split by feature group.

    ``groups[g] = (offset int64[rows+1], keys uint64[nnz], vals float32[nnz] | None)``
    """

    labels: np.ndarray
    groups: dict = field(default_factory=dict)

    @property
    def rows(self) -> int:
        return int(self.labels.size)

    def info(self) -> dict:
        """ExampleInfo-like summary: {num_ex, slots: {id: {min_key, max_key, nnz_ele, nnz_ex}}}."""
        slots = {0: {"min_key": 0, "max_key": 1, "nnz_ele": self.rows, "nnz_ex": self.rows}}
        for g, (off, keys, _) in self.groups.items():
            if keys.size == 0:
                continue
            slots[g] = {"min_key": int(keys.min()), "max_key": int(keys.max()) + 1,
                        "nnz_ele": int(keys.size), "nnz_ex": int(np.count_nonzero(np.diff(off)))}
        return {"num_ex": self.rows, "slots": slots}

    @staticmethod
    def from_batch(batch) -> "SlotData":
        """Split a CSR ``ExampleBatch`` (with per-nnz slot ids) into slots."""
        rows = batch.rows
        row_of = np.repeat(np.arange(rows, dtype=np.int64), np.diff(batch.row_ptr))
        out = SlotData(labels=batch.labels.astype(np.float32))
        for g in np.unique(batch.slots):
            m = batch.slots == g
            r = row_of[m]
            off = np.zeros(rows + 1, dtype=np.int64)
            np.cumsum(np.bincount(r, minlength=rows), out=off[1:])
            out.groups[int(g)] = (off, batch.keys[m].astype(np.uint64),
                                  None if batch.vals is None else batch.vals[m].astype(np.float32))
        return out

    @staticmethod
    def concat(parts: list["SlotData"]) -> "SlotData":
        if len(parts) == 1:
            return parts[0]
        out = SlotData(labels=np.concatenate([p.labels for p in parts]))
        gids = sorted({g for p in parts for g in p.groups})
        for g in gids:
            offs, keys, vals = [np.zeros(1, np.int64)], [], []
            binary = all(p.groups.get(g, (None, None, None))[2] is None for p in parts)
            base = 0
            for p in parts:
                if g in p.groups:
                    off, k, v = p.groups[g]
                else:
                    off, k, v = np.zeros(p.rows + 1, np.int64), np.zeros(0, np.uint64), None
                offs.append(off[1:] + base)
                base += int(off[-1])
                keys.append(k)
                if not binary:
                    vals.append(np.ones(k.size, np.float32) if v is None else v)
            out.groups[g] = (np.concatenate(offs), np.concatenate(keys),
                             None if binary else np.concatenate(vals))
        return out


class SlotReader:
    def __init__(self, files, fmt: str = "LIBSVM", cache_prefix: str | None = None,
                 ignore_slot: bool = False, hadoop_home: str = "", nthreads: int = 4):
        self.files = list(files)
        self.fmt = fmt
        self.cache = cache_prefix
        self.ignore_slot = ignore_slot
        self.hadoop = hadoop_home
        self.nthreads = max(1, nthreads)
        self.hit_cache = 0

    @staticmethod
    def from_config(data_conf, cache_conf=None, nthreads: int = 4) -> "SlotReader":
        cache = None
        if cache_conf is not None and cache_conf.has("file") and cache_conf.file:
            cache = cache_conf.file[0]
        hadoop = data_conf.hdfs.home if data_conf.has("hdfs") else ""
        return SlotReader(list(data_conf.file), data_conf.text, cache,
                          data_conf.ignore_feature_group, hadoop, nthreads)

    def _cache_name(self, path: str) -> str:
        return f"{self.cache}{os.path.basename(path)}"

    def _load_cached(self, path: str) -> SlotData | None:
        if not self.cache:
            return None
        base = self._cache_name(path)
        try:
            with open(base + ".info") as f:
                info = json.load(f)
        except (OSError, ValueError):
            return None
        labels = np.load(base + ".label.npy", allow_pickle=False)
        sd = SlotData(labels=labels)
        for g in info["groups"]:
            off = np.load(f"{base}.{g}.rowsiz.npy", allow_pickle=False)
            keys = np.load(f"{base}.{g}.colidx.npy", allow_pickle=False)
            vf = f"{base}.{g}.value.npy"
            vals = np.load(vf, allow_pickle=False) if os.path.exists(vf) else None
            offset = np.zeros(labels.size + 1, np.int64)
            np.cumsum(off.astype(np.int64), out=offset[1:])
            sd.groups[int(g)] = (offset, keys, vals)
        return sd

    def _store_cache(self, path: str, sd: SlotData):
        if not self.cache:
            return
        base = self._cache_name(path)
        os.makedirs(os.path.dirname(base) or ".", exist_ok=True)
        np.save(base + ".label.npy", sd.labels, allow_pickle=False)
        for g, (off, keys, vals) in sd.groups.items():
            # per-example row sizes (uint16 in the reference; uint32 here)
            np.save(f"{base}.{g}.rowsiz.npy", np.diff(off).astype(np.uint32), allow_pickle=False)
            np.save(f"{base}.{g}.colidx.npy", keys, allow_pickle=False)
            if vals is not None:
                np.save(f"{base}.{g}.value.npy", vals, allow_pickle=False)
        with open(base + ".info", "w") as f:  # written last: marks the cache complete
            json.dump({"groups": sorted(sd.groups), "info": _jsonable(sd.info())}, f)

    def _read_one(self, path: str) -> SlotData:
        sd = self._load_cached(path)
        if sd is not None:
            self.hit_cache += 1
            return sd
        batch = parse_text(read_file(path, self.hadoop), self.fmt, ignore_slot=self.ignore_slot)
        sd = SlotData.from_batch(batch)
        self._store_cache(path, sd)
        return sd

    def read(self) -> SlotData:
        self.hit_cache = 0
        with ThreadPoolExecutor(self.nthreads) as pool:
            parts = list(pool.map(self._read_one, self.files))
        if not parts:
            return SlotData(labels=np.zeros(0, np.float32))
        return SlotData.concat(parts)


def _jsonable(info: dict) -> dict:
    return {"num_ex": info["num_ex"], "slots": {str(k): v for k, v in info["slots"].items()}}


def merge_slot_info(infos: list[dict]) -> dict:
    """Sum of per-worker infos (reference mergeExampleInfo, data/common.cc:120-150)."""
    slots = merge_example_info([{int(k): v for k, v in i["slots"].items()} for i in infos])
    return {"num_ex": sum(i["num_ex"] for i in infos), "slots": slots}
