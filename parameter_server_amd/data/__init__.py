"""Data ingestion: example batches, text/RecordIO readers, file partitioning.

Reference (src/data/): ExampleParser text formats (text_parser.cc), StreamReader
minibatch streaming (stream_reader.h), SlotReader per-feature-group loading with a
local disk cache (slot_reader.cc), searchFiles / divideFiles (data/common.cc).
Parsing runs in the C++ runtime (``_pscore.parse_text``, csrc/core/data.cc).
"""
from __future__ import annotations

import os
import random
import re
import threading
from dataclasses import dataclass, field

import numpy as np

from ..ops.native import core
from ..utils.threads import ThreadsafeLimitedQueue

TEXT_FORMATS = {"DENSE": 1, "SPARSE": 2, "SPARSE_BINARY": 3, "ADFEA": 4, "LIBSVM": 5,
                "TERAFEA": 6, "VW": 7, "CRITEO": 8}


@dataclass
class ExampleBatch:
    """CSR minibatch: row r has features keys[row_ptr[r]:row_ptr[r+1]]."""

    labels: np.ndarray
    row_ptr: np.ndarray
    keys: np.ndarray
    vals: np.ndarray | None
    slots: np.ndarray
    info: dict = field(default_factory=dict)

    @property
    def rows(self) -> int:
        return int(self.labels.size)

    @property
    def nnz(self) -> int:
        return int(self.keys.size)

    def slice_rows(self, a: int, b: int) -> "ExampleBatch":
        s, e = int(self.row_ptr[a]), int(self.row_ptr[b])
        return ExampleBatch(self.labels[a:b], self.row_ptr[a:b + 1] - s, self.keys[s:e],
                            None if self.vals is None else self.vals[s:e], self.slots[s:e])

    @staticmethod
    def concat(batches: list["ExampleBatch"]) -> "ExampleBatch":
        if len(batches) == 1:
            return batches[0]
        rp = [batches[0].row_ptr]
        off = int(batches[0].row_ptr[-1])
        for b in batches[1:]:
            rp.append(b.row_ptr[1:] + off)
            off += int(b.row_ptr[-1])
        vals = None if any(b.vals is None for b in batches) else np.concatenate([b.vals for b in batches])
        return ExampleBatch(np.concatenate([b.labels for b in batches]), np.concatenate(rp),
                            np.concatenate([b.keys for b in batches]), vals,
                            np.concatenate([b.slots for b in batches]))

    def to_torch(self, device="cpu", num_features: int = 0):
        """(keys int64, labels f32, row_ptr int64, vals f32|None) torch tensors;
        keys are reduced mod num_features when given (hashing trick)."""
        import torch

        k = self.keys
        if num_features:
            k = k % np.uint64(num_features)
        keys = torch.from_numpy(k.view(np.int64).copy()).to(device)
        labels = torch.from_numpy(self.labels.astype(np.float32)).to(device)
        row_ptr = torch.from_numpy(self.row_ptr.astype(np.int64)).to(device)
        vals = None if self.vals is None else torch.from_numpy(self.vals.astype(np.float32)).to(device)
        return keys, labels, row_ptr, vals


def parse_text(data: bytes, fmt: str | int, *, ignore_slot=False, shuffle_fea_id=False,
               hash_mod=0, nthreads=4, max_lines=-1) -> ExampleBatch:
    f = TEXT_FORMATS[fmt] if isinstance(fmt, str) else int(fmt)
    d = core().parse_text(data, f, ignore_slot, shuffle_fea_id, hash_mod, nthreads, max_lines)
    vals = None if d["binary"] else d["vals"]
    return ExampleBatch(d["labels"], d["row_ptr"], d["keys"], vals, d["slots"],
                        {"info": d["info"], "bad_lines": d["bad_lines"]})


# --------------------------------------------------------------------- files
def search_files(conf) -> list[str]:
    """Expand each ``file`` entry as a regex over its directory listing
    (reference searchFiles, src/data/common.cc:13-60)."""
    out = []
    hadoop = conf.hdfs.home if conf.has("hdfs") else ""
    for pat in conf.file:
        d, base = os.path.split(pat)
        d = d or "."
        if not any(ch in base for ch in "*?[]()|+^$\\"):
            out.append(pat)
            continue
        rx = re.compile(base)
        for name in core().list_dir(d, hadoop):
            if rx.fullmatch(name) or rx.match(name):
                out.append(os.path.join(d, name))
    return sorted(set(out))


def divide_files(files: list[str], n: int, max_per_part: int = -1) -> list[list[str]]:
    """Round-robin split of files over n workers (divideFiles, data/common.cc:152-167)."""
    parts = [[] for _ in range(n)]
    for i, f in enumerate(files):
        parts[i % n].append(f)
    if max_per_part > 0:
        parts = [p[:max_per_part] for p in parts]
    return parts


def read_file(path: str, hadoop_home: str = "") -> bytes:
    return core().read_file(path, hadoop_home)


def merge_example_info(infos: list[dict]) -> dict:
    out: dict = {}
    for info in infos:
        for sid, s in info.items():
            t = out.setdefault(sid, {"min_key": (1 << 64) - 1, "max_key": 0, "nnz_ele": 0,
                                     "nnz_ex": 0, "format": s.get("format", 0)})
            t["min_key"] = min(t["min_key"], s["min_key"])
            t["max_key"] = max(t["max_key"], s["max_key"])
            t["nnz_ele"] += s["nnz_ele"]
            t["nnz_ex"] += s["nnz_ex"]
    return out


# ------------------------------------------------------------- stream reader
class StreamReader:
    """Minibatch stream over a file list (reference StreamReader::readMatrices),
    with a producer thread bounded by ``data_buf`` MB (ProducerConsumer,
    src/util/producer_consumer.h)."""

    def __init__(self, files, fmt="LIBSVM", minibatch=1000, *, ignore_slot=False,
                 data_buf_mb=1000, hash_mod=0, passes=1, shuffle=False, seed=0, hadoop_home="",
                 max_lines_per_file=-1, recordio=False, max_nnz=0, nthreads=4,
                 cache_dir: str | None = None):
        self.files = list(files)
        # write every parsed text file as a binary cache there (data/bincache.py), once
        self.cache_dir = cache_dir if (cache_dir and not recordio) else None
        # a minibatch also ends before it exceeds max_nnz features (0 = no cap): a
        # device consumer sizes its workspaces for minibatch rows x a per-row bound
        self.max_nnz = int(max_nnz)
        self.nthreads = int(nthreads)
        self.fmt = fmt
        self.minibatch = minibatch
        self.ignore_slot = ignore_slot
        self.cap_bytes = max(1, data_buf_mb) << 20
        self.hash_mod = hash_mod
        self.passes = max(1, passes)
        self.shuffle = shuffle
        self.rng = random.Random(seed)
        self.hadoop = hadoop_home
        self.max_lines = max_lines_per_file
        self.recordio = recordio
        self._q = ThreadsafeLimitedQueue(self.cap_bytes)
        self._error: BaseException | None = None
        self._thread = None
        self.num_examples = 0

    def _file_order(self):
        for _ in range(self.passes):
            order = list(self.files)
            if self.shuffle:
                self.rng.shuffle(order)
            yield from order

    def _produce(self):
        pending: list[ExampleBatch] = []
        have = 0
        try:
            for f in self._file_order():
                raw = read_file(f, self.hadoop)
                if self.recordio:
                    from .recordio import decode_examples

                    b = decode_examples(raw)
                else:
                    b = parse_text(raw, self.fmt, ignore_slot=self.ignore_slot,
                                   hash_mod=self.hash_mod, max_lines=self.max_lines,
                                   nthreads=self.nthreads)
                    if self.cache_dir:
                        self._write_cache(f, b)
                pending.append(b)
                have += b.rows
                nnz = sum(x.nnz for x in pending)
                while have >= self.minibatch or (self.max_nnz and nnz > self.max_nnz):
                    allb = ExampleBatch.concat(pending)
                    r = self._cut(allb)
                    self._put(allb.slice_rows(0, r))
                    rest = allb.slice_rows(r, allb.rows)
                    pending, have = ([rest], rest.rows) if rest.rows else ([], 0)
                    nnz = rest.nnz if rest.rows else 0
            while have:
                allb = ExampleBatch.concat(pending)
                r = self._cut(allb)
                self._put(allb.slice_rows(0, r))
                rest = allb.slice_rows(r, allb.rows)
                pending, have = ([rest], rest.rows) if rest.rows else ([], 0)
        except BaseException as e:  # noqa: BLE001  (re-raised by the consumer)
            self._error = e
        finally:
            self._q.push(None, 0, finished=True)

    def _write_cache(self, f: str, b: ExampleBatch):
        from . import bincache

        fid = TEXT_FORMATS[self.fmt] if isinstance(self.fmt, str) else int(self.fmt)
        cf = bincache.open_valid(f, self.cache_dir, self.fmt, fid, self.hash_mod,
                                 self.ignore_slot)
        if cf is not None:  # (another pass or run wrote it already)
            cf.close()
            return
        bincache.write_cache(bincache.cache_path(self.cache_dir, f, self.fmt, self.hash_mod,
                                                 self.ignore_slot), b, src=f, fmt_id=fid,
                             hash_mod=self.hash_mod, ignore_slot=self.ignore_slot)

    def _cut(self, b: ExampleBatch) -> int:
        """Rows of the next minibatch: <= minibatch rows and <= max_nnz features."""
        r = min(self.minibatch, b.rows)
        if self.max_nnz and int(b.row_ptr[r]) > self.max_nnz:
            r = int(np.searchsorted(b.row_ptr, self.max_nnz, side="right")) - 1
            if r < 1:
                raise ValueError(f"an example has {int(b.row_ptr[1])} features > the "
                                 f"per-minibatch capacity {self.max_nnz}")
        return r

    def _put(self, b):
        self._q.push(b, max(1, b.keys.nbytes + b.labels.nbytes + b.row_ptr.nbytes))

    def start(self):
        self._thread = threading.Thread(target=self._produce, daemon=True, name="stream-reader")
        self._thread.start()
        return self

    def __iter__(self):
        if self._thread is None:
            self.start()
        while True:
            ok, b = self._q.pop()
            if not ok:
                if self._error is not None:
                    raise self._error
                return
            self.num_examples += b.rows
            yield b
