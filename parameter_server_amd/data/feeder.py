"""File -> HBM minibatch feeder: the device-side half of the reference's
``MinibatchReader`` (src/learner/sgd.h:103-157, a producer thread bounded by
``data_buf`` MB that reads ``minibatch``-row matrices ahead of the worker).

Three stages overlap, so a training step on the GPU never waits for text parsing
as long as the parser keeps up on average:

1. ``StreamReader`` (data/__init__.py): the C++ text parser (``_pscore.parse_text``,
   csrc/core/data.cc, ``nthreads`` parser threads per file chunk) on a producer
   thread; minibatches are cut at ``minibatch`` rows AND at ``max_nnz`` features
   (the trainer's localisation workspace), keys reduced mod ``num_features`` inside
   the parser (hashing trick; 0 keeps raw 64-bit keys).
2. a staging thread copies each minibatch into one of ``depth`` **pinned** host slots
   and issues its host->HBM copy on a dedicated copy stream (``non_blocking``), then
   records an event. A pinned slot is refilled only after its previous copy finished
   (host wait on that event); a device slot only after the step that read it was
   issued (the copy stream waits on the consumer's release event -- a GPU-side wait).
3. the consumer (``__iter__``) makes the current stream wait for the batch's copy
   event and hands out device views; ``release(batch)`` after issuing the step.

With ``device="cpu"`` the same interface yields CPU tensors (no pinned memory, no
streams): the CPU test path of the GPU app."""
from __future__ import annotations

import queue
import threading
from dataclasses import dataclass

import numpy as np
import torch

from . import StreamReader


@dataclass
class DeviceBatch:
    keys: torch.Tensor           # int64 [nnz] (raw or mod num_features)
    labels: torch.Tensor         # float32 [B]
    row_ptr: torch.Tensor        # int64 [B + 1]
    vals: torch.Tensor | None    # float32 [nnz] or None (binary features)
    rows: int
    nnz: int
    slot: int = -1
    width: int = 0               # > 0: every row has exactly this many features


class DeviceFeeder:
    def __init__(self, files, fmt: str, minibatch: int, max_nnz: int, device, *,
                 num_features: int = 0, passes: int = 1, shuffle: bool = False, seed: int = 0,
                 data_buf_mb: int = 1000, nthreads: int = 4, depth: int = 3,
                 ignore_slot: bool = True, hadoop_home: str = "", max_lines_per_file: int = -1):
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.minibatch, self.max_nnz = int(minibatch), int(max_nnz)
        self.reader = StreamReader(files, fmt, minibatch, ignore_slot=ignore_slot,
                                   data_buf_mb=data_buf_mb, hash_mod=int(num_features),
                                   passes=passes, shuffle=shuffle, seed=seed,
                                   hadoop_home=hadoop_home, max_lines_per_file=max_lines_per_file,
                                   max_nnz=self.max_nnz, nthreads=nthreads)
        self.depth = max(2, int(depth))
        self.num_examples = 0
        self.bytes_h2d = 0
        self._ready: queue.Queue = queue.Queue(maxsize=self.depth)
        self._free: queue.Queue = queue.Queue()
        self._error: BaseException | None = None
        self._thread = None
        if self.gpu:
            B, n = self.minibatch, self.max_nnz
            pin = dict(pin_memory=True)
            self._h = [dict(keys=torch.empty(n, dtype=torch.int64, **pin),
                            vals=torch.empty(n, dtype=torch.float32, **pin),
                            labels=torch.empty(B, dtype=torch.float32, **pin),
                            row_ptr=torch.empty(B + 1, dtype=torch.int64, **pin))
                       for _ in range(self.depth)]
            dev = self.device
            self._d = [dict(keys=torch.empty(n, dtype=torch.int64, device=dev),
                            vals=torch.empty(n, dtype=torch.float32, device=dev),
                            labels=torch.empty(B, dtype=torch.float32, device=dev),
                            row_ptr=torch.empty(B + 1, dtype=torch.int64, device=dev))
                       for _ in range(self.depth)]
            self._copy_stream = torch.cuda.Stream(self.device)
            self._h2d_done = [torch.cuda.Event() for _ in range(self.depth)]
            self._released = [torch.cuda.Event() for _ in range(self.depth)]
            self._used = [False] * self.depth
        for s in range(self.depth):
            self._free.put(s)

    # ------------------------------------------------------------ staging thread
    def _stage(self):
        try:
            for b in self.reader:
                B, n = b.rows, b.nnz
                if B > self.minibatch or n > self.max_nnz:
                    raise ValueError(f"minibatch of {B} rows / {n} features exceeds the feeder "
                                     f"capacity {self.minibatch} / {self.max_nnz}")
                keys = torch.from_numpy(np.ascontiguousarray(b.keys).view(np.int64))
                labels = torch.from_numpy(np.ascontiguousarray(b.labels, dtype=np.float32))
                row_ptr = torch.from_numpy(np.ascontiguousarray(b.row_ptr, dtype=np.int64))
                # all-ones values (one-hot LIBSVM rows) are binary features: the trainer's
                # binary / fixed-width paths apply and no value array is copied
                vals = (None if b.vals is None or bool(np.all(b.vals == 1.0)) else
                        torch.from_numpy(np.ascontiguousarray(b.vals, dtype=np.float32)))
                rp = np.asarray(b.row_ptr)
                width = n // B if B and n % B == 0 and np.all(np.diff(rp) == n // B) else 0
                if not self.gpu:
                    self._ready.put(DeviceBatch(keys.clone(), labels.clone(), row_ptr.clone(),
                                                None if vals is None else vals.clone(), B, n,
                                                width=width))
                    continue
                s = self._free.get()
                h, d = self._h[s], self._d[s]
                if self._used[s]:
                    self._h2d_done[s].synchronize()  # pinned slot: its last copy is done
                h["keys"][:n].copy_(keys)
                h["labels"][:B].copy_(labels)
                h["row_ptr"][:B + 1].copy_(row_ptr)
                if vals is not None:
                    h["vals"][:n].copy_(vals)
                cs = self._copy_stream
                if self._used[s]:
                    cs.wait_event(self._released[s])  # device slot: its step was issued
                with torch.cuda.stream(cs):
                    d["keys"][:n].copy_(h["keys"][:n], non_blocking=True)
                    d["labels"][:B].copy_(h["labels"][:B], non_blocking=True)
                    d["row_ptr"][:B + 1].copy_(h["row_ptr"][:B + 1], non_blocking=True)
                    if vals is not None:
                        d["vals"][:n].copy_(h["vals"][:n], non_blocking=True)
                    self._h2d_done[s].record(cs)
                self._used[s] = True
                self.bytes_h2d += n * (8 + (4 if vals is not None else 0)) + B * 12 + 8
                self._ready.put(DeviceBatch(d["keys"][:n], d["labels"][:B], d["row_ptr"][:B + 1],
                                            None if vals is None else d["vals"][:n], B, n, s,
                                            width))
        except BaseException as e:  # noqa: BLE001  (re-raised by the consumer)
            self._error = e
        finally:
            self._ready.put(None)

    def start(self):
        self._thread = threading.Thread(target=self._stage, daemon=True, name="device-feeder")
        self._thread.start()
        return self

    # ------------------------------------------------------------ consumer
    def __iter__(self):
        if self._thread is None:
            self.start()
        while True:
            b = self._ready.get()
            if b is None:
                if self._error is not None:
                    raise self._error
                return
            if self.gpu:  # the step's stream waits for the batch's host->HBM copy
                torch.cuda.current_stream(self.device).wait_event(self._h2d_done[b.slot])
            self.num_examples += b.rows
            yield b

    def release(self, b: DeviceBatch):
        """The step reading ``b`` has been issued on the current stream: its device slot
        may be refilled behind it."""
        if self.gpu and b.slot >= 0:
            self._released[b.slot].record(torch.cuda.current_stream(self.device))
            self._free.put(b.slot)
