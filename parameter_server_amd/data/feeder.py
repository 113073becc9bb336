"""File -> HBM minibatch feeder: the device-side half of the reference's
``MinibatchReader`` (src/learner/sgd.h:103-157, a producer thread bounded by
``data_buf`` MB that reads ``minibatch``-row matrices ahead of the worker).

Two sources, the same consumer interface (``__iter__`` yields ``DeviceBatch`` views of
device slots; ``release(batch)`` after the step that reads it was issued):

* **text** (``StreamReader``, data/__init__.py): the C++ text parser
  (``_pscore.parse_text``, csrc/core/data.cc, ``nthreads`` parser threads per file) on a
  producer thread; minibatches cut at ``minibatch`` rows AND at ``max_nnz`` features (the
  trainer's localisation workspace), keys reduced mod ``num_features`` inside the parser
  (hashing trick; 0 keeps raw 64-bit keys). A staging thread copies each minibatch into
  one of ``depth`` pinned host slots and issues its host->HBM copy on a copy stream.
  With ``cache_dir`` every parsed file is also written as a binary cache file
  (data/bincache.py) -- the reference's SlotReader cache semantics
  (src/data/slot_reader.cc:60-155): written on the first text pass, reused by later
  passes and later runs while the source file is unchanged.
* **cache** (every file of the run has a valid cache): no parsing and no per-batch host
  pass over the features. ``io_threads`` reader threads ``pread`` each minibatch's
  contiguous sections (labels, u32 / u64 keys, values, row offsets) straight into a
  pinned slot; the consumer issues the slot's host->HBM copies (u32 keys widened to
  int64 on the device) on the copy stream in minibatch order. A pinned slot is refilled
  after its copy completed, a device slot after the step that read it was issued (a
  GPU-side wait). The number of minibatches is known up front (``planned_batches``), so
  a multi-rank app agrees on its step count once instead of every step.

With ``device="cpu"`` the same interface yields CPU tensors (no pinned memory, no
streams): the CPU test path of the GPU app."""
from __future__ import annotations

import os
import queue
import random
import threading
from dataclasses import dataclass

import numpy as np
import torch

from . import TEXT_FORMATS, StreamReader
from . import bincache


@dataclass
class DeviceBatch:
    keys: torch.Tensor           # int64 [nnz] (raw or mod num_features)
    labels: torch.Tensor         # float32 [B]
    row_ptr: torch.Tensor | None  # int64 [B + 1]; None when every row has ``width`` features
    vals: torch.Tensor | None    # float32 [nnz] or None (binary features)
    rows: int
    nnz: int
    slot: int = -1
    width: int = 0               # > 0: every row has exactly this many features


class DeviceFeeder:
    def __init__(self, files, fmt: str, minibatch: int, max_nnz: int, device, *,
                 num_features: int = 0, passes: int = 1, shuffle: bool = False, seed: int = 0,
                 data_buf_mb: int = 1000, nthreads: int = 4, depth: int = 3,
                 ignore_slot: bool = True, hadoop_home: str = "", max_lines_per_file: int = -1,
                 cache_dir: str | None = None, io_threads: int = 4):
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self.files = list(files)
        self.fmt = fmt
        self.minibatch, self.max_nnz = int(minibatch), int(max_nnz)
        self.num_features = int(num_features)
        self.passes = max(1, int(passes))
        self.shuffle = shuffle
        self.rng = random.Random(seed)
        self.ignore_slot = ignore_slot
        self.nthreads, self.data_buf_mb = nthreads, data_buf_mb
        self.hadoop_home, self.max_lines = hadoop_home, max_lines_per_file
        # (a line cap changes what a cache would hold: no cache then)
        self.cache_dir = cache_dir if (cache_dir and max_lines_per_file <= 0) else None
        if self.cache_dir:
            os.makedirs(self.cache_dir, exist_ok=True)
        self.io_threads = max(1, int(io_threads))
        # (cached streaming: a pinned slot per reader thread plus two in flight)
        self.depth = max(2, int(depth), self.io_threads + 2 if self.cache_dir else 0)
        self.num_examples = 0
        self.bytes_h2d = 0
        self.text_passes = 0    # passes that parsed text
        self.cached_passes = 0  # passes streamed from the binary cache
        self._fmt_id = TEXT_FORMATS.get(fmt, 0) if isinstance(fmt, str) else int(fmt)
        # the pass order of the files (StreamReader's per-pass shuffle)
        self._orders = []
        for _ in range(self.passes):
            order = list(self.files)
            if self.shuffle:
                self.rng.shuffle(order)
            self._orders.append(order)
        self._caches = self._open_caches()
        self._error: BaseException | None = None
        self._mode = "text"
        self._vcache = {}
        self._alloc_slots(self.depth)

    # ------------------------------------------------------------ setup
    def _open_caches(self):
        """{file: CacheFile} when every file has a valid cache, else None."""
        if not self.cache_dir:
            return None
        out = {}
        for f in self.files:
            cf = bincache.open_valid(f, self.cache_dir, self.fmt, self._fmt_id,
                                     self.num_features, self.ignore_slot)
            if cf is None:
                for c in out.values():
                    c.close()
                return None
            out[f] = cf
        return out

    def _alloc_slots(self, depth: int):
        self.depth = depth
        self._free: queue.Queue = queue.Queue()
        if self.gpu:
            B, n = self.minibatch, self.max_nnz
            pin = dict(pin_memory=True)
            # host slots as raw bytes: the cache reads u32 or u64 keys into them
            self._h = [dict(keys=torch.empty(8 * n, dtype=torch.uint8, **pin),
                            vals=torch.empty(n, dtype=torch.float32, **pin),
                            labels=torch.empty(B, dtype=torch.float32, **pin),
                            row_ptr=torch.empty(B + 1, dtype=torch.int64, **pin))
                       for _ in range(depth)]
            dev = self.device
            self._d = [dict(keys=torch.empty(n, dtype=torch.int64, device=dev),
                            keys32=torch.empty(n, dtype=torch.int32, device=dev),
                            vals=torch.empty(n, dtype=torch.float32, device=dev),
                            labels=torch.empty(B, dtype=torch.float32, device=dev),
                            row_ptr=torch.empty(B + 1, dtype=torch.int64, device=dev))
                       for _ in range(depth)]
            self._copy_stream = torch.cuda.Stream(self.device)
            self._h2d_done = [torch.cuda.Event() for _ in range(depth)]
            self._released = [torch.cuda.Event() for _ in range(depth)]
            self._used = [False] * depth
        for s in range(depth):
            self._free.put(s)

    def _views(self, s: int, B: int, n: int, rp: bool, vals: bool):
        """Device-slot views of one minibatch shape, the SAME tensor objects whenever the
        shape repeats: the trainer caches its native launch lists per tensor identity, so
        fresh views every step would rebuild (and re-validate) them every step."""
        key = (s, B, n, rp, vals)
        v = self._vcache.get(key)
        if v is None:
            d = self._d[s]
            if len(self._vcache) > 64:
                self._vcache.clear()
            v = self._vcache[key] = (d["keys"][:n], d["labels"][:B],
                                     d["row_ptr"][:B + 1] if rp else None,
                                     d["vals"][:n] if vals else None)
        return v

    # ------------------------------------------------------------ planning (cache)
    def _plan_pass(self, order) -> list[list[tuple]]:
        """Minibatches of one cached pass: lists of (CacheFile, row a, row b) segments, at
        most ``minibatch`` rows and ``max_nnz`` features each (StreamReader._cut rules;
        a minibatch continues into the next file)."""
        out, cur, rows, nnz = [], [], 0, 0
        for f in order:
            cf = self._caches[f]
            rp = None if cf.fixed else cf.row_ptr()
            r = 0
            while r < cf.rows:
                room_r = self.minibatch - rows
                if cf.fixed:
                    fit = room_r if cf.width == 0 else min(room_r, (self.max_nnz - nnz) // cf.width)
                    b = min(cf.rows, r + fit)
                else:
                    lim = int(rp[r]) + self.max_nnz - nnz
                    b = min(cf.rows, r + room_r,
                            int(np.searchsorted(rp, lim, side="right")) - 1)
                if b <= r:
                    if rows == 0:
                        raise ValueError(f"{f}: an example has more features than the "
                                         f"per-minibatch capacity {self.max_nnz}")
                    out.append(cur)
                    cur, rows, nnz = [], 0, 0
                    continue
                cur.append((cf, r, b))
                nnz += cf.nnz_at(b) - cf.nnz_at(r)
                rows += b - r
                r = b
                if rows == self.minibatch or nnz == self.max_nnz:
                    out.append(cur)
                    cur, rows, nnz = [], 0, 0
        if cur:
            out.append(cur)
        return out

    def planned_batches(self) -> int | None:
        """Minibatches of the whole run when every pass streams from the cache (known
        before the first step), else None."""
        if self._caches is None:
            return None
        return sum(self.planned_pass(p) for p in range(self.passes))

    def planned_pass(self, p: int) -> int | None:
        """Minibatches of pass ``p`` when it will stream from the cache (every file has a
        valid cache now), else None."""
        if self._caches is None:
            return None
        if getattr(self, "_plans", None) is None:
            self._plans = [None] * self.passes
        if self._plans[p] is None:
            self._plans[p] = self._plan_pass(self._orders[p])
        return len(self._plans[p])

    # ------------------------------------------------------------ text staging
    def _stage_text(self, order, out_q: queue.Queue):
        try:
            reader = StreamReader(order, self.fmt, self.minibatch, ignore_slot=self.ignore_slot,
                                  data_buf_mb=self.data_buf_mb, hash_mod=self.num_features,
                                  passes=1, shuffle=False, hadoop_home=self.hadoop_home,
                                  max_lines_per_file=self.max_lines, max_nnz=self.max_nnz,
                                  nthreads=self.nthreads, cache_dir=self.cache_dir)
            for b in reader:
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
                    out_q.put(DeviceBatch(keys.clone(), labels.clone(), row_ptr.clone(),
                                          None if vals is None else vals.clone(), B, n,
                                          width=width))
                    continue
                s = self._free.get()
                h, d = self._h[s], self._d[s]
                if self._used[s]:
                    self._h2d_done[s].synchronize()  # pinned slot: its last copy is done
                hk = h["keys"].view(torch.int64)
                hk[:n].copy_(keys)
                h["labels"][:B].copy_(labels)
                h["row_ptr"][:B + 1].copy_(row_ptr)
                if vals is not None:
                    h["vals"][:n].copy_(vals)
                cs = self._copy_stream
                if self._used[s]:
                    cs.wait_event(self._released[s])  # device slot: its step was issued
                with torch.cuda.stream(cs):
                    d["keys"][:n].copy_(hk[:n], non_blocking=True)
                    d["labels"][:B].copy_(h["labels"][:B], non_blocking=True)
                    d["row_ptr"][:B + 1].copy_(h["row_ptr"][:B + 1], non_blocking=True)
                    if vals is not None:
                        d["vals"][:n].copy_(h["vals"][:n], non_blocking=True)
                    self._h2d_done[s].record(cs)
                self._used[s] = True
                self.bytes_h2d += n * (8 + (4 if vals is not None else 0)) + B * 12 + 8
                v = self._views(s, B, n, True, vals is not None)
                out_q.put(DeviceBatch(v[0], v[1], v[2], v[3], B, n, s, width))
        except BaseException as e:  # noqa: BLE001  (re-raised by the consumer)
            self._error = e
        finally:
            out_q.put(None)

    def _iter_text(self, order):
        q: queue.Queue = queue.Queue(maxsize=self.depth)
        th = threading.Thread(target=self._stage_text, args=(order, q), daemon=True,
                              name="device-feeder")
        th.start()
        while True:
            b = q.get()
            if b is None:
                th.join()
                if self._error is not None:
                    raise self._error
                return
            if self.gpu:  # the step's stream waits for the batch's host->HBM copy
                torch.cuda.current_stream(self.device).wait_event(self._h2d_done[b.slot])
            yield b

    # ------------------------------------------------------------ cached streaming
    def _run_props(self):
        cfs = list(self._caches.values())
        kb = {c.key_bytes for c in cfs}
        if len(kb) != 1:
            raise ValueError("cache files of one run with different key widths")
        widths = {c.width if c.fixed else 0 for c in cfs}
        fixed = len(widths) == 1 and 0 not in widths
        return kb.pop(), any(c.has_vals for c in cfs), (widths.pop() if fixed else 0)

    def _fill(self, s: int, segs, kb: int, has_vals: bool, width: int) -> tuple[int, int]:
        """pread one minibatch into pinned slot s (reader thread)."""
        if self.gpu:
            h = self._h[s]
            lab = memoryview(h["labels"].numpy()).cast("B")
            keys = memoryview(h["keys"].numpy()).cast("B")
            vals = memoryview(h["vals"].numpy()).cast("B")
            rpv = h["row_ptr"].numpy()
        else:
            h = self._hc[s]
            lab, keys, vals = (memoryview(h["labels"]).cast("B"), memoryview(h["keys"]).cast("B"),
                               memoryview(h["vals"]).cast("B"))
            rpv = h["row_ptr"]
        rows = nnz = 0
        for cf, a, b in segs:
            rp_mv = None if width else memoryview(rpv).cast("B")[8 * rows:]
            r, n = cf.read_into(a, b, lab[4 * rows:], keys[kb * nnz:],
                                vals[4 * nnz:] if has_vals else None, rp_mv)
            if has_vals and not cf.has_vals:  # (binary file in a valued run)
                np.frombuffer(vals, dtype=np.float32)[nnz:nnz + n] = 1.0
            if not width:  # the file's offsets -> this minibatch's
                seg = rpv[rows:rows + r + 1]
                if cf.fixed:
                    seg[:] = np.arange(nnz, nnz + (r + 1) * cf.width, cf.width)
                else:
                    seg -= seg[0] - nnz
            rows += r
            nnz += n
        return rows, nnz

    def _iter_cached(self, plan):
        kb, has_vals, width = self._run_props()
        D = self.depth
        if not self.gpu:
            B, n = self.minibatch, self.max_nnz
            self._hc = [dict(labels=np.empty(B, np.float32), keys=np.empty(8 * n, np.uint8),
                             vals=np.empty(n, np.float32), row_ptr=np.empty(B + 1, np.int64))
                        for _ in range(D)]
        filled = [threading.Event() for _ in range(len(plan))]
        sizes = [None] * len(plan)
        slot_ok = [threading.Semaphore(1) for _ in range(D)]  # pinned slot free for refill
        nxt = {"i": 0}
        lock = threading.Lock()
        stop = threading.Event()

        def reader():
            try:
                while not stop.is_set():
                    with lock:
                        i = nxt["i"]
                        if i >= len(plan):
                            return
                        nxt["i"] = i + 1
                    s = i % D
                    while not slot_ok[s].acquire(timeout=0.5):  # (batch i - D consumed)
                        if stop.is_set():
                            return
                    if self.gpu and self._used[s]:
                        self._h2d_done[s].synchronize()  # its last copy finished
                    sizes[i] = self._fill(s, plan[i], kb, has_vals, width)
                    filled[i].set()
            except BaseException as e:  # noqa: BLE001
                self._error = e
                stop.set()
                for ev in filled:
                    ev.set()

        ths = [threading.Thread(target=reader, daemon=True, name=f"cache-reader-{k}")
               for k in range(min(self.io_threads, D))]
        for th in ths:
            th.start()
        try:
            for i in range(len(plan)):
                filled[i].wait()
                if self._error is not None:
                    raise self._error
                s = i % D
                B, n = sizes[i]
                if not self.gpu:
                    h = self._hc[s]
                    k = h["keys"][:kb * n].view(np.uint32 if kb == 4 else np.int64)
                    keys = torch.from_numpy(k.astype(np.int64))
                    b = DeviceBatch(keys, torch.from_numpy(h["labels"][:B].copy()),
                                    None if width else torch.from_numpy(h["row_ptr"][:B + 1].copy()),
                                    torch.from_numpy(h["vals"][:n].copy()) if has_vals else None,
                                    B, n, s, width)
                    slot_ok[s].release()
                    yield b
                    continue
                h, d = self._h[s], self._d[s]
                cs = self._copy_stream
                if self._used[s]:
                    cs.wait_event(self._released[s])  # the device slot's step was issued
                with torch.cuda.stream(cs):
                    if kb == 4:
                        d["keys32"][:n].copy_(h["keys"][:4 * n].view(torch.int32),
                                              non_blocking=True)
                        d["keys"][:n].copy_(d["keys32"][:n])  # u32 -> int64 on the device
                        d["keys"][:n].bitwise_and_(0xFFFFFFFF)
                    else:
                        d["keys"][:n].copy_(h["keys"][:8 * n].view(torch.int64),
                                            non_blocking=True)
                    d["labels"][:B].copy_(h["labels"][:B], non_blocking=True)
                    if not width:
                        d["row_ptr"][:B + 1].copy_(h["row_ptr"][:B + 1], non_blocking=True)
                    if has_vals:
                        d["vals"][:n].copy_(h["vals"][:n], non_blocking=True)
                    self._h2d_done[s].record(cs)
                self._used[s] = True
                slot_ok[s].release()  # (the reader syncs on the copy before refilling)
                self.bytes_h2d += n * (kb + (4 if has_vals else 0)) + B * 4 + \
                    (0 if width else 8 * (B + 1))
                torch.cuda.current_stream(self.device).wait_event(self._h2d_done[s])
                v = self._views(s, B, n, not width, has_vals)
                yield DeviceBatch(v[0], v[1], v[2], v[3], B, n, s, width)
        finally:
            stop.set()
            for th in ths:
                th.join(timeout=5)

    # ------------------------------------------------------------ consumer
    def __iter__(self):
        for p in range(self.passes):
            yield from self.iter_pass(p)

    def iter_pass(self, p: int):
        """The minibatches of pass ``p`` (text, or the binary cache once every file has
        one); passes run in order."""
        order = self._orders[p]
        self._mode = "text" if self._caches is None else "cache"
        if self._caches is None:
            self.text_passes += 1
            src = self._iter_text(order)
            if self.cache_dir:  # the caches exist after this pass
                src = self._then_open(src)
        else:
            self.cached_passes += 1
            self.planned_pass(p)
            src = self._iter_cached(self._plans[p])
        for b in src:
            self.num_examples += b.rows
            yield b

    def _then_open(self, src):
        yield from src
        self._caches = self._open_caches()

    def release(self, b: DeviceBatch):
        """The step reading ``b`` has been issued on the current stream: its device slot
        may be refilled behind it."""
        if self.gpu and b.slot >= 0:
            self._released[b.slot].record(torch.cuda.current_stream(self.device))
            if self._mode == "text":  # (cached streaming assigns slots round-robin)
                self._free.put(b.slot)
