"""Binary example cache: the text of a data file parsed ONCE into flat arrays on local
disk, reused by later passes and later runs (the reference keeps a per-slot binary cache
across runs, src/data/slot_reader.cc:60-155, and a binary RecordIO format,
src/util/recordio.h:17-77).

One cache file per data file (``<cache_dir>/<basename>.<digest>.psbin``)::

    header (4096 B): magic, version, rows, nnz, key bytes (4 for keys hashed mod
        <= 2^32, else 8), flags (values present, fixed width), width,
        hash_mod, format, ignore_slot, and the source file's size / mtime (a changed
        source invalidates the cache)
    labels  float32 [rows]
    row_ptr int64   [rows + 1]   (absent when every row has ``width`` features)
    keys    u32 / u64 [nnz]
    vals    float32 [nnz]        (absent for binary features: every value 1)

Every section starts on a 4 KiB boundary, so a minibatch is a few contiguous ``pread``
calls straight into pinned host memory (no parsing, no per-batch numpy pass): the
device feeder (data/feeder.py) streams it to HBM with asynchronous copies and widens u32
keys on the device.
"""
from __future__ import annotations

import hashlib
import os
import struct

import numpy as np

MAGIC = 0x43425350  # "PSBC"
VERSION = 1
HDR = 4096
_FMT = "<IIQQIIIIQIIQQ"  # magic ver rows nnz key_bytes flags width pad hash_mod fmt ign size mtime
F_VALS, F_FIXED = 1, 2


def _al(x: int) -> int:
    return (x + 4095) & ~4095


def cache_path(cache_dir: str, src: str, fmt, hash_mod: int, ignore_slot: bool) -> str:
    """The cache file of ``src`` under ``cache_dir`` (the digest keys the parse options)."""
    tag = f"{os.path.abspath(src)}|{fmt}|{int(hash_mod)}|{int(bool(ignore_slot))}"
    h = hashlib.sha1(tag.encode()).hexdigest()[:12]
    return os.path.join(cache_dir, f"{os.path.basename(src)}.{h}.psbin")


def _src_stamp(src: str) -> tuple[int, int]:
    try:
        st = os.stat(src)
        return int(st.st_size), int(st.st_mtime_ns)
    except OSError:  # (hdfs or vanished: no invalidation by stamp)
        return 0, 0


def write_cache(path: str, batch, *, src: str, fmt_id: int, hash_mod: int,
                ignore_slot: bool) -> str:
    """Write one parsed file (``data.ExampleBatch``, keys already reduced mod
    ``hash_mod`` by the parser) as a cache file (atomically: a temporary name renamed into
    place). Keys are u32 exactly when ``0 < hash_mod <= 2^32`` -- a property of the options,
    so every file of a run has the same key width. Returns ``path``."""
    rows, nnz = batch.rows, batch.nnz
    keys = np.ascontiguousarray(batch.keys).view(np.uint64)
    kb = 4 if 0 < int(hash_mod) <= (1 << 32) else 8
    rp = np.ascontiguousarray(batch.row_ptr, dtype=np.int64)
    w = rp[1:] - rp[:-1] if rows else np.zeros(0, np.int64)
    fixed = rows > 0 and bool((w == w[0]).all())
    width = int(w[0]) if fixed else 0
    vals = batch.vals
    has_vals = vals is not None and not bool(np.all(np.asarray(vals) == 1.0))
    flags = (F_VALS if has_vals else 0) | (F_FIXED if fixed else 0)
    size, mtime = _src_stamp(src)
    hdr = struct.pack(_FMT, MAGIC, VERSION, rows, nnz, kb, flags, width, 0, int(hash_mod),
                      int(fmt_id), int(bool(ignore_slot)), size, mtime)
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "wb") as f:
        def section(arr):
            pos = f.tell()
            f.write(b"\0" * (_al(pos) - pos))
            f.write(np.ascontiguousarray(arr).tobytes())

        f.write(hdr + b"\0" * (HDR - len(hdr)))
        section(np.asarray(batch.labels, dtype=np.float32))
        if not fixed:
            section(rp)
        section(keys.astype(np.uint32) if kb == 4 else keys)
        if has_vals:
            section(np.asarray(vals, dtype=np.float32))
        pos = f.tell()
        f.write(b"\0" * (_al(pos) - pos))
    os.replace(tmp, path)
    return path


class CacheFile:
    """An open cache file: its header, the byte offset of every section, and a ``pread``
    of any row range's arrays into caller buffers."""

    def __init__(self, path: str):
        self.path = path
        self.fd = os.open(path, os.O_RDONLY)
        raw = os.pread(self.fd, struct.calcsize(_FMT), 0)
        (magic, ver, self.rows, self.nnz, self.key_bytes, flags, self.width, _, self.hash_mod,
         self.fmt_id, self.ignore_slot, self.src_size, self.src_mtime) = struct.unpack(_FMT, raw)
        if magic != MAGIC or ver != VERSION:
            os.close(self.fd)
            raise ValueError(f"{path}: not a psamd example cache (or another version)")
        self.has_vals = bool(flags & F_VALS)
        self.fixed = bool(flags & F_FIXED)
        off = HDR
        self.o_labels = off
        off = _al(off + 4 * self.rows)
        self.o_rowptr = None
        if not self.fixed:
            self.o_rowptr = off
            off = _al(off + 8 * (self.rows + 1))
        self.o_keys = off
        off = _al(off + self.key_bytes * self.nnz)
        self.o_vals = None
        if self.has_vals:
            self.o_vals = off
            off = _al(off + 4 * self.nnz)
        if os.fstat(self.fd).st_size < off:
            os.close(self.fd)
            raise ValueError(f"{path}: truncated cache file")
        self._rp = None

    def close(self):
        if self.fd >= 0:
            os.close(self.fd)
            self.fd = -1

    def valid_for(self, src: str, hash_mod: int, fmt_id: int, ignore_slot: bool) -> bool:
        size, mtime = _src_stamp(src)
        return (self.hash_mod == int(hash_mod) and self.fmt_id == int(fmt_id)
                and bool(self.ignore_slot) == bool(ignore_slot)
                and (size, mtime) == (self.src_size, self.src_mtime))

    def row_ptr(self) -> np.ndarray:
        """The row offsets (memory-mapped; arithmetic for fixed-width rows)."""
        if self._rp is None:
            if self.fixed:
                self._rp = np.arange(0, (self.rows + 1) * self.width, self.width, dtype=np.int64) \
                    if self.rows else np.zeros(1, np.int64)
            else:
                self._rp = np.memmap(self.path, dtype=np.int64, mode="r", offset=self.o_rowptr,
                                     shape=(self.rows + 1,))
        return self._rp

    def nnz_at(self, r: int) -> int:
        return r * self.width if self.fixed else int(self.row_ptr()[r])

    def read_into(self, a: int, b: int, labels: memoryview, keys: memoryview,
                  vals: memoryview | None, row_ptr: memoryview | None) -> tuple[int, int]:
        """Rows [a, b): labels (4 B each), keys (key_bytes each), values and row offsets
        (the file's own, int64, rows + 1 of them) by ``pread`` into the given byte
        buffers. Returns (rows, nnz)."""
        s, e = self.nnz_at(a), self.nnz_at(b)
        _pread(self.fd, labels[:4 * (b - a)], self.o_labels + 4 * a)
        kb = self.key_bytes
        _pread(self.fd, keys[:kb * (e - s)], self.o_keys + kb * s)
        if vals is not None and self.has_vals:
            _pread(self.fd, vals[:4 * (e - s)], self.o_vals + 4 * s)
        if row_ptr is not None and not self.fixed:
            _pread(self.fd, row_ptr[:8 * (b - a + 1)], self.o_rowptr + 8 * a)
        return b - a, e - s


def _pread(fd: int, buf: memoryview, off: int) -> None:
    """Fill ``buf`` from ``off`` (the GIL is released inside the read system call)."""
    n, want = 0, len(buf)
    while n < want:
        got = os.preadv(fd, [buf[n:]], off + n)
        if got <= 0:
            raise EOFError(f"short read at offset {off + n}")
        n += got


def open_valid(src: str, cache_dir: str, fmt, fmt_id: int, hash_mod: int,
               ignore_slot: bool) -> CacheFile | None:
    """The valid cache of ``src`` or None (absent, stale or unreadable)."""
    p = cache_path(cache_dir, src, fmt, hash_mod, ignore_slot)
    if not os.path.exists(p):
        return None
    try:
        cf = CacheFile(p)
    except (OSError, ValueError, struct.error):
        return None
    if not cf.valid_for(src, hash_mod, fmt_id, ignore_slot):
        cf.close()
        return None
    return cf
