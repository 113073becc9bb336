"""RecordIO example files (DataConfig.format = PROTO).

Reference: RecordIO framing ``[magic 0x3ed7230a][u32 len][bytes]`` around
protobuf ``Example`` messages (src/util/recordio.h:9,17-77). The framing is the
C++ runtime's (``_pscore.recordio_pack/unpack``); without a protobuf runtime the
payload is a compact binary example record:
``f32 label | u16 nslots | per slot: i32 id, u32 n, u8 has_val, u64[n] keys, f32[n] vals``.
"""
from __future__ import annotations

import struct

import numpy as np

from ..ops.native import core
from . import ExampleBatch


def encode_examples(batch: ExampleBatch) -> bytes:
    recs = []
    for r in range(batch.rows):
        a, b = int(batch.row_ptr[r]), int(batch.row_ptr[r + 1])
        keys = batch.keys[a:b]
        slots = batch.slots[a:b]
        vals = None if batch.vals is None else batch.vals[a:b]
        ids = list(dict.fromkeys(slots.tolist()))
        parts = [struct.pack("<fH", float(batch.labels[r]), len(ids))]
        for sid in ids:
            m = slots == sid
            k = keys[m].astype(np.uint64)
            parts.append(struct.pack("<iIB", int(sid), int(k.size), 0 if vals is None else 1))
            parts.append(k.tobytes())
            if vals is not None:
                parts.append(vals[m].astype(np.float32).tobytes())
        recs.append(b"".join(parts))
    return core().recordio_pack(recs)


def decode_examples(data: bytes) -> ExampleBatch:
    labels, row_ptr, keys, vals, slots = [], [0], [], [], []
    has_any_val = False
    for rec in core().recordio_unpack(data):
        y, ns = struct.unpack_from("<fH", rec, 0)
        off = 6
        labels.append(y)
        n_row = 0
        for _ in range(ns):
            sid, n, hv = struct.unpack_from("<iIB", rec, off)
            off += 9
            k = np.frombuffer(rec, dtype=np.uint64, count=n, offset=off)
            off += 8 * n
            if hv:
                v = np.frombuffer(rec, dtype=np.float32, count=n, offset=off)
                off += 4 * n
                has_any_val = True
            else:
                v = np.ones(n, np.float32)
            keys.append(k)
            vals.append(v)
            slots.append(np.full(n, sid, np.int32))
            n_row += n
        row_ptr.append(row_ptr[-1] + n_row)
    cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)  # noqa: E731
    return ExampleBatch(np.asarray(labels, np.float32), np.asarray(row_ptr, np.int64),
                        cat(keys, np.uint64), cat(vals, np.float32) if has_any_val else None,
                        cat(slots, np.int32))
