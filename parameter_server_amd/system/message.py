"""Messages: a task header plus a key array and value arrays.

Reference: ``Message`` (src/system/message.h:18-159) carries a protobuf ``Task``
(src/system/proto/task.proto:11-93), ``SArray<char> key``, ``vector<SArray<char>>
value``, routing fields and the ``recv_handle`` / ``fin_handle`` callbacks;
``sliceKeyOrderedMsg`` splits a sorted-key message into per-server pieces by
binary search on the key-range boundaries.

Here the header is a plain dict serialised with msgpack (no protobuf runtime),
arrays are numpy and travel as raw frames through the C++ Van.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import Any, Callable

import msgpack
import numpy as np

INVALID_TIME = -1
KEY_MAX = (1 << 64) - 1  # exclusive end of the key space (2^64-1 itself is reserved)

# Task.type
TERMINATE, TERMINATE_CONFIRM, REPLY, MANAGE, CALL_CUSTOMER, HEARTBEATING = 1, 2, 3, 4, 5, 6
# node groups (reference src/system/executor.h:8-18)
SERVER_GROUP = "all_servers"
WORKER_GROUP = "all_workers"
COMP_GROUP = "all_comp_nodes"
REPLICA_GROUP = "all_replicas"
OWNER_GROUP = "all_owners"
LIVE_GROUP = "all_lives"
GROUPS = (SERVER_GROUP, WORKER_GROUP, COMP_GROUP, REPLICA_GROUP, OWNER_GROUP, LIVE_GROUP)

_DT = {np.dtype(t).str: t for t in ("i1", "i2", "i4", "i8", "u1", "u2", "u4", "u8", "f4", "f8")}


def new_task(**kw) -> dict:
    t = {"type": CALL_CUSTOMER, "request": False, "customer": "", "time": INVALID_TIME,
         "wait_time": [], "key_channel": 0, "has_key": False, "filter": []}
    t.update(kw)
    return t


@dataclass
class Message:
    task: dict = field(default_factory=new_task)
    key: np.ndarray | None = None
    value: list = field(default_factory=list)
    sender: str = ""
    recver: str = ""
    original_recver: str = ""
    replied: bool = False
    finished: bool = True
    valid: bool = True
    terminate: bool = False
    wait: bool = False
    recv_handle: Callable[[], Any] | None = None
    fin_handle: Callable[[], Any] | None = None

    # ------------------------------------------------------------- payload
    def set_key(self, key):
        self.key = np.ascontiguousarray(key)
        self.task["has_key"] = True
        self.task["key_type"] = self.key.dtype.str

    def clear_key(self):
        self.key = None
        self.task["has_key"] = False

    def add_value(self, v):
        v = np.ascontiguousarray(v)
        self.value.append(v)
        self.task.setdefault("value_type", []).append(v.dtype.str)

    def clear_value(self):
        self.value = []
        self.task["value_type"] = []

    def has_key(self) -> bool:
        return self.key is not None and self.key.size > 0

    def add_filter(self, ftype: str, **conf) -> dict:
        f = {"type": ftype, **conf}
        self.task.setdefault("filter", []).append(f)
        return f

    def find_filter(self, ftype: str) -> dict | None:
        for f in self.task.get("filter", []):
            if f["type"] == ftype:
                return f
        return None

    def copy_header(self) -> "Message":
        return Message(task=copy.deepcopy(self.task), sender=self.sender, recver=self.recver,
                       original_recver=self.original_recver)

    # --------------------------------------------------------- wire format
    def encode(self) -> list:
        t = dict(self.task)
        t["has_key"] = self.key is not None
        if self.key is not None:
            t["key_type"] = self.key.dtype.str
        t["value_type"] = [v.dtype.str for v in self.value]
        frames = [msgpack.packb(t, use_bin_type=True)]
        if self.key is not None:
            frames.append(self.key)
        frames.extend(self.value)
        return frames

    @staticmethod
    def decode(sender: str, frames: list) -> "Message":
        task = msgpack.unpackb(frames[0], raw=False, strict_map_key=False)
        m = Message(task=task, sender=sender)
        i = 1
        if task.get("has_key"):
            m.key = np.frombuffer(frames[1], dtype=np.dtype(task["key_type"])).copy()
            i = 2
        for dt, f in zip(task.get("value_type", []), frames[i:]):
            m.value.append(np.frombuffer(f, dtype=np.dtype(dt)).copy())
        return m

    def short(self) -> str:
        t = self.task
        kind = {1: "TERMINATE", 3: "REPLY", 4: "MANAGE", 5: "CALL", 6: "HEARTBEAT"}.get(t["type"], "?")
        return (f"{self.sender}=>{self.recver} {kind} req={t['request']} cust={t['customer']} "
                f"t={t['time']} wait={t.get('wait_time')} key={0 if self.key is None else self.key.size} "
                f"vals={[v.size for v in self.value]}")


def slice_key_ordered(msg: Message, key_ranges: list[tuple[int, int]]) -> list[Message]:
    """Split a message with a sorted key array into one piece per key range
    (reference sliceKeyOrderedMsg, src/system/message.h:120-159). Every piece keeps
    the message's own ``key_range`` (receivers align buffers to it); a piece is
    invalid (answered locally instead of sent) iff the receiver's range does not
    intersect the message range. Values carry k entries per key."""
    out = []
    key = msg.key
    mlo, mhi = msg.task.get("key_range", [0, KEY_MAX])
    ukey = None if key is None else key.astype(np.uint64, copy=False)
    for lo, hi in key_ranges:
        m = msg.copy_header()
        m.fin_handle, m.recv_handle, m.wait = msg.fin_handle, msg.recv_handle, msg.wait
        m.valid = max(lo, mlo) < min(hi, mhi)
        if ukey is None:
            m.value = list(msg.value)
            out.append(m)
            continue
        plo, phi = min(max(lo, mlo), mhi), min(max(hi, mlo), mhi)  # Range::project
        a = int(np.searchsorted(ukey, np.uint64(plo), side="left"))
        b = int(np.searchsorted(ukey, np.uint64(phi), side="left")) \
            if phi < KEY_MAX else ukey.size
        b = max(a, b)
        m.key = key[a:b]
        m.task["has_key"] = True
        n = key.size
        m.value = [v[a * (v.size // n):b * (v.size // n)] if n else v[0:0] for v in msg.value]
        out.append(m)
    return out
