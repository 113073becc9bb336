"""Distributed key/value objects over the runtime (CPU plumbing mode).

Reference ``SharedParameter<K>`` (src/parameter/shared_parameter.h:12-162):
``push/pull(msg)`` set ``CallSharedPara.cmd`` and submit to the receiver (a node or
group); ``process`` dispatches push-request / pull-reply -> ``set_value``,
pull-request -> reply with ``get_value``; it also implements the tail-filter
protocol (``insert_count`` -> CountMin insert, ``query_key`` -> return only the
keys whose count > freq, ``query_value`` -> with their values).
"""
from __future__ import annotations

import math

import numpy as np

from ..ops.countmin import CountMinSketch
from ..system.customer import KeyOrderedCustomer
from ..system.message import CALL_CUSTOMER, KEY_MAX, Message, slice_key_ordered

OPS = {
    "PLUS": np.add, "MINUS": np.subtract, "TIMES": np.multiply, "DIVIDE": np.divide,
    "AND": np.bitwise_and, "OR": np.bitwise_or, "XOR": np.bitwise_xor,
}


def comp_ass_op(op: str, dst: np.ndarray, src: np.ndarray):
    """dst op= src (reference compAssOp, shared_parameter.h:173-193)."""
    OPS[op](dst, src, out=dst)


class FrequencyFilter:
    """CountMin-backed key frequency filter (src/parameter/frequency_filter.h:9-45)."""

    def __init__(self, n: int = 0, k: int = 2):
        self.cm = CountMinSketch(n, k) if n else None

    def empty(self):
        return self.cm is None

    def resize(self, n, k):
        self.cm = CountMinSketch(int(n), int(k))

    def clear(self):
        if self.cm is not None:
            self.cm.clear()

    def insert_keys(self, keys: np.ndarray, counts: np.ndarray):
        import torch

        self.cm.insert(torch.from_numpy(keys.astype(np.int64, copy=False).copy()),
                       torch.from_numpy(np.minimum(counts, 255).astype(np.uint8)))

    def query_keys(self, keys: np.ndarray, freq: int) -> np.ndarray:
        import torch

        keep, _ = self.cm.query(torch.from_numpy(keys.astype(np.int64, copy=False).copy()), freq)
        return keys[keep.numpy().astype(bool)]


class SharedParameter(KeyOrderedCustomer):
    def __init__(self, name: str, parent: str | None = None, po=None):
        super().__init__(name, parent, po)
        self.key_filter: dict[int, FrequencyFilter] = {}
        self.key_filter_ignore_chl = True

    # ------------------------------------------------------------ API
    def sync(self, msg: Message) -> int:
        msg.task["type"] = CALL_CUSTOMER
        msg.task.setdefault("key_range", [0, KEY_MAX])
        return self.port(msg.recver).submit(msg)

    def push(self, msg: Message) -> int:
        msg.task.setdefault("shared_para", {})["cmd"] = "PUSH"
        return self.sync(msg)

    def pull(self, msg: Message) -> int:
        msg.task.setdefault("shared_para", {})["cmd"] = "PULL"
        return self.sync(msg)

    def wait_in_msg(self, node: str, t: int):
        self.port(node).wait_incoming(t)

    def wait_out_msg(self, node: str, t: int):
        self.port(node).wait_outgoing(t)

    def finish(self, node: str, t: int):
        self.port(node).finish_incoming(t)

    def set_tail_filter_size(self, chl: int, n: int, k: int):
        self.key_filter.setdefault(chl, FrequencyFilter()).resize(n, k)

    def clear_tail_filter(self, chl: int):
        self.key_filter.pop(chl, None)

    def my_key_range(self):
        n = self.po.my_node
        return (n.key_begin, n.key_end)

    # ---------------------------------------------------- override points
    def get_value(self, msg: Message):
        raise NotImplementedError

    def set_value(self, msg: Message):
        raise NotImplementedError

    def slice(self, msg, key_ranges):
        if msg.task.get("shared_para", {}).get("replica"):
            return super(KeyOrderedCustomer, self).slice(msg, key_ranges)
        return slice_key_ordered(msg, key_ranges)

    # ------------------------------------------------------------ process
    def process(self, msg: Message):
        req = msg.task.get("request", False)
        call = msg.task.get("shared_para", {})
        cmd = call.get("cmd")
        push, pull = cmd == "PUSH", cmd == "PULL"
        reply = None
        if pull and req:
            reply = Message(task=dict(msg.task), key=msg.key)
            reply.task["request"] = False
            reply.task["value_type"] = []
            reply.task["filter"] = [dict(f) for f in msg.task.get("filter", [])
                                    if f["type"] != "COMPRESSING"]
        tf = call.get("tail_filter")
        if tf is not None:
            chl = 0 if self.key_filter_ignore_chl else msg.task.get("key_channel", 0)
            if tf.get("insert_count") and req and msg.key is not None and msg.key.size:
                f = self.key_filter.setdefault(chl, FrequencyFilter())
                if f.empty():
                    w = max(1.0, float(self.po.yp.num_workers))
                    f.resize(max(64, int(w * tf.get("countmin_n", 1 << 20) / math.log(w + 1))),
                             tf.get("countmin_k", 2))
                f.insert_keys(msg.key, msg.value[0])
            if "query_key" in tf and pull:
                if req:
                    f = self.key_filter.get(chl)
                    keys = msg.key if f is None or f.empty() else f.query_keys(msg.key, tf["query_key"])
                    reply.key, reply.value = keys, []
                    if tf.get("query_value"):
                        self.get_value(reply)
                else:
                    self.set_value(msg)
        else:
            if (push and req) or (pull and not req):
                self.set_value(msg)
            elif pull and req:
                self.get_value(reply)
        if pull and req:
            self.po.reply(msg, reply)
