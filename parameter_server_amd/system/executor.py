"""Per-customer task DAG engine and remote-node handles.

Reference: ``Executor`` (src/system/executor.cc:148-277) keeps received messages
and processes the first one whose ``wait_time`` dependencies are finished in the
sender's incoming TaskTracker; requests are processed by the customer and
auto-replied, replies run ``recv_handle`` and, once every member of the original
group replied, ``fin_handle``. ``RNode::submit`` (src/system/remote_node.cc:57-129)
picks the logical timestamp (explicit, or ++time over the group), records
pending messages and handlers, encodes filters and queues one message per
group member. Node groups: src/system/executor.h:8-18.
"""
from __future__ import annotations

import threading
import traceback

from ..ops.native import core as core_mod
from .message import (COMP_GROUP, GROUPS, INVALID_TIME, KEY_MAX, LIVE_GROUP, REPLY, SERVER_GROUP,
                      WORKER_GROUP, Message, new_task)


class RNode:
    def __init__(self, ex: "Executor", node_id: str, is_group: bool = False, node=None):
        self.ex = ex
        self.id = node_id
        self.is_group = is_group
        self.node = node
        C = core_mod()
        self.incoming = C.TaskTracker()
        self.outgoing = C.TaskTracker()
        self.time = INVALID_TIME
        self.mu = threading.RLock()
        self.pending = {}
        self.recv_handles = {}
        self.fin_handles = {}
        self.filters = {}

    def key_range(self):
        if self.node is None:
            return (0, KEY_MAX)
        return (self.node.key_begin, self.node.key_end)

    # ----------------------------------------------------------- submit
    def submit(self, msgs) -> int:
        if isinstance(msgs, Message):
            msgs = [msgs]
        members = self.ex.group(self.id)
        if len(msgs) == 1 and len(members) > 1:
            # one logical message to a group: slice by key ranges via the customer
            msgs = self.ex.customer.slice(msgs[0], [m.key_range() for m in members])
        if len(msgs) != len(members):
            raise ValueError(f"{len(msgs)} messages for group {self.id} of {len(members)}")
        t = INVALID_TIME
        for m in msgs:
            mt = m.task.get("time", INVALID_TIME)
            if mt is not None and mt > INVALID_TIME:
                if t != INVALID_TIME and t != mt:
                    raise ValueError("all messages of one submit must share the timestamp")
                t = mt
        with self.mu:
            if t > INVALID_TIME:
                self.time = max(t, self.time)
            else:
                for w in members:
                    self.time = max(self.time, w.time)
                self.time += 1
                t = self.time
            if msgs[0].fin_handle is not None:
                self.fin_handles[t] = msgs[0].fin_handle
        me = self.ex.my_id
        for m in msgs:
            m.task["request"] = True
            m.task["customer"] = self.ex.customer.name
            m.task["time"] = t
            m.original_recver = self.id
            m.sender = me
        self.outgoing.start(t)
        for w, m in zip(members, msgs):
            with w.mu:
                m.recver = w.id
                w.time = max(t, w.time)
                w.pending[t] = m
                if m.recv_handle is not None:
                    w.recv_handles[t] = m.recv_handle
            w.outgoing.start(t)
            w.encode_filter(m)
            self.ex.po.queue(m)
        for w, m in zip(members, msgs):
            if m.wait:
                w.outgoing.wait(t)
        return t

    def submit_and_wait(self, msgs) -> int:
        if isinstance(msgs, Message):
            msgs = [msgs]
        for m in msgs:
            m.wait = True
        t = self.submit(msgs)
        self.wait_outgoing(t)
        return t

    def submit_tasks(self, tasks, wait=False, recv_handle=None) -> int:
        msgs = [Message(task=new_task(**t) if isinstance(t, dict) else t) for t in tasks]
        for m in msgs:
            m.wait = wait
            m.recv_handle = recv_handle
        return self.submit(msgs)

    # ------------------------------------------------------------ waits
    def wait_outgoing(self, t, timeout=-1.0):
        for w in self.ex.group(self.id):
            if not w.outgoing.wait(t, timeout):
                return False
        return True

    def try_wait_outgoing(self, t) -> bool:
        return all(w.outgoing.has_finished(t) for w in self.ex.group(self.id))

    def wait_incoming(self, t, timeout=-1.0):
        for w in self.ex.group(self.id):
            if not w.incoming.wait(t, timeout):
                return False
        return True

    def try_wait_incoming(self, t) -> bool:
        return all(w.incoming.has_finished(t) for w in self.ex.group(self.id))

    def finish_incoming(self, t):
        for w in self.ex.group(self.id):
            w.incoming.finish(t)
        self.ex.notify()

    def finish_outgoing(self, t):
        for w in self.ex.group(self.id):
            w.outgoing.finish(t)

    # ---------------------------------------------------------- filters
    def _filter(self, ftype):
        from ..filter import create_filter

        if ftype not in self.filters:
            self.filters[ftype] = create_filter(ftype)
        return self.filters[ftype]

    def encode_filter(self, msg: Message):
        if self.ex.po.message_compression and msg.valid and not msg.find_filter("COMPRESSING"):
            msg.add_filter("COMPRESSING")
        for f in list(msg.task.get("filter", [])):
            self._filter(f["type"]).encode(msg)

    def decode_filter(self, msg: Message):
        for f in reversed(list(msg.task.get("filter", []))):
            self._filter(f["type"]).decode(msg)


class Executor:
    def __init__(self, customer, po):
        self.customer = customer
        self.po = po
        self.my_id = po.my_node.id
        self.nodes: dict[str, RNode] = {}
        self.groups: dict[str, list[RNode]] = {g: [] for g in GROUPS}
        self.group_nodes = {g: RNode(self, g, is_group=True) for g in GROUPS}
        self._msgs: list[Message] = []
        self._cv = threading.Condition()
        self._done = False
        self.active = None
        self.error = None
        for n in po.yp.nodes.values():
            self.add_node(n)
        self._thread = threading.Thread(target=self.run, name=f"exec-{customer.name}",
                                        daemon=True)
        self._thread.start()

    # -------------------------------------------------------------- nodes
    def add_node(self, node):
        if node.id in self.nodes:
            self.nodes[node.id].node = node
            return
        r = RNode(self, node.id, node=node)
        self.nodes[node.id] = r
        role = node.role
        if role == "SERVER":
            self._join(SERVER_GROUP, r)
            self._join(COMP_GROUP, r)
        elif role == "WORKER":
            self._join(WORKER_GROUP, r)
            self._join(COMP_GROUP, r)
        self._join(LIVE_GROUP, r)

    def _join(self, g, r):
        lst = self.groups[g]
        lst.append(r)
        lst.sort(key=lambda x: (x.key_range()[0], x.id))

    def rnode(self, node_id: str) -> RNode | None:
        if node_id in self.group_nodes:
            return self.group_nodes[node_id]
        return self.nodes.get(node_id)

    def group(self, node_id: str) -> list[RNode]:
        if node_id in self.groups:
            return self.groups[node_id]
        r = self.nodes.get(node_id)
        if r is None:
            raise KeyError(f"unknown node {node_id}")
        return [r]

    # ---------------------------------------------------------- messages
    def accept(self, msg: Message):
        r = self.nodes.get(msg.sender)
        if r is not None:
            r.decode_filter(msg)
        with self._cv:
            self._msgs.append(msg)
            self._cv.notify_all()

    def notify(self):
        with self._cv:
            self._cv.notify_all()

    def stop(self):
        with self._cv:
            self._done = True
            self._cv.notify_all()
        if threading.current_thread() is not self._thread:
            self._thread.join(timeout=5)

    def _pick(self):
        for i, m in enumerate(self._msgs):
            sender = self.nodes.get(m.sender)
            if sender is None:
                self._msgs.pop(i)  # unknown sender: drop (reference executor.cc:160-166)
                return None
            if not m.task.get("request"):
                return self._msgs.pop(i)
            ok = all(wt <= INVALID_TIME or sender.incoming.has_finished(wt)
                     for wt in m.task.get("wait_time", []))
            if ok:
                return self._msgs.pop(i)
        return None

    def run(self):
        while True:
            with self._cv:
                msg = None
                while not self._done:
                    msg = self._pick()
                    if msg is not None:
                        break
                    self._cv.wait(timeout=0.5)
                if self._done:
                    return
            try:
                self._process(msg)
            except Exception as e:  # surface errors to the node's main thread
                self.error = e
                traceback.print_exc()
                self.po.fail(e)

    def _process(self, msg: Message):
        self.active = msg
        req = msg.task.get("request", False)
        t = msg.task.get("time", INVALID_TIME)
        sender = self.nodes[msg.sender]
        if req:
            sender.incoming.start(t)
        if msg.task["type"] != REPLY:
            self.customer.process(msg)
        if req:
            if msg.finished:
                sender.incoming.finish(t)
                self.notify()
                if not msg.replied:
                    self.po.reply(msg)
            return
        with sender.mu:
            h = sender.recv_handles.pop(t, None)
        if h:
            h()
        sender.outgoing.finish(t)
        with sender.mu:
            orig = sender.pending.pop(t, None)
        o = self.rnode(orig.original_recver) if orig is not None else sender
        if o is not None and o.try_wait_outgoing(t):
            o.outgoing.finish(t)
            with o.mu:
                fh = o.fin_handles.pop(t, None)
            if fh:
                fh()

    def last_reply(self) -> Message:
        return self.active
