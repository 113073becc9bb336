"""Process-wide node runtime: transport, registry, bootstrap and app lifecycle.

Reference: ``Postoffice`` (src/system/postoffice.cc:45-347) parses flags, owns
the Van and YellowPages, runs the send/recv threads and the bootstrap protocol
CONNECT -> app ADD -> node ADD (ranks + key ranges) -> INIT -> RUN -> DONE ->
TERMINATE; ``queue()`` answers invalid (empty) slices locally instead of sending.
``Postmaster`` (src/system/postmaster.cc) partitions data files over workers and
the key space over servers and assigns per-role ranks.

Same protocol here, over the C++ ``Van``; every node runs one receive thread and
sends from the calling thread (the Van serialises per-peer writes).
"""
from __future__ import annotations

import os
import re
import sys
import threading
import time
from dataclasses import asdict, dataclass

from ..ops.native import core
from .message import (CALL_CUSTOMER, HEARTBEATING, MANAGE, REPLY, TERMINATE, Message,
                      new_task)

from .message import KEY_MAX  # noqa: E402


@dataclass
class Node:
    role: str            # SCHEDULER | SERVER | WORKER
    id: str
    hostname: str = "127.0.0.1"
    port: int = 0
    rank: int = -1
    key_begin: int = 0
    key_end: int = KEY_MAX

    @staticmethod
    def parse(spec: str) -> "Node":
        """Reference node text proto: ``role:SERVER,hostname:'127.0.0.1',port:9600,id:'S0'``."""
        kv = {}
        for part in re.split(r"[,\s]+", spec.strip().strip("{}")):
            if not part:
                continue
            k, v = part.split(":", 1)
            kv[k.strip()] = v.strip().strip("'\"")
        return Node(role=kv.get("role", "WORKER").upper(), id=kv.get("id", ""),
                    hostname=kv.get("hostname", "127.0.0.1"), port=int(kv.get("port", 0)))


class YellowPages:
    """Registry of nodes and customers (src/system/yellow_pages.cc)."""

    def __init__(self):
        self.nodes: dict[str, Node] = {}
        self.customers = {}

    def num(self, role):
        return sum(1 for n in self.nodes.values() if n.role == role)

    @property
    def num_servers(self):
        return self.num("SERVER")

    @property
    def num_workers(self):
        return self.num("WORKER")


def partition_key_space(servers: list[Node], begin=0, end=KEY_MAX):
    """Server s owns evenDivide(s) of [begin, end) (postmaster.cc:17-31)."""
    n = len(servers)
    for i, s in enumerate(sorted(servers, key=lambda x: x.id)):
        s.key_begin = begin + (end - begin) * i // n
        s.key_end = begin + (end - begin) * (i + 1) // n
        s.rank = i


def assign_ranks(nodes: list[Node]):
    for role in ("WORKER", "SCHEDULER"):
        for i, n in enumerate(sorted((x for x in nodes if x.role == role), key=lambda x: x.id)):
            n.rank = i


class Postoffice:
    _inst = None

    @classmethod
    def instance(cls) -> "Postoffice":
        if cls._inst is None:
            cls._inst = Postoffice()
        return cls._inst

    @classmethod
    def reset(cls):
        cls._inst = None

    def __init__(self):
        self.yp = YellowPages()
        self.van = None
        self.my_node: Node | None = None
        self.scheduler: Node | None = None
        self.app = None
        self.message_compression = False
        self.verbose = False
        self.print_van = None
        self._mng_cv = threading.Condition()
        self._mng_replies = {}
        self._connect_cv = threading.Condition()
        self._stopped = threading.Event()
        self._error = None
        self._recv_thread = None
        self._app_conf = ""
        self._lifecycle = {}
        self._manage_time = 0
        self.hb = None
        self._terminated = False

    # ----------------------------------------------------------- start
    def start(self, my_node: Node, scheduler: Node, *, num_servers: int = 0, num_workers: int = 0,
              app_conf: str = "", app_factory=None, message_compression=False, verbose=False,
              print_van=False, heartbeat_interval: float = 0.0, timeout: float = 300.0):
        self.my_node, self.scheduler = my_node, scheduler
        self.message_compression = message_compression
        self.verbose = verbose
        self.app_factory = app_factory
        self.van = core().Van(my_node.id)
        import atexit

        atexit.register(self.stop)  # never leave transport threads running at exit
        bind_host = "*"
        my_node.port = self.van.bind(bind_host, my_node.port)
        if print_van:
            self.print_van = open(f"van_{my_node.id}", "w")
        self.yp.nodes[my_node.id] = my_node
        self._recv_thread = threading.Thread(target=self._recv_loop, name="po-recv", daemon=True)
        self._recv_thread.start()
        if heartbeat_interval > 0:
            from .heartbeat import HeartbeatReporter

            self.hb = HeartbeatReporter(self, heartbeat_interval)
        if my_node.role == "SCHEDULER":
            self._app_conf = app_conf
            self.n_expected = (num_servers, num_workers)
            self._wait_for(lambda: self.yp.num_servers >= num_servers and
                           self.yp.num_workers >= num_workers, timeout, "nodes to CONNECT")
            nodes = list(self.yp.nodes.values())
            partition_key_space([n for n in nodes if n.role == "SERVER"])
            assign_ranks(nodes)
            my_node.rank = 0
            for n in nodes:
                if n.id != my_node.id:
                    self.van.connect(n.id, n.hostname, n.port)
            self.app = self._create_app(app_conf)
            t = self._manage_all("ADD", nodes=[asdict(n) for n in nodes], conf=app_conf)
            self._wait_replies(t, timeout)
        else:
            self.van.connect(scheduler.id, scheduler.hostname, scheduler.port)
            self.yp.nodes[scheduler.id] = scheduler
            m = Message(task=new_task(type=MANAGE, request=True,
                                      mng={"cmd": "CONNECT", "node": asdict(my_node)}))
            m.recver = scheduler.id
            self._send(m)
            self._wait_for(lambda: self.app is not None, timeout, "app ADD from scheduler")
        return self

    def _create_app(self, conf: str):
        from .customer import App

        factory = self.app_factory or App.create
        return factory(conf)

    def run(self, timeout: float = 3600.0):
        """Scheduler drives INIT/RUN; other nodes block until TERMINATE."""
        if self.my_node.role == "SCHEDULER":
            try:
                t = self._manage_all("INIT")
                self.app.init()
                self._wait_replies(t, timeout)
                t = self._manage_all("RUN")
                self.app.run()
                self._wait_replies(t, timeout)
            finally:
                self.stop()  # TERMINATE every node, also when the job failed
        else:
            while not self._stopped.wait(0.2):
                if self._error:
                    raise self._error
        if self._error:
            raise self._error

    def stop(self):
        if self.my_node and self.my_node.role == "SCHEDULER" and not self._terminated:
            self._terminated = True
            for n in list(self.yp.nodes.values()):
                if n.id != self.my_node.id:
                    m = Message(task=new_task(type=TERMINATE))
                    m.recver = n.id
                    try:
                        self._send(m)
                    except Exception:
                        pass
            time.sleep(0.05)
        self._stopped.set()
        if self.hb:
            self.hb.stop()
        for c in list(self.yp.customers.values()):
            c.executor.stop()
        if self._recv_thread is not None and threading.current_thread() is not self._recv_thread:
            self._recv_thread.join(timeout=5)
        if self.van:
            self.van.stop()

    def fail(self, e):
        self._error = e
        self._stopped.set()

    # -------------------------------------------------------- messaging
    def queue(self, msg: Message):
        """Send, or answer an empty slice locally (postoffice.cc:192-207)."""
        if not msg.valid:
            rep = Message(task=new_task(type=REPLY, request=False, customer=msg.task["customer"],
                                        time=msg.task["time"]))
            rep.sender = msg.recver
            rep.recver = self.my_node.id
            self._deliver(rep)
            return
        self._send(msg)

    def _send(self, msg: Message):
        msg.sender = self.my_node.id
        if msg.recver == self.my_node.id:
            frames = [f if isinstance(f, bytes) else f.tobytes() for f in msg.encode()]
            loop = Message.decode(self.my_node.id, frames)
            loop.recver = self.my_node.id
            self._deliver(loop)
            return
        if self.print_van:
            self.print_van.write(f"|>>> {msg.short()}\n")
            self.print_van.flush()
        self.van.send(msg.recver, msg.encode())

    def reply(self, req: Message, rep: Message | None = None):
        """Answer a request. With no payload this is the empty REPLY ack (reference
        Postoffice::reply); a data reply (e.g. a pull answer) keeps CALL_CUSTOMER so the
        requester's customer processes it (shared_parameter.h:105-109)."""
        if rep is None:
            rep = Message(task=new_task(type=REPLY))
        rep.task.update({"request": False, "customer": req.task.get("customer", ""),
                         "time": req.task.get("time", -1), "key_channel": req.task.get("key_channel", 0)})
        rep.recver = req.sender
        req.replied = True
        self._send(rep)

    def _recv_loop(self):
        while not self._stopped.is_set():
            got = self.van.recv(0.2)
            if got is None:
                continue
            sender, frames = got
            try:
                msg = Message.decode(sender, frames)
                msg.recver = self.my_node.id
                if self.print_van:
                    self.print_van.write(f"|<<< {msg.short()}\n")
                    self.print_van.flush()
                self._deliver(msg)
            except Exception as e:  # pragma: no cover
                import traceback

                traceback.print_exc()
                self.fail(e)

    def _deliver(self, msg: Message):
        typ = msg.task["type"]
        if typ == TERMINATE:
            self._stopped.set()
            return
        if typ == MANAGE:
            threading.Thread(target=self._manage, args=(msg,), daemon=True).start()
            return
        if typ == HEARTBEATING:
            if self.hb:
                self.hb.on_report(msg)
            return
        if typ == REPLY and msg.task.get("customer") == "__manage__":
            with self._mng_cv:
                self._mng_replies.setdefault(msg.task["time"], set()).add(msg.sender)
                self._mng_cv.notify_all()
            return
        name = msg.task.get("customer", "")
        c = self._wait_customer(name)
        if c is None:
            print(f"[{self.my_node.id}] no customer {name!r}; drop {msg.short()}", file=sys.stderr)
            return
        c.executor.accept(msg)

    def _wait_customer(self, name, timeout=30.0):
        deadline = time.time() + timeout
        while time.time() < deadline:
            c = self.yp.customers.get(name)
            if c is not None:
                return c
            time.sleep(0.005)
        return None

    # ------------------------------------------------------- management
    def _manage_all(self, cmd, **kw) -> int:
        self._manage_time += 1
        t = self._manage_time
        for n in list(self.yp.nodes.values()):
            if n.id == self.my_node.id:
                continue
            m = Message(task=new_task(type=MANAGE, request=True, customer="__manage__", time=t,
                                      mng={"cmd": cmd, **kw}))
            m.recver = n.id
            self._send(m)
        return t

    def _wait_replies(self, t, timeout):
        others = {n.id for n in self.yp.nodes.values() if n.id != self.my_node.id}
        self._wait_for(lambda: self._mng_replies.get(t, set()) >= others, timeout,
                       f"manage replies t={t}", cv=self._mng_cv)

    def _wait_for(self, pred, timeout, what, cv=None):
        cv = cv or self._connect_cv
        deadline = time.time() + timeout
        with cv:
            while not pred():
                if self._error:
                    raise self._error
                left = deadline - time.time()
                if left <= 0:
                    raise TimeoutError(f"[{self.my_node.id}] timed out waiting for {what}")
                cv.wait(min(left, 0.2))

    def _manage(self, msg: Message):
        mng = msg.task["mng"]
        cmd = mng["cmd"]
        try:
            if cmd == "CONNECT":  # scheduler side
                n = Node(**mng["node"])
                with self._connect_cv:
                    self.yp.nodes[n.id] = n
                    self._connect_cv.notify_all()
                return
            if cmd == "ADD":
                for d in mng["nodes"]:
                    n = Node(**d)
                    self.yp.nodes[n.id] = n
                    if n.id == self.my_node.id:
                        self.my_node.rank, self.my_node.key_begin, self.my_node.key_end = \
                            n.rank, n.key_begin, n.key_end
                for n in self.yp.nodes.values():
                    if n.id != self.my_node.id:
                        self.van.connect(n.id, n.hostname, n.port)
                for c in list(self.yp.customers.values()):
                    for n in self.yp.nodes.values():
                        c.executor.add_node(n)
                app = self._create_app(mng.get("conf", ""))
                with self._connect_cv:
                    self.app = app
                    self._connect_cv.notify_all()
            elif cmd == "INIT":
                self.app.init()
            elif cmd == "RUN":
                self.app.run()
            rep = Message(task=new_task(type=REPLY, customer="__manage__", time=msg.task["time"]))
            rep.recver = msg.sender
            self._send(rep)
        except Exception as e:
            import traceback

            traceback.print_exc()
            self.fail(e)


# ----------------------------------------------------------------- helpers
def my_node() -> Node:
    return Postoffice.instance().my_node


def is_scheduler() -> bool:
    return my_node().role == "SCHEDULER"


def is_server() -> bool:
    return my_node().role == "SERVER"


def is_worker() -> bool:
    return my_node().role == "WORKER"


def rank_size() -> int:
    yp = Postoffice.instance().yp
    return yp.num_workers if is_worker() else (yp.num_servers if is_server() else 1)
