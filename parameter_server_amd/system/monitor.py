"""Progress monitoring: slaves report to a master on the scheduler.

Reference: ``MonitorSlaver`` submits ``Task{CALL_CUSTOMER, msg = serialized
progress}`` to the scheduler; ``MonitorMaster`` merges per sender and calls a
printer every ``interval`` seconds (src/system/monitor.h:6-77). Customers are
named ``<app>monitor``.
"""
from __future__ import annotations

import threading
import time

import msgpack

from .customer import Customer
from .message import Message, new_task


class MonitorMaster(Customer):
    def __init__(self, app_name: str, merger=None, printer=None, interval: float = 1.0, po=None):
        super().__init__(app_name + "monitor", app_name, po)
        self.merger = merger or (lambda src, dst: dst.update(src) or dst)
        self.printer = printer
        self.interval = interval
        self.progress: dict[str, dict] = {}
        self.mu = threading.Lock()
        self.t0 = time.time()
        self._stop = threading.Event()
        self._thr = None

    def set_merger(self, f):
        self.merger = f

    def set_printer(self, interval, f):
        self.interval, self.printer = interval, f
        if self._thr is None and f is not None:
            self._thr = threading.Thread(target=self._loop, daemon=True, name="monitor-print")
            self._thr.start()

    def _loop(self):
        while not self._stop.wait(self.interval):
            self.flush()

    def flush(self):
        with self.mu:
            if self.progress and self.printer:
                self.printer(time.time() - self.t0, self.progress)

    def process(self, msg: Message):
        prog = msgpack.unpackb(msg.task["msg"], raw=False, strict_map_key=False)
        with self.mu:
            dst = self.progress.setdefault(msg.sender, {})
            self.progress[msg.sender] = self.merger(prog, dst)

    def stop(self):
        self._stop.set()
        super().stop()


class MonitorSlaver(Customer):
    def __init__(self, master_id: str, app_name: str, po=None):
        super().__init__(app_name + "monitor", app_name, po)
        self.master = master_id

    def report(self, prog: dict):
        m = Message(task=new_task(msg=msgpack.packb(prog, use_bin_type=True)))
        m.recver = self.master
        self.port(self.master).submit(m)
