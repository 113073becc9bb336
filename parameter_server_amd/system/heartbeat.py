"""Heartbeats, resource dashboard and dead-node detection for the control plane.

Reference: ``HeartbeatInfo`` samples process / host CPU, RSS and NIC bytes from
``/proc`` (src/system/heartbeat_info.{h,cc}); ``Dashboard`` renders one row per
node (src/system/dashboard.{h,cc}); both are compiled but disabled there (call
sites commented out, postoffice.cc:248-250, 355-398) and dead peers are ignored.

Here they are live when ``--heartbeat_interval > 0``: every non-scheduler node
sends a ``HEARTBEATING`` task with a msgpack report to the scheduler, which keeps
a ``Dashboard`` and declares a node dead after ``dead_after`` missed intervals
(SURVEY §5.3 "heartbeat with rank-failure abort"): the scheduler fails the job
(``Postoffice.fail``) so no rank hangs forever, and the run can be restarted from
the last binary snapshot (utils.checkpoint).
"""
from __future__ import annotations

import os
import socket
import sys
import threading
import time

import msgpack

from .message import HEARTBEATING, Message, new_task


def _read(path: str) -> str:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return ""


class HeartbeatInfo:
    """CPU / memory / network / van traffic sampler (heartbeat_info.cc)."""

    def __init__(self, interface: str = "", van=None):
        self.interface = interface or self._default_interface()
        self.hostname = socket.gethostname()
        self.van = van
        self.hz = os.sysconf("SC_CLK_TCK") if hasattr(os, "sysconf") else 100
        self.ncpu = os.cpu_count() or 1
        self.t0 = time.time()
        self._last = self._snapshot()
        self.busy = 0.0
        self._busy_start = None

    @staticmethod
    def _default_interface() -> str:
        for line in _read("/proc/net/dev").splitlines()[2:]:
            name = line.split(":")[0].strip()
            if name and name != "lo":
                return name
        return "lo"

    def _snapshot(self) -> dict:
        s = {"t": time.time(), "pu": 0, "ps": 0, "hu": 0, "hs": 0, "ht": 0, "in": 0, "out": 0}
        st = _read("/proc/self/stat").rsplit(")", 1)
        if len(st) == 2:
            f = st[1].split()
            s["pu"], s["ps"] = int(f[11]), int(f[12])
        cpu = _read("/proc/stat").splitlines()
        if cpu and cpu[0].startswith("cpu "):
            v = [int(x) for x in cpu[0].split()[1:]]
            s["hu"], s["hs"], s["ht"] = v[0] + v[1], v[2], sum(v)
        for line in _read("/proc/net/dev").splitlines()[2:]:
            name, _, rest = line.partition(":")
            if name.strip() == self.interface:
                f = rest.split()
                s["in"], s["out"] = int(f[0]), int(f[8])
        return s

    def start_busy(self):
        self._busy_start = time.time()

    def stop_busy(self):
        if self._busy_start is not None:
            self.busy += time.time() - self._busy_start
            self._busy_start = None

    def get(self) -> dict:
        """One report; rates are over the interval since the previous call."""
        cur = self._snapshot()
        last, self._last = self._last, cur
        dt = max(cur["t"] - last["t"], 1e-6)
        dh = max(cur["ht"] - last["ht"], 1)
        rss = 0
        for line in _read("/proc/self/status").splitlines():
            if line.startswith("VmRSS:"):
                rss = int(line.split()[1]) // 1024
        mem_total = mem_avail = 0
        for line in _read("/proc/meminfo").splitlines():
            if line.startswith("MemTotal:"):
                mem_total = int(line.split()[1]) // 1024
            elif line.startswith("MemAvailable:"):
                mem_avail = int(line.split()[1]) // 1024
        rep = {
            "hostname": self.hostname,
            "seconds": time.time() - self.t0,
            "process_cpu_usage": 100.0 * ((cur["pu"] - last["pu"]) + (cur["ps"] - last["ps"]))
            / self.hz / dt,
            "host_cpu_usage": 100.0 * ((cur["hu"] - last["hu"]) + (cur["hs"] - last["hs"])) / dh,
            "process_rss_mb": rss,
            "host_in_use_mb": mem_total - mem_avail,
            "host_mem_total_mb": mem_total,
            "host_net_in_mb_s": (cur["in"] - last["in"]) / dt / 2 ** 20,
            "host_net_out_mb_s": (cur["out"] - last["out"]) / dt / 2 ** 20,
            "busy_time": self.busy,
        }
        if self.van is not None:
            st = self.van.stats()
            rep["van_sent_mb"] = (st["sent_local"] + st["sent_remote"]) / 2 ** 20
            rep["van_recv_mb"] = (st["recv_local"] + st["recv_remote"]) / 2 ** 20
        return rep


def _node_key(node_id: str):
    """Sort S0 < S2 < S10 (reference NodeIDCmp: alpha prefix, then number)."""
    i = len(node_id)
    while i > 0 and node_id[i - 1].isdigit():
        i -= 1
    return (node_id[:i], int(node_id[i:]) if i < len(node_id) else -1)


class Dashboard:
    COLS = [("Node", None, "{}"), ("MyCPU(%)", "process_cpu_usage", "{:.1f}"),
            ("HostCPU(%)", "host_cpu_usage", "{:.1f}"), ("MyRSS(M)", "process_rss_mb", "{}"),
            ("HostMem(M)", "host_in_use_mb", "{}"), ("In(M/s)", "host_net_in_mb_s", "{:.1f}"),
            ("Out(M/s)", "host_net_out_mb_s", "{:.1f}"), ("VanTx(M)", "van_sent_mb", "{:.1f}"),
            ("VanRx(M)", "van_recv_mb", "{:.1f}"), ("Age(s)", "_age", "{:.1f}")]

    def __init__(self):
        self.data: dict[str, dict] = {}
        self.seen: dict[str, float] = {}
        self.mu = threading.Lock()

    def add_report(self, node: str, rep: dict):
        with self.mu:
            self.data[node] = rep
            self.seen[node] = time.time()

    def render(self) -> str:
        w = 11
        now = time.time()
        lines = ["=" * 20 + " Dashboard " + time.ctime() + " " + "=" * 20,
                 "".join(f"{c[0]:<{w}}" for c in self.COLS)]
        with self.mu:
            for node in sorted(self.data, key=_node_key):
                rep = dict(self.data[node])
                rep["_age"] = now - self.seen[node]
                row = [f"{node:<{w}}"]
                for _, key, fmt in self.COLS[1:]:
                    v = rep.get(key)
                    row.append(f"{(fmt.format(v) if v is not None else '-'):<{w}}")
                lines.append("".join(row))
        return "\n".join(lines)

    def stale(self, max_age: float) -> list[str]:
        now = time.time()
        with self.mu:
            return [n for n, t in self.seen.items() if now - t > max_age]


class HeartbeatReporter:
    """Runs on every node: reporters send, the scheduler collects and watches."""

    def __init__(self, po, interval: float, dead_after: float = 10.0, show: bool = False,
                 abort_on_dead: bool = True):
        self.po = po
        self.interval = float(interval)
        self.dead_after = dead_after
        self.show = show or po.verbose
        self.abort_on_dead = abort_on_dead
        self.info = HeartbeatInfo(van=po.van)
        self.dashboard = Dashboard()
        self.dead: set[str] = set()
        self._stop = threading.Event()
        self._thr = threading.Thread(target=self._loop, name="heartbeat", daemon=True)
        self._thr.start()

    def _loop(self):
        is_sched = self.po.my_node.role == "SCHEDULER"
        failures = 0
        while not self._stop.wait(self.interval):
            try:
                if is_sched:
                    self._watch()
                else:
                    m = Message(task=new_task(type=HEARTBEATING,
                                              msg=msgpack.packb(self.info.get(),
                                                                use_bin_type=True)))
                    m.recver = self.po.scheduler.id
                    self.po._send(m)
                failures = 0
            except Exception as e:  # never let monitoring itself kill the node ...
                if self._stop.is_set():
                    return
                failures += 1
                if failures == 1:
                    print(f"[{self.po.my_node.id}] heartbeat: {e!r}", file=sys.stderr)
                if not is_sched and failures * self.interval >= self.dead_after * self.interval:
                    # ... but a scheduler that stays unreachable means the job is gone
                    self.po.fail(RuntimeError(f"scheduler {self.po.scheduler.id} unreachable"))
                    return

    def _watch(self):
        if self.show:
            print(self.dashboard.render(), file=sys.stderr)
        for node in self.dashboard.stale(self.dead_after * self.interval):
            if node in self.dead:
                continue
            self.dead.add(node)
            msg = f"node {node} missed heartbeats for {self.dead_after * self.interval:.1f}s"
            print(f"[{self.po.my_node.id}] {msg}", file=sys.stderr)
            if self.abort_on_dead:
                self.po.fail(RuntimeError(msg))

    def on_report(self, msg: Message):
        rep = msgpack.unpackb(msg.task["msg"], raw=False, strict_map_key=False)
        self.dashboard.add_report(msg.sender, rep)

    def stop(self):
        self._stop.set()
        if threading.current_thread() is not self._thr:
            self._thr.join(timeout=2)
