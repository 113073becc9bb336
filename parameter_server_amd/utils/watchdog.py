"""Host-side stall watchdog for the SPMD data plane.

Every rank's host loop calls ``beat(phase, step)``; a daemon thread checks that
the beats keep coming. When none has arrived for ``timeout`` seconds (a peer that
never joins a collective, a hung kernel the host waits on) it prints which rank,
phase, step and last collective it was in, and ends the process with exit code
``EXIT_STALL`` (the launcher then tears the other ranks down), instead of letting
the job sit until an outer lease expires. The collective timeout of the process
group (parallel/comm.py) usually fires first; this is the backstop that also
covers waits outside collectives (``torch.cuda.synchronize`` on a stuck stream).

The reference has no such bound: a node waiting on a dead peer's reply blocks its
Executor thread forever (src/system/executor.cc:160-166) and the heartbeat
monitor that could have noticed is commented out (src/system/postoffice.cc:248-250).

``PSAMD_INJECT_STALL=<rank>:<step>:<seconds>`` makes ``maybe_inject`` sleep on that
rank at that timed step (fault injection for the fail-fast tests).
"""
from __future__ import annotations

import os
import sys
import threading
import time

EXIT_STALL = 3
CURRENT = None  # the process's StallWatch (bench.py reports it on failure)


class StallWatch:
    def __init__(self, rank: int, timeout: float, comm=None, enabled: bool = True):
        self.rank = int(rank)
        self.timeout = float(timeout)
        self.comm = comm
        self.phase, self.step = "start", None
        self.last = time.monotonic()
        self._stop = threading.Event()
        self._t = None
        global CURRENT
        CURRENT = self
        if enabled and self.timeout > 0:
            self._t = threading.Thread(target=self._loop, name="psamd-stallwatch", daemon=True)
            self._t.start()

    def beat(self, phase: str | None = None, step: int | None = None) -> None:
        if phase is not None:
            self.phase = phase
        self.step = step
        self.last = time.monotonic()

    def describe(self) -> str:
        op = getattr(self.comm, "last_op", "none") if self.comm is not None else "none"
        st = "" if self.step is None else f" step {self.step}"
        return f"rank {self.rank}: phase {self.phase}{st}, last collective {op}"

    def _loop(self):
        poll = min(1.0, max(0.05, self.timeout / 10))
        while not self._stop.wait(poll):
            idle = time.monotonic() - self.last
            if idle > self.timeout:
                print(f"[psamd] STALL {self.describe()}: no progress for {idle:.0f} s "
                      f"(timeout {self.timeout:.0f} s); exiting with code {EXIT_STALL}",
                      file=sys.stderr, flush=True)
                os._exit(EXIT_STALL)

    def stop(self):
        self._stop.set()


def default_timeout() -> float:
    """PSAMD_STALL_TIMEOUT, else the collective timeout + 30 s (so the process
    group's own timeout, with its diagnostics, normally fires first)."""
    v = os.environ.get("PSAMD_STALL_TIMEOUT")
    if v:
        return float(v)
    return float(os.environ.get("PSAMD_COMM_TIMEOUT", "180")) + 30.0


def maybe_inject(rank: int, step: int) -> None:
    spec = os.environ.get("PSAMD_INJECT_STALL")
    if not spec:
        return
    r, s, sec = spec.split(":")
    if int(r) == rank and int(s) == step:
        print(f"[psamd] injected stall: rank {rank} sleeps {sec} s at step {step}",
              file=sys.stderr, flush=True)
        time.sleep(float(sec))


def maybe_inject_post(rank: int) -> None:
    """Fault injection after the timed region (tests/test_bench_spawn.py):
    ``PSAMD_INJECT_POST_EXIT=rank:code`` exits that rank with ``code`` right after the
    report; ``PSAMD_INJECT_TEARDOWN_HANG=rank:sec`` sleeps there (a teardown hang)."""
    spec = os.environ.get("PSAMD_INJECT_POST_EXIT")
    if spec:
        r, code = spec.split(":")
        if int(r) == rank:
            print(f"[psamd] injected post-timing exit {code} on rank {rank}", file=sys.stderr,
                  flush=True)
            os._exit(int(code))
    spec = os.environ.get("PSAMD_INJECT_TEARDOWN_HANG")
    if spec:
        r, sec = spec.split(":")
        if int(r) == rank:
            print(f"[psamd] injected teardown hang: rank {rank} sleeps {sec} s", file=sys.stderr,
                  flush=True)
            time.sleep(float(sec))
