"""Bounded-delay consistency: BSP (tau=0), SSP (finite tau), ASP (tau=inf).

Reference: Darlin submits block t+1 with ``wait_time = t - tau`` and the
per-customer Executor only admits a task whose dependencies are finished
(src/app/linear_method/darlin.h:81-93, src/system/executor.cc:172-177); the
async-SGD ``max_delay`` flag is declared but never read (linear.proto:47).
Here one vector clock per shard records, for every worker, the last step whose
push has been applied; a pull for step c may be served only when
min_w clock[w] >= c - 1 - tau. GPU pipelines record a HIP event per applied
push so a stream can wait on exactly the step it depends on.
"""
from __future__ import annotations

import threading

INF = float("inf")


class VectorClock:
    def __init__(self, num_workers: int, tau: float = 0):
        self.clock = [-1] * num_workers
        self.tau = tau
        self._cv = threading.Condition()

    def tick(self, worker: int, step: int):
        with self._cv:
            if step > self.clock[worker]:
                self.clock[worker] = step
            self._cv.notify_all()

    def min_clock(self) -> int:
        return min(self.clock)

    def admissible(self, step: int) -> bool:
        """Can a pull for minibatch ``step`` be served now?"""
        return self.tau == INF or self.min_clock() >= step - 1 - self.tau

    def wait(self, step: int, timeout: float | None = None) -> bool:
        with self._cv:
            return self._cv.wait_for(lambda: self.admissible(step), timeout=timeout)

    def staleness(self, step: int) -> int:
        """How many of this worker's predecessors' pushes the pull may miss."""
        return max(0, step - 1 - self.min_clock())


def parse_consistency(mode: str | int | float) -> float:
    """'bsp' -> 0, 'asp' -> inf, 'ssp:4' / 4 -> 4."""
    if isinstance(mode, (int, float)):
        return float(mode)
    m = str(mode).lower()
    if m == "bsp":
        return 0.0
    if m == "asp":
        return INF
    if m.startswith("ssp"):
        return float(m.split(":")[1]) if ":" in m else 4.0
    return float(m)


class EventClock:
    """Per-step HIP events of applied pushes (device-side vector clock)."""

    def __init__(self):
        self.events = {}

    def record(self, step: int, stream=None):
        import torch

        ev = torch.cuda.Event()
        ev.record(stream)
        self.events[step] = ev
        for s in [s for s in self.events if s < step - 64]:
            del self.events[s]

    def wait_for(self, step: int, stream=None):
        ev = self.events.get(step)
        if ev is not None:
            import torch

            (stream or torch.cuda.current_stream()).wait_event(ev)
