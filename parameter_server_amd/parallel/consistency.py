"""Bounded-delay consistency: BSP (tau=0), SSP (finite tau), ASP (tau=inf).

Reference: Darlin submits block t+1 with ``wait_time = t - tau`` and the
per-customer Executor only admits a task whose dependencies are finished
(src/app/linear_method/darlin.h:81-93, src/system/executor.cc:172-177); the
async-SGD ``max_delay`` flag is declared but never read (linear.proto:47).

On the GPU data plane there are no per-message dependencies to check: every
step is one collective exchange, so the schedule itself is the vector clock.
``ExchangeSchedule`` fixes which step's pushes ride which exchange and which
ring buffers a step uses: the pushes of step t ride exchange t+1+lag and the
owner applies them before it resolves that exchange's pulls (or, ssp, they ride
exchange t+lag and are applied right after its pulls), so a pull of step
t has seen exactly the pushes of steps <= t-1-lag of EVERY worker (the
collective cannot start before all ranks have packed those gradients: the
vector clock min_w clock[w] >= t-1-lag holds by construction). ASP decouples the
owner's push apply from the pulls (its own stream, no event the pulls wait on);
``EventClock`` holds the per-exchange HIP events of those applies, which gate
only buffer reuse (``apply_gate``).

``VectorClock`` is the host-side admissibility clock of the KVWorker/KVServer
API (parameter/sharded_kv.py): a pull with timestamp t may be served once every
worker's pushes through t-1-tau are applied.
"""
from __future__ import annotations

import math
import threading

INF = float("inf")


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


class ExchangeSchedule:
    """Step -> exchange / buffer bookkeeping of the padded multi-GPU exchange.

    ``lag``: the pull of step t sees exactly the pushes of steps <= t-1-lag (bsp 0,
    ssp:tau tau unless a smaller ``lag`` is asked for, asp 1: at least). ``depth``
    (asp only): exchanges whose push applies may still be running when a later
    exchange resolves its pulls. Buffers live in rings of ``R = max(2, lag + 1 +
    depth)`` entries indexed by step.

    Where the owner applies the pushes an exchange carries:
    * pre (bsp, asp): exchange t carries the pushes of step t-1-lag and applies them
      BEFORE resolving its pulls (asp: asynchronously beside them);
    * post (ssp with lag >= 1, the default there): exchange t carries the pushes of
      step t-lag and applies them AFTER its pulls are resolved and the weights have
      gone back, so the worker never waits for an apply; the next exchange resolves
      after it. The pull of step t still sees exactly the pushes of steps <= t-1-lag
      (applied by exchanges <= t-1), one step of staleness fewer to carry.
    """

    def __init__(self, tau: float, lag: int = -1, asp_depth: int = 4, post: bool = True):
        self.tau = float(tau)
        self.asp = math.isinf(self.tau)
        if self.asp:
            self.lag = int(lag) if lag >= 0 else 1
            self.depth = max(1, int(asp_depth))
        else:
            self.lag = int(lag) if lag >= 0 else int(self.tau)
            self.depth = 0
            if self.lag > self.tau:
                raise ValueError(f"exchange_lag {self.lag} exceeds the staleness bound {self.tau}")
        if self.lag < 0:
            raise ValueError("exchange lag must be >= 0")
        self.R = max(2, self.lag + 1 + self.depth)
        self.post = bool(post) and not self.asp and self.lag >= 1

    def ring(self, t: int) -> int:
        """Ring entry of step t's pull (resolved slots, weights, offsets) and of the
        gradients step t computes."""
        return t % self.R

    def carried(self, t: int) -> int:
        """Step whose pushes ride exchange t (negative: none yet)."""
        return t - self.lag if self.post else t - 1 - self.lag

    def grad_ring(self, t: int) -> int:
        """Ring entry holding the gradients exchange t carries (its send buffer)."""
        return self.carried(t) % self.R

    def visible_through(self, t: int) -> int:
        """Every push of steps <= this is applied before the pull of step t (bsp/ssp);
        asp: a lower bound only."""
        return t - 1 - self.lag - self.depth

    def apply_gate(self, t: int) -> int | None:
        """asp: exchange whose (asynchronous) push apply must have finished before
        exchange t starts (it frees the slot ring entry exchange t overwrites)."""
        if not self.asp:
            return None
        g = t - self.depth
        return g if g >= 0 else None

    def pending(self, exchanged: int, computed: int) -> range:
        """Steps computed whose gradients no issued exchange has carried yet."""
        return range(max(0, self.carried(exchanged)), computed)

    def staleness_bounds(self) -> tuple[int, float]:
        """(min, max) steps of pushes a pull may miss."""
        return self.lag, (self.lag + self.depth if self.asp else self.lag)


class MergedSchedule:
    """One collective per step (padded exchange, lag >= 1): exchange s carries, per peer
    row, ``[keys(s+1) | grads(s-d) | weights answering keys(s)]`` -- the keys of the NEXT
    step, the pushes of step s-d, and the weights the owner resolved for the keys it
    received in exchange s-1. After exchange s lands:

    * the worker of step s unpacks its weights straight from the received rows;
    * the owner resolves keys(s+1) (weights into the send rows of exchange s+1);
    * the owner applies grads(s-d): ``post`` = after that resolve (off the path to the
      next collective), ``pre`` = before it.

    The pull of step u is resolved right after exchange u-1, so it sees the pushes
    carried by exchanges <= u-2 (post) / <= u-1 (pre), i.e. exactly the pushes of steps
    <= u-1-lag with lag = d+1 (post) or d (pre) -- the same bound as ExchangeSchedule
    with half the collectives. The worker of step u-d must have packed its gradients
    before exchange u is issued, so d >= 2 lets the exchange chain run while the worker
    computes (d = 1 serialises them; kept for lag 1 / tests). Target lag: ssp tau ->
    tau; asp -> 3 (an admissible asp schedule: staleness exactly 3).

    Rings (send, recv, resolved slots) have R = d + 2 entries indexed by exchange / pull
    step: the send row of exchange s is complete once worker s-d and the resolve after
    exchange s-1 wrote it; the received rows of exchange s are read by worker s, the
    resolve of s+1 and the apply of s-d; resolved slots of pull step u are read by the
    apply in exchange u+d."""

    def __init__(self, tau: float, lag: int = -1):
        self.tau = float(tau)
        self.asp = math.isinf(self.tau)
        L = int(lag) if lag >= 0 else (3 if self.asp else int(self.tau))
        if not self.asp and L > self.tau:
            raise ValueError(f"exchange_lag {L} exceeds the staleness bound {self.tau}")
        if L < 1:
            raise ValueError("the merged exchange needs lag >= 1 (bsp: two collectives)")
        self.lag = L
        self.post = L >= 3
        self.d = L - 1 if self.post else L
        self.R = self.d + 2
        self.depth = 0

    def ring(self, i: int) -> int:
        return i % self.R

    def grads_in(self, s: int) -> int:
        """Step whose gradients exchange s carries (negative: none)."""
        return s - self.d

    def grad_ring(self, u: int) -> int:
        """Send ring entry that worker u packs its gradients into (exchange u + d)."""
        return (u + self.d) % self.R

    def visible_through(self, u: int) -> int:
        return u - 1 - self.lag

    def staleness_bounds(self) -> tuple[int, float]:
        return self.lag, self.lag


class EventClock:
    """Per-exchange HIP events of applied pushes (device-side vector clock)."""

    def __init__(self, size: int = 64):
        self.size = int(size)
        self.events = {}

    def record(self, step: int, stream=None):
        import torch

        ev = self.events.get(step % self.size)
        if ev is None:
            ev = torch.cuda.Event()
            self.events[step % self.size] = ev
        ev.record(stream)
        return ev

    def wait_for(self, step: int | None, stream=None):
        """Make ``stream`` wait for the apply of exchange ``step`` (no-op if None or
        never recorded)."""
        if step is None:
            return
        ev = self.events.get(step % self.size)
        if ev is not None:
            import torch

            (stream or torch.cuda.current_stream()).wait_event(ev)


class VectorClock:
    """Host-side vector clock: clock[w] = last step whose push from worker w is applied."""

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
        """Can a pull for timestamp ``step`` be served now?"""
        return self.tau == INF or self.min_clock() >= step - 1 - self.tau

    def wait(self, step: int, timeout: float | None = None) -> bool:
        with self._cv:
            return self._cv.wait_for(lambda: self.admissible(step), timeout=timeout)

    def staleness(self, step: int) -> int:
        """How many steps of pushes a pull at ``step`` may miss right now."""
        return max(0, step - 1 - self.min_clock())
