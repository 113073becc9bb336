"""Tracing: roctx ranges, phase timers and per-rank traffic counters.

Reference tracing: ``--print_van`` logs every message
(src/system/van.cc:29-32,69-71,108-111), ``--verbose`` logs executor decisions,
``--traffic_statistics`` prints GB sent/received split local vs remote at
TERMINATE (src/system/van.cc:225-233), and ``Timer``/``busy_timer_`` feed
Darlin's time table (src/app/linear_method/darlin.h:350-368).

MI355X equivalent:
* ``trace_range(name)`` — a roctx range (``torch.cuda.nvtx`` is roctx on ROCm,
  so the ranges show up in ``rocprofv3 --marker-trace`` next to the kernels) plus
  a host wall-clock accumulator per phase name;
* ``count_traffic(kind, nbytes)`` — bytes moved per collective kind (all-to-all,
  all-reduce, all-gather), recorded by ``parallel.comm.DistComm`` always (it is
  a few integer adds); the TCP control plane's Van keeps the reference's
  local-vs-remote split itself (``Van.stats``);
* ``dump(path)`` writes one JSON per rank: phases, traffic, and the TCP control
  plane's Van counters when given.

Phase timing and roctx ranges are off unless ``PSAMD_TRACE=1`` (or
``enable(True)``): the hot loop then pays one attribute check per range.
"""
from __future__ import annotations

import json
import os
import threading
import time
from collections import defaultdict
from contextlib import contextmanager, nullcontext

_lock = threading.Lock()
_enabled = os.environ.get("PSAMD_TRACE", "0") == "1"
_phases: dict[str, list] = defaultdict(lambda: [0, 0.0, 0.0])  # count, total s, max s
_traffic: dict[str, list] = defaultdict(lambda: [0, 0, 0])     # calls, bytes sent, bytes recv


def enable(on: bool = True) -> None:
    global _enabled
    _enabled = bool(on)


def enabled() -> bool:
    return _enabled


def _nvtx():
    try:
        import torch

        if torch.cuda.is_available():
            return torch.cuda.nvtx
    except Exception:  # pragma: no cover
        pass
    return None


_NULL = nullcontext()


def trace_range(name: str, sync: bool = False):
    """roctx range + host timer for phase ``name``; a shared no-op context when
    tracing is off. ``sync=True`` synchronises the device at both ends so the host
    time is the GPU time of the phase (use for coarse phases only)."""
    return _trace_range(name, sync) if _enabled else _NULL


@contextmanager
def _trace_range(name: str, sync: bool):
    nv = _nvtx()
    if nv is not None:
        if sync:
            import torch

            torch.cuda.synchronize()
        nv.range_push(name)
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if nv is not None:
            if sync:
                import torch

                torch.cuda.synchronize()
            nv.range_pop()
        dt = time.perf_counter() - t0
        with _lock:
            p = _phases[name]
            p[0] += 1
            p[1] += dt
            p[2] = max(p[2], dt)


def count_traffic(kind: str, sent: int, recv: int = 0) -> None:
    with _lock:
        t = _traffic[kind]
        t[0] += 1
        t[1] += int(sent)
        t[2] += int(recv)


def snapshot(van_stats: dict | None = None) -> dict:
    with _lock:
        out = {
            "phases": {k: {"count": v[0], "total_s": v[1], "max_s": v[2],
                           "mean_ms": 1e3 * v[1] / max(1, v[0])} for k, v in _phases.items()},
            "traffic": {k: {"calls": v[0], "bytes_sent": v[1], "bytes_recv": v[2]}
                        for k, v in _traffic.items()},
        }
    if van_stats is not None:
        out["van"] = dict(van_stats)
    return out


def reset() -> None:
    with _lock:
        _phases.clear()
        _traffic.clear()


def dump(path: str, rank: int | None = None, van_stats: dict | None = None) -> str:
    """Write this rank's snapshot as JSON; ``{rank}`` in ``path`` is substituted."""
    if rank is None:
        rank = int(os.environ.get("RANK", "0"))
    p = path.format(rank=rank)
    d = os.path.dirname(p)
    if d:
        os.makedirs(d, exist_ok=True)
    snap = snapshot(van_stats)
    snap["rank"] = rank
    with open(p, "w") as f:
        json.dump(snap, f, indent=1, sort_keys=True)
    return p


def format_traffic(snap: dict | None = None) -> str:
    """One-line summary like the reference's --traffic_statistics printer."""
    snap = snap or snapshot()
    gb = 1.0 / (1 << 30)
    parts = [f"{k}: {v['calls']} calls, sent {v['bytes_sent'] * gb:.3f} GB, "
             f"recv {v['bytes_recv'] * gb:.3f} GB" for k, v in sorted(snap["traffic"].items())]
    return "; ".join(parts) if parts else "no collective traffic"
