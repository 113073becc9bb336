"""Timers, process/host resource usage and local machine facts.

Reference: src/util/resource_usage.h (tic/toc, ScopedTimer, Timer, MilliTimer,
ResUsage::myVirMem/myPhyMem/hostInUseMem/hostTotalMem read from /proc) and
src/util/local_machine.h (VirMem/PhyMem, IP(interface),
pickupAvailableInterfaceAndIP, pickupAvailablePort). The IP / port helpers are
the host runtime's (csrc/core/runtime.cc ``interface_ip`` / ``free_port``). GPU
facts (device count, HBM per device, CU count, arch) are added because the
MI355X build sizes its tables and shards from them.
"""
from __future__ import annotations

import os
import time


def tic() -> float:
    return time.perf_counter()


def toc(t0: float) -> float:
    """Seconds since ``t0``."""
    return time.perf_counter() - t0


def milli_toc(t0: float) -> float:
    return 1e3 * (time.perf_counter() - t0)


class Timer:
    """Accumulating stopwatch (reference Timer; MilliTimer = ``Timer(milli=True)``)."""

    def __init__(self, milli: bool = False):
        self._scale = 1e3 if milli else 1.0
        self._t = 0.0
        self._tp = tic()

    def start(self):
        self._tp = tic()
        return self

    def reset(self):
        self._t = 0.0

    def restart(self):
        self.reset()
        self.start()

    def stop(self) -> float:
        self._t += toc(self._tp) * self._scale
        return self._t

    def get(self) -> float:
        return self._t

    def get_and_restart(self) -> float:
        t = self._t
        self.restart()
        return t

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()


class ScopedTimer:
    """Adds the scope's duration (seconds) to ``holder[key]`` (reference ScopedTimer
    aggregating into a double*)."""

    def __init__(self, holder: dict, key: str = "time"):
        self.holder, self.key = holder, key

    def __enter__(self):
        self._t0 = tic()
        return self

    def __exit__(self, *exc):
        self.holder[self.key] = self.holder.get(self.key, 0.0) + toc(self._t0)


def _proc_kb(path: str, field: str) -> float:
    try:
        with open(path) as f:
            for line in f:
                if line.startswith(field):
                    return float(line.split()[1])
    except OSError:
        pass
    return -1.0


class ResUsage:
    """Memory in MB, from /proc like the reference; CPU seconds from getrusage."""

    @staticmethod
    def my_vir_mem() -> float:
        return _proc_kb("/proc/self/status", "VmSize:") / 1e3

    @staticmethod
    def my_phy_mem() -> float:
        return _proc_kb("/proc/self/status", "VmRSS:") / 1e3

    @staticmethod
    def host_in_use_mem() -> float:
        g = lambda f: _proc_kb("/proc/meminfo", f)  # noqa: E731
        return (g("MemTotal:") - g("MemFree:") - g("Buffers:") - g("Cached:")) / 1024

    @staticmethod
    def host_total_mem() -> float:
        return _proc_kb("/proc/meminfo", "MemTotal:") / 1024

    @staticmethod
    def my_cpu_seconds() -> float:
        import resource

        r = resource.getrusage(resource.RUSAGE_SELF)
        return r.ru_utime + r.ru_stime


class LocalMachine:
    vir_mem = staticmethod(ResUsage.my_vir_mem)
    phy_mem = staticmethod(ResUsage.my_phy_mem)

    @staticmethod
    def ip(interface: str = "") -> str:
        from ..ops.native import core

        return core().interface_ip(interface)

    @staticmethod
    def pickup_available_interface_and_ip() -> tuple[str, str]:
        """First non-loopback interface with an IPv4 address (reference
        pickupAvailableInterfaceAndIP); ('lo', '127.0.0.1') if none."""
        from ..ops.native import core

        try:
            names = sorted(os.listdir("/sys/class/net"))
        except OSError:
            names = []
        for n in names:
            if n == "lo":
                continue
            ip = core().interface_ip(n)
            if ip:
                return n, ip
        return "lo", "127.0.0.1"

    @staticmethod
    def pickup_available_port() -> int:
        from ..ops.native import core

        return core().free_port()

    @staticmethod
    def num_cpus() -> int:
        try:
            return len(os.sched_getaffinity(0))
        except AttributeError:  # pragma: no cover
            return os.cpu_count() or 1

    @staticmethod
    def gpus() -> list[dict]:
        """One dict per visible GPU: name, arch, CUs, HBM bytes (empty without GPUs)."""
        import torch

        out = []
        if not torch.cuda.is_available():
            return out
        for i in range(torch.cuda.device_count()):
            p = torch.cuda.get_device_properties(i)
            out.append({"index": i, "name": p.name,
                        "arch": getattr(p, "gcnArchName", ""),
                        "compute_units": p.multi_processor_count,
                        "hbm_bytes": p.total_memory})
        return out
