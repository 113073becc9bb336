"""Fault-injection app for the failure detector (no reference counterpart: the
reference has no fault injection and hangs when a peer dies).

Every worker "works" for ``-work`` seconds; worker ``-kill_rank`` instead dies
abruptly (``os._exit``) after ``-die_after`` seconds. With ``-heartbeat_interval``
set, the scheduler notices the missing heartbeats, fails the job and TERMINATEs
the survivors instead of waiting for the RUN replies forever.

    python -m parameter_server_amd.launch local 1 3 -- python -m \\
        parameter_server_amd.app.fault_injection -heartbeat_interval 0.2 -kill_rank 1
"""
from __future__ import annotations

import os
import sys
import time

from .. import ps


def _arg(argv, name, default):
    if name in argv:
        return type(default)(argv[argv.index(name) + 1])
    return default


def worker_main(argv):
    work = _arg(argv, "-work", 30.0)
    kill = _arg(argv, "-kill_rank", -1)
    die_after = _arg(argv, "-die_after", 0.5)
    t0 = time.time()
    if ps.my_rank() == kill:
        time.sleep(die_after)
        print(f"{ps.my_node_id()}: injected crash", file=sys.stderr, flush=True)
        os._exit(17)
    while time.time() - t0 < work:
        time.sleep(0.05)
    return 0


if __name__ == "__main__":
    sys.exit(ps.run(worker_main))
