"""User-facing node API (reference src/ps.h, src/ps_main.cc).

A parameter-server program defines ``worker_main(argv)`` and optionally
``create_server(conf)``; ``run()`` starts the node from the command line flags
(``-my_node``, ``-scheduler``, ``-num_servers``, ``-num_workers`` ...), runs the
worker main on workers, and shuts the node down.

    from parameter_server_amd import ps
    ps.run(worker_main, create_server)

Helpers: ``my_app``, ``my_node``, ``my_node_id``, ``is_worker/is_server/is_scheduler``,
``my_rank``, ``rank_size``.

For GPU jobs (one process per GPU, RCCL data plane) use
``parameter.sharded_kv.KVWorker`` (push / pull / wait of k values per key with
BSP / SSP / ASP; demo ``app/hello_world_gpu.py``) or the trainers in ``models``
(``SparseLRTrainer``, ``DarlinTrainer``, ``WideDeepTrainer``, ``FMTrainer``); see README.
"""
from __future__ import annotations

import sys

from .system.customer import App
from .system.postoffice import (Node, Postoffice, is_scheduler, is_server, is_worker, my_node,
                                rank_size)
from .utils.flags import Flags, parse_flags

__all__ = ["run", "start_node", "my_app", "my_node", "my_node_id", "is_worker", "is_server",
           "is_scheduler", "my_rank", "rank_size", "Node", "App"]


def my_app():
    return Postoffice.instance().app


def my_node_id() -> str:
    return my_node().id


def my_rank() -> int:
    return my_node().rank


class _WorkerApp(App):
    def __init__(self, main, argv, name="app"):
        super().__init__(name)
        self.main, self.argv = main, argv
        self.ret = 0

    def run(self):
        self.ret = self.main(self.argv) or 0


def assemble_my_node(flags: Flags, scheduler: Node) -> Node:
    """Role, id, IP and port from ``-my_rank`` (reference Van::assembleMyNode,
    src/system/van.cc:235-272): rank 0 is the scheduler, ranks 1..W the workers
    W0.., then the servers S0..; IP of ``-interface`` (or the first non-loopback
    interface) and a free port. Used by MPI launches (scripts/mpi_node.sh)."""
    from .ops.native import core

    r, W, S = flags.my_rank, flags.num_workers, flags.num_servers
    if r == 0:
        return scheduler
    if r <= W:
        role, nid = "WORKER", f"W{r - 1}"
    elif r <= W + S:
        role, nid = "SERVER", f"S{r - W - 1}"
    else:
        role, nid = "UNUSED", f"U{r - W - S - 1}"
    ip = core().interface_ip(flags.interface) or "127.0.0.1"
    return Node(role, nid, hostname=ip, port=core().free_port())


def start_node(flags: Flags, app_factory=None) -> Postoffice:
    if not flags.scheduler or not (flags.my_node or flags.my_rank >= 0):
        raise SystemExit("need -scheduler and -my_node (or -my_rank); see scripts/local.sh")
    sch = Node.parse(flags.scheduler)
    me = Node.parse(flags.my_node) if flags.my_node else assemble_my_node(flags, sch)
    conf = ""
    if flags.app_file:
        with open(flags.app_file) as f:
            conf = f.read() + "\n"
    conf += flags.app_conf
    po = Postoffice.instance()
    po.start(me, sch, num_servers=flags.num_servers, num_workers=flags.num_workers,
             app_conf=conf, app_factory=app_factory,
             message_compression=flags.message_compression, verbose=flags.verbose,
             print_van=flags.print_van, heartbeat_interval=flags.heartbeat_interval,
             timeout=flags.timeout)
    return po


def run(worker_main, create_server=None, argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    flags = parse_flags(argv)
    holder = {}

    def factory(conf_text):
        role = Postoffice.instance().my_node.role
        if role == "SERVER" and create_server is not None:
            return create_server(conf_text)
        if role == "WORKER":
            holder["app"] = _WorkerApp(worker_main, flags.rest)
            return holder["app"]
        return App()

    po = start_node(flags, factory)
    po.run(timeout=flags.timeout)
    if flags.traffic_statistics:
        print(f"[{po.my_node.id}] traffic {po.van.stats()}", file=sys.stderr)
    return holder["app"].ret if "app" in holder else 0
