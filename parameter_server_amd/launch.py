"""Single-host launchers.

``local S W -- <program> [args]``: one scheduler + S servers + W workers on
127.0.0.1 (reference script/local.sh: H@8001, S_i@9600+i, W_i@9500+i; here free
ports are picked unless --base-port is given). Returns the first non-zero exit code.

``gpu N -- <program> [args]``: one process per GPU via torch.distributed.run
(RCCL data plane), master on 127.0.0.1.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def local(num_servers: int, num_workers: int, cmd: list[str], base_port: int = 0,
          timeout: float = 600.0, env=None) -> int:
    ports = ([base_port + i for i in range(1 + num_servers + num_workers)] if base_port
             else [_free_port() for _ in range(1 + num_servers + num_workers)])
    sch = f"role:SCHEDULER,hostname:'127.0.0.1',port:{ports[0]},id:'H'"
    common = ["-num_servers", str(num_servers), "-num_workers", str(num_workers),
              "-scheduler", sch]
    specs = [sch]
    specs += [f"role:SERVER,hostname:'127.0.0.1',port:{ports[1 + i]},id:'S{i}'"
              for i in range(num_servers)]
    specs += [f"role:WORKER,hostname:'127.0.0.1',port:{ports[1 + num_servers + i]},id:'W{i}'"
              for i in range(num_workers)]
    e = dict(os.environ if env is None else env)
    e.setdefault("OMP_NUM_THREADS", "1")
    procs = [subprocess.Popen(cmd + ["-my_node", s] + common, env=e) for s in specs]
    rc = 0
    try:
        for p in procs:
            r = p.wait(timeout=timeout)
            rc = rc or r
    except subprocess.TimeoutExpired:
        rc = 124
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return rc


def gpu(n: int, cmd: list[str]) -> int:
    port = _free_port()
    full = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", "--master-port", str(port)] + cmd
    return subprocess.call(full)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if "--" not in argv:
        raise SystemExit("usage: launch {local S W | gpu N} [--base-port P] -- program args")
    i = argv.index("--")
    head, cmd = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["local", "gpu"])
    ap.add_argument("counts", nargs="+", type=int)
    ap.add_argument("--base-port", type=int, default=0)
    ap.add_argument("--timeout", type=float, default=600.0)
    a = ap.parse_args(head)
    if a.mode == "local":
        return local(a.counts[0], a.counts[1], cmd, a.base_port, a.timeout)
    return gpu(a.counts[0], cmd)


if __name__ == "__main__":
    sys.exit(main())
