"""Minimal push/pull demo (reference src/app/hello_world/main.cc).

Servers hold a KVVector "w" with keys 0..5 and values .0 .. .5; each worker pulls
its own key subset from the server group, waits, and prints it:

    python -m parameter_server_amd.launch local 3 2 -- python -m parameter_server_amd.app.hello_world
"""
from __future__ import annotations

import sys

import numpy as np

from .. import ps
from ..parameter.kv import KVVector
from ..system.customer import App
from ..system.message import SERVER_GROUP, Message


class HelloServer(App):
    def init(self):
        print(f"{self.my_node_id()}, this is server {self.my_rank()}", file=sys.stderr, flush=True)
        self.model = KVVector("w")
        self.model.set_key(0, np.arange(6, dtype=np.uint64))
        self.model.set_val(0, np.arange(6, dtype=np.float32) / 10)


def worker_main(argv):
    print(f"{ps.my_node_id()}: this is worker {ps.my_rank()}", file=sys.stderr, flush=True)
    model = KVVector("w")
    keys = [0, 2, 4, 5] if ps.my_rank() == 0 else [0, 1, 3, 4]
    model.set_key(0, np.array(keys, dtype=np.uint64))
    msg = Message()
    msg.recver = SERVER_GROUP
    msg.set_key(model.key(0))
    t = model.pull(msg)
    model.wait_out_msg(SERVER_GROUP, t)
    k, v = model.key(0), model.value(0)
    print(f"{ps.my_node_id()}: key: [{k.size}]: {' '.join(map(str, k.tolist()))} ; value: "
          f"[{v.size}]: {' '.join(f'{x:g}' for x in v.tolist())}", flush=True)
    return 0


def create_server(conf):
    return HelloServer()


if __name__ == "__main__":
    sys.exit(ps.run(worker_main, create_server))
