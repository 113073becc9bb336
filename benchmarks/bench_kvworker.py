"""KVWorker push + pull of one key list per step: keyed calls vs a registered key list
(key caching: key-less push rows, request-free pulls). One GPU; ``--peers N`` emulates
the N-rank exchange geometry over a loopback (every row owned locally).

    python benchmarks/bench_kvworker.py --keys 1000000 --dim 16 --peers 8
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from parameter_server_amd.parallel.comm import LoopbackComm  # noqa: E402
from parameter_server_amd.parameter.sharded_kv import KVWorker  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=1 << 20)
    ap.add_argument("--distinct", type=int, default=1 << 22)
    ap.add_argument("--dim", type=int, default=16)
    ap.add_argument("--peers", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda")
    comm = LoopbackComm(args.peers, dev) if args.peers > 1 else None
    kv = KVWorker(comm, dev, capacity=1 << 24, dim=args.dim, key_bits=32,
                  max_keys=args.keys)
    keys = torch.randint(0, args.distinct, (args.keys,), device=dev)
    vals = torch.randn(args.keys, args.dim, device=dev)
    h = kv.register_keys(keys)
    out = {"keys": args.keys, "dim": args.dim, "peers": args.peers}
    for name, k in (("keyed", keys), ("registered", h)):
        for _ in range(3):
            kv.wait(kv.push(k, vals))
            kv.wait(kv.pull(k))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            kv.push(k, vals)
            kv.wait(kv.pull(k))
        torch.cuda.synchronize()
        out[f"{name}_us_per_push_pull"] = (time.perf_counter() - t0) / args.steps * 1e6
    got_h = kv.wait(kv.pull(h))
    got_k = kv.wait(kv.pull(keys))
    out["max_abs_diff_handle_vs_keyed"] = float((got_h - got_k).abs().max())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
