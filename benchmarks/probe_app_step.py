#!/usr/bin/env python3
"""Probe: the cost of one eager ``SparseLRTrainer.step`` as the file-fed app issues it
(one HBM-resident minibatch, no pipelining): wall per step with and without a device sync
per step, and a cProfile of the host side. Prints one JSON line + the profile top 25."""
import cProfile
import io
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer
    from parameter_server_amd.ops.synthetic import criteo_batch

    dev = torch.device("cuda", 0)
    B = int(os.environ.get("PROBE_B", "65536"))
    cfg = SparseLRConfig(num_features=10 ** 8, minibatch=B, table_capacity=1 << 27,
                         lr_type="decay", alpha=0.01, beta=10, l1=10, l2=1)
    tr = SparseLRTrainer(cfg, device=dev)
    keys = torch.empty(B * 39, dtype=torch.int64, device=dev)
    labels = torch.empty(B, dtype=torch.float32, device=dev)
    dist = os.environ.get("PROBE_DIST", "criteo")
    if dist == "criteo":  # bench.py's generator
        criteo_batch(B, seed=1, row0=0, num_features=cfg.num_features, device=dev, keys=keys,
                     labels=labels)
    else:  # "pow<e>": bench_app.py's files, id = N * U^e (e = 4: ~30 % of occurrences < 10^6)
        g = torch.Generator(device=dev)
        g.manual_seed(1)
        e = float(dist[3:] or 4)
        u = torch.rand(B, 39, device=dev, generator=g, dtype=torch.float64)
        keys.copy_((cfg.num_features * u ** e).long().sort(dim=1).values.reshape(-1))
        labels.copy_((torch.rand(B, device=dev, generator=g) < 0.3).float() * 2 - 1)
    for _ in range(5):
        tr.step(keys, labels, width=39)
    torch.cuda.synchronize()
    n = 50
    t0 = time.perf_counter()
    for _ in range(n):
        tr.step(keys, labels, width=39)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    for _ in range(n):
        tr.step(keys, labels, width=39)
        torch.cuda.synchronize()
    t3 = time.perf_counter()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        tr.step(keys, labels, width=39)
    pr.disable()
    torch.cuda.synchronize()
    print(json.dumps({"probe": "app_step", "B": B, "dist": dist, "localize": tr.localize_mode,
                      "host_issue_ms": (t1 - t0) / n * 1e3, "wall_ms": (t2 - t0) / n * 1e3,
                      "synced_ms": (t3 - t2) / n * 1e3}), flush=True)
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(25)
    print(s.getvalue(), flush=True)


if __name__ == "__main__":
    main()
