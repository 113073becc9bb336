"""Variable-width, valued minibatches (rcv1-like: ~75 features per row, tf-idf values)
through the 1-GPU trainer: the flat layout with the CSR fused forward + tile backward
(``tp_fwd_bwd_csr``) against the compact layout with the generic kernels (PSAMD_FLAT=0).

    python benchmarks/bench_csr.py --minibatch 1000 10000 --steps 200

A pool of 8 minibatches is generated on the device first and cycled (the timed step is
localisation + pull + forward/backward + push/update; no parsing, no host copies -- the
file-fed path is app/gpu.py). Prints one JSON line per (B, path)."""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def csr_pool(B, count, N, device, seed=0, kind="rcv1"):
    """Minibatches of variable-width rows:
    rcv1:   5..145 features per row (~75) drawn Zipf(1.0) over 47,236 ids (the rcv1
            vocabulary), tf-idf-like values;
    ctr:    Criteo-shaped rows (criteo_batch: 13 + 26 slots, power-law ids hashed into N)
            with each feature present with probability 0.75 (missing slots), binary;
    unique: 5..145 features per row over N ids, u^4-skewed but nearly all distinct (the
            stress case of the localiser: per-bucket hashes near capacity)."""
    from parameter_server_amd.ops.synthetic import criteo_batch

    out = []
    g = torch.Generator(device=device).manual_seed(seed)
    zipf = None
    if kind == "rcv1":
        zipf = 1.0 / torch.arange(1, 47237, dtype=torch.float32, device=device)
    for c in range(count):
        if kind == "ctr":
            k39, labels = criteo_batch(B, seed=seed + 1, row0=c * B, num_features=N, device=device)
            keep = torch.rand(B * 39, device=device, generator=g) < 0.75
            w = keep.view(B, 39).sum(1)
            keys = k39[keep]
            vals = None
        else:
            w = torch.randint(5, 145, (B,), device=device, generator=g)
            n = int(w.sum())
            if kind == "rcv1":
                keys = torch.multinomial(zipf, n, replacement=True, generator=g)
            else:
                u = torch.rand(n, device=device, generator=g, dtype=torch.float64)
                keys = (N * u ** 4).long().clamp(max=N - 1)
            vals = torch.rand(n, device=device, generator=g) * 0.9 + 0.1
            labels = torch.where(torch.rand(B, device=device, generator=g) < 0.35, 1.0, -1.0)
        row_ptr = torch.zeros(B + 1, dtype=torch.int64, device=device)
        row_ptr[1:] = torch.cumsum(w, 0)
        out.append((keys, labels, row_ptr, vals))
    return out


def run(B, flat, steps, warmup, N, device, kind):
    os.environ["PSAMD_FLAT"] = "1" if flat else "0"
    from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer

    if kind == "rcv1":
        N = 47236
    pool = csr_pool(B, 8, N, device, kind=kind)
    maxn = max(int(p[2][-1]) for p in pool)
    cfg = SparseLRConfig(num_features=N, minibatch=B, max_nnz_per_example=(maxn + B - 1) // B,
                         table_capacity=1 << 24)
    tr = SparseLRTrainer(cfg, device=device)
    for i in range(warmup):
        k, lab, rp, v = pool[i % 8]
        tr.step(k, lab, row_ptr=rp, vals=v)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        k, lab, rp, v = pool[i % 8]
        tr.step(k, lab, row_ptr=rp, vals=v)
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    p = tr.progress()
    tr.check_ok()
    nnz = sum(int(q[2][-1]) for q in pool) / len(pool)
    distinct = sum(int(torch.unique(q[0]).numel()) for q in pool) / len(pool)
    return {"bench": "csr_rows", "kind": kind, "minibatch": B, "nnz_per_row": round(nnz / B, 1),
            "distinct_keys": int(distinct), "valued": pool[0][3] is not None,
            "path": "flat+csr fused" if flat else "compact+generic",
            "localize": tr.localize_mode, "ms_per_step": dt / steps * 1e3,
            "host_issue_ms_per_step": t_issue / steps * 1e3,
            "examples_per_s": B * steps / dt, "loss": p["loss"], "auc": p["auc"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--minibatch", type=int, nargs="+", default=[1000, 10000])
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--num-features", type=float, default=1e8)
    ap.add_argument("--kind", nargs="+", default=["rcv1", "ctr", "unique"])
    a = ap.parse_args()
    dev = torch.device("cuda")
    for kind in a.kind:
        for B in a.minibatch:
            for flat in (True, False):
                print(json.dumps(run(B, flat, a.steps, a.warmup, int(a.num_features), dev, kind)),
                      flush=True)


if __name__ == "__main__":
    main()
