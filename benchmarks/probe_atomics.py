#!/usr/bin/env python3
"""Throughput of global fp32 atomics on MI355X (torch index_add_ = atomicAdd per
element): N adds into U addresses, uniformly random vs hot-skewed indices."""
import torch

def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3

for N, U in ((796_000, 234_000), (2_560_000, 234_000), (234_000, 234_000), (796_000, 4_000_000)):
    idx = torch.randint(0, U, (N,), device="cuda")
    v = torch.rand(N, device="cuda")
    g = torch.zeros(U, device="cuda")
    us = t(lambda: g.index_add_(0, idx, v))
    cp = t(lambda: g.index_copy_(0, idx[:U] if N >= U else idx, v[:U] if N >= U else v))
    print(f"N={N} U={U}: index_add {us:.1f} us  ({N / us:.0f} atomics/us); index_copy {cp:.1f} us", flush=True)
