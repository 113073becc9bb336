#!/usr/bin/env python3
"""Owner-side push apply of G source rows, standalone (no concurrent streams):
chained-hash pair (kv_update_rows: fill + link + apply) vs the key-range
partitioned one-launch kernel (kv_apply_part) at several partition counts.

    python benchmarks/bench_owner_apply.py --peers 8 --cap 45120 --fill 29000
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, default=8)
    ap.add_argument("--cap", type=int, default=45120, help="C: keys per row capacity")
    ap.add_argument("--fill", type=int, default=29000, help="keys per row")
    ap.add_argument("--shared", type=float, default=0.3, help="fraction of keys from a hot pool")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--lgp", default="8,9,10,11,12")
    args = ap.parse_args()
    from parameter_server_amd.ops.kv_table import KVTable, UpdateRule, next_pow2
    from parameter_server_amd.ops.native import hipops

    dev = torch.device("cuda")
    G, C, n = args.peers, args.cap, args.fill
    lo, span = 1 << 28, 1 << 28  # this owner's mixed-key range
    g = torch.Generator().manual_seed(0)
    hot = torch.randint(0, span, (n,), generator=g)
    H = (4 + C + C + 3) // 4 * 4
    recv = torch.zeros(G * H, dtype=torch.int32)
    for s in range(G):
        nh = int(n * args.shared)
        k = torch.cat([hot[torch.randperm(n, generator=g)[:nh]],
                       torch.randint(0, span, (n - nh,), generator=g)])
        k = torch.unique(k)[:n] + lo
        row = recv[s * H:(s + 1) * H]
        row[0] = row[1] = k.numel()
        row[4:4 + k.numel()] = k.to(torch.int32)
        row[4 + C:4 + C + k.numel()] = torch.randn(k.numel(), generator=g).view(torch.int32)
    recv = recv.to(dev)
    tb = KVTable(1 << 24, dev, key_range=(lo, lo + span))
    rule = UpdateRule(algo="ftrl", alpha=0.1, beta=1.0, l1=1.0, l2=0.1)
    hh = hipops()
    slot = torch.full((G * C,), -1, dtype=torch.int64, device=dev)
    w = torch.zeros(G * C, dtype=torch.float32, device=dev)
    keys = torch.zeros(G * C, dtype=torch.int64, device=dev)
    gsrc = recv.view(torch.float32)[4 + C:]
    from parameter_server_amd.ops.linear import new_accum
    stats = new_accum(dev)  # striped, as the trainer's
    it, iv, isd, seed = tb.init.args()

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3 / args.reps

    out = {"peers": G, "cap": C, "fill": n, "entries": G * n}
    link = torch.empty(next_pow2(2 * G * C), dtype=torch.int64, device=dev)
    nxt = torch.empty(G * C, dtype=torch.int32, device=dev)
    hh.kv_resolve_rows(tb.slots, recv, H, C, 1, slot, w, True, it, iv, isd, seed, tb._err, None,
                       tb.home_base, tb.home_m)
    out["resolve_rows_us"] = timed(lambda: hh.kv_resolve_rows(
        tb.slots, recv, H, C, 1, slot, w, True, it, iv, isd, seed, tb._err, None, tb.home_base,
        tb.home_m))
    out["link_us"] = timed(lambda: hh.kv_update_rows(tb.slots, slot, gsrc, H, recv, H, C, link,
                                                     nxt, *rule.args(), stats))
    for lgp in [int(x) for x in args.lgp.split(",")]:
        bnd = torch.zeros(G * ((1 << lgp) + 1), dtype=torch.int32, device=dev)
        out[f"resolve_rows_bnd_lgp{lgp}_us"] = timed(lambda: hh.kv_resolve_rows(
            tb.slots, recv, H, C, 1, slot, w, True, it, iv, isd, seed, tb._err, None,
            tb.home_base, tb.home_m, keys, bnd, lgp))
        out[f"part_lgp{lgp}_us"] = timed(lambda: hh.kv_apply_part(
            tb.slots, slot, keys, gsrc, H, recv, H, C, bnd, lgp, *rule.args(), stats))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
