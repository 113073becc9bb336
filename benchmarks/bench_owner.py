"""Owner side of the multi-GPU exchange in isolation: kv_resolve_rows (lookup-or-insert of
the pulled keys of G source rows, their weights into the next send rows, partition
bounds) and kv_apply_part (the pushes of G rows, one optimizer step per source row, at
the slots the resolve recorded), timed with HIP events over back-to-back launches.

    python benchmarks/bench_owner.py --G 8 --keys 29000 --lgp 8 9 10 11

Rows: G sorted lists of 34-bit mixed keys (the flat layout's row shape at 8 peers for a
65,536 x 39 Criteo minibatch: ~234 k distinct keys over 8 owners); ``--dup`` = fraction
of each row drawn from a shared hot pool (a real N-GPU owner sees the hot keys in every
row; the 1-GPU loopback emulation sees none)."""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_rows(G, n, C, dup, dev, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    gh = torch.Generator(device=dev).manual_seed(12345)  # the hot pool: the same in every set
    H = (4 + 2 * C + C + C + 3) // 4 * 4
    recv = torch.zeros(G * H, dtype=torch.int32, device=dev)
    hot = torch.randint(0, 1 << 34, (max(1, int(n * dup)),), device=dev, generator=gh)
    for s in range(G):
        nh = int(n * dup)
        cold = torch.randint(0, 1 << 34, (n - nh,), device=dev, generator=g)
        k = torch.unique(torch.cat([hot[:nh], cold]))  # sorted, distinct
        m = k.numel()
        row = recv[s * H:(s + 1) * H]
        row[0] = m
        row[1] = m
        row[4:4 + 2 * m] = k.view(torch.int32)
        row[4 + 2 * C:4 + 2 * C + m] = torch.randn(m, device=dev, generator=g).view(torch.int32)
    return recv, H


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--G", type=int, default=8)
    ap.add_argument("--keys", type=int, default=29000, help="keys per source row")
    ap.add_argument("--dup", type=float, default=0.0)
    ap.add_argument("--lgp", type=int, nargs="+", default=[8, 9, 10, 11])
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--capacity", type=float, nargs="+", default=[2 ** 27])
    ap.add_argument("--fresh", type=int, default=0,
                    help="> 0: cycle through this many row sets, each resolved for the first "
                         "time (inserts), timing resolve and apply launch by launch")
    a = ap.parse_args()
    from parameter_server_amd.ops.kv_table import KVTable, UpdateRule
    from parameter_server_amd.ops.native import hipops

    dev = torch.device("cuda")
    G, n = a.G, a.keys
    C = (int(n * 1.2) + 63) // 64 * 64
    sets = [make_rows(G, n, C, a.dup, dev, seed=i) for i in range(max(1, a.fresh))]
    H = sets[0][1]
    rule = UpdateRule(algo="ftrl", alpha=0.1, beta=1.0, l1=1.0, l2=0.1)
    hh = hipops()
    slot = torch.full((G * C,), -1, dtype=torch.int64, device=dev)
    keys = torch.zeros(G * C, dtype=torch.int64, device=dev)
    wout = torch.zeros(G * H, dtype=torch.float32, device=dev)
    stats = torch.zeros(64 * 16, dtype=torch.float64, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(a.iters):
            fn()
        ev[1].record()
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / a.iters * 1e3

    for cap in a.capacity:
        for lgP in a.lgp:  # (a fresh table each: the fresh row sets insert)
            tb = KVTable(int(cap), dev, key_range=(0, 1 << 34))
            it, iv, isd, seed = tb.init.args()
            P = 1 << lgP
            bnd = torch.zeros(G * (P + 1), dtype=torch.int32, device=dev)

            def resolve(recv, bounds=True):
                hh.kv_resolve_rows(tb.slots, recv, H, C, 2, slot, wout, True, it, iv, isd, seed,
                                   tb._err, None, tb.home_base, tb.home_m,
                                   keys if bounds else None, bnd if bounds else None,
                                   lgP if bounds else 0, wstride=H)

            def apply(recv, st):
                gsrc = recv.view(torch.float32)[4 + 2 * C:]
                hh.kv_apply_part(tb.slots, slot, keys, gsrc, H, recv, H, C, bnd, lgP,
                                 *rule.args(), st)

            out = {"bench": "owner", "G": G, "keys_per_row": n, "dup": a.dup, "C": C,
                   "capacity": int(cap), "table_gb": round(cap * 32 / 2 ** 30, 1), "lgP": lgP}
            if a.fresh:  # every resolve inserts its row set's keys
                evs = [torch.cuda.Event(enable_timing=True) for _ in range(3 * a.fresh)]
                torch.cuda.synchronize()
                for i, (recv, _) in enumerate(sets):
                    evs[3 * i].record()
                    resolve(recv)
                    evs[3 * i + 1].record()
                    apply(recv, stats)
                    evs[3 * i + 2].record()
                torch.cuda.synchronize()
                k = a.fresh - 1
                out["fresh_resolve_us"] = round(sum(evs[3 * i].elapsed_time(evs[3 * i + 1])
                                                    for i in range(1, a.fresh)) / k * 1e3, 2)
                out["fresh_apply_part_us"] = round(sum(evs[3 * i + 1].elapsed_time(evs[3 * i + 2])
                                                       for i in range(1, a.fresh)) / k * 1e3, 2)
            recv = sets[0][0]
            out["resolve_us"] = round(timed(lambda: resolve(recv)), 2)
            out["resolve_no_bounds_us"] = round(timed(lambda: resolve(recv, False)), 2)
            resolve(recv)
            out["apply_part_us"] = round(timed(lambda: apply(recv, stats)), 2)
            out["apply_part_no_stats_us"] = round(timed(lambda: apply(recv, None)), 2)
            print(json.dumps(out), flush=True)
            del tb
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
