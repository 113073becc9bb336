"""Phase marks of the tile kernel (tploc.hip tp_tile_kernel, shader clock per workgroup):
where a tile's time goes, at the driver's B = 65,536 (8192-key tiles) and B = 10,000
(2048-key tiles).

    python benchmarks/prof_tile_phases.py [--minibatch 65536 10000]

Phases: init (hash / count clears), loads (all 8 keys of every lane landed; a barrier
only in this profiling mode), insert (mix + LDS hash insert + bucket-rank atomics),
scan (bucket offsets, toff / dcnt), place (tile keys out, slots -> entry positions),
rep (every occurrence's entry out)."""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--minibatch", type=int, nargs="+", default=[65536, 10000])
    a = ap.parse_args()
    from parameter_server_amd.ops.localize import Localizer
    from parameter_server_amd.ops.native import hipops
    from parameter_server_amd.ops.synthetic import criteo_batch

    H = hipops()
    for B in a.minibatch:
        keys, _ = criteo_batch(B, seed=3, row0=0, num_features=10 ** 9, device="cuda")
        n = keys.numel()
        lz = Localizer(n, 30, "cuda", mode="tpf")
        T = (n + (1 << H.tpf_tile_log2(n)) - 1) >> H.tpf_tile_log2(n)
        for _ in range(5):
            lz(keys)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            lz(keys)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 50 * 1e3
        prof = torch.zeros(T * 16, dtype=torch.int64, device="cuda")
        H.tp_tile_set_prof(prof)
        lz(keys)
        torch.cuda.synchronize()
        H.tp_tile_set_prof(None)
        p = prof.view(T, 16).cpu()
        ph = p[:, :7].double()
        d = ph[:, 1:] - ph[:, :-1]
        tot = ph[:, 6] - ph[:, 0]
        print(f"B={B}: n={n}, {T} tiles of {1 << H.tpf_tile_log2(n)}; tile+bucket {us:.1f} us "
              f"per localisation; cycles per tile workgroup mean {tot.mean():.0f} max {tot.max():.0f}")
        for i, name in enumerate(["init", "loads", "insert", "scan", "place", "rep"]):
            print(f"  {name:7s} mean {d[:, i].mean():8.0f}  max {d[:, i].max():8.0f}")
        rt0, rt1 = p[:, 8].double(), p[:, 9].double()  # 100 MHz realtime
        t0 = rt0.min()
        print(f"  wall (realtime, us): last start {(rt0.max() - t0) / 100:.1f}, "
              f"last end {(rt1.max() - t0) / 100:.1f}, mean duration {((rt1 - rt0) / 100).mean():.1f}")


if __name__ == "__main__":
    main()
