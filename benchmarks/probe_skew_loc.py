#!/usr/bin/env python3
"""Probe: the flat localiser's layout on skewed ids (bench_app's N * U^e files) vs bench.py's
generator: entries per tile, per bucket workgroup (distinct keys D, entries E, units split
by the light path), localisation time alone. One JSON line per distribution."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def keys_of(dist, B, N, dev):
    from parameter_server_amd.ops.synthetic import criteo_batch

    if dist == "criteo":
        return criteo_batch(B, seed=1, row0=0, num_features=N, device=dev)[0]
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    u = torch.rand(B, 39, device=dev, generator=g, dtype=torch.float64)
    return (N * u ** float(dist[3:])).long().sort(dim=1).values.reshape(-1).contiguous()


def main():
    from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer
    from parameter_server_amd.ops.native import hipops

    H = hipops()
    dev = torch.device("cuda", 0)
    B, N = 65536, 10 ** 8
    tr = SparseLRTrainer(SparseLRConfig(num_features=N, minibatch=B, table_capacity=1 << 27),
                         device=dev)
    for dist in os.environ.get("PROBE_DISTS", "criteo pow4 pow2 pow1").split():
        keys = keys_of(dist, B, N, dev)
        loc = tr.localizer(keys)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            loc = tr.localizer(keys)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 20 * 1e3
        g = H.tpf_groups(loc.nnz, loc.bits)
        c = loc.cnt[:4 * g].view(g, 4).cpu().long()
        E = c[:, 1] + c[:, 3]
        D = c[:, 0] + c[:, 2]
        split = int((c[:, 2] + c[:, 3] > 0).sum())
        dc = loc.dcnt.cpu().long()
        dc = dc[dc > 0]
        uk = torch.unique(keys).numel()
        top = torch.topk(E, 5).values.tolist()
        print(json.dumps({"dist": dist, "localize_ms": round(ms, 4), "groups": g,
                          "distinct_keys": uk, "D_sum": int(D.sum()), "E_sum": int(E.sum()),
                          "E_mean": round(float(E.float().mean()), 1), "E_top5": top,
                          "D_max": int(D.max()), "split_groups": split,
                          "tiles": int(dc.numel()), "tile_entries_mean": round(float(dc.float().mean()), 1),
                          "tile_entries_max": int(dc.max()), "err": int(loc.err.max())}),
              flush=True)


if __name__ == "__main__":
    main()
