#!/usr/bin/env python3
"""Per-bucket timeline of bl_bucket_kernel (wall_clock64 ticks, 100 MHz) for one
65,536 x 39 Criteo-shaped minibatch: phase A (bitmap count), look-back wait, rest."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from parameter_server_amd.ops.localize import Localizer  # noqa: E402
from parameter_server_amd.ops.native import hipops  # noqa: E402
from parameter_server_amd.ops.synthetic import criteo_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
keys, _ = criteo_batch(B, seed=3, row0=0, num_features=10 ** 9, device="cuda")
L = Localizer(B * 39, 30, "cuda", mode="bucket")
dbg = torch.zeros(4096 * 5, dtype=torch.int64, device="cuda")
H = hipops()
for _ in range(3):
    H.localize_bucket(keys, 30, L.btemp, L.pos_s, L.segid, L.uniq, L.seg_start, L.local_col,
                      L.n_uniq, L.grad, None, dbg)
torch.cuda.synchronize()
d = dbg.view(4096, 5).cpu().numpy().astype(np.int64)
t0 = d[:, 0].min()
start, a_end, lb_end, end, size = (d[:, i] for i in range(5))
print("span us", (end.max() - t0) / 100)
for name, v in (("phaseA", a_end - start), ("lookback", lb_end - a_end), ("rest", end - lb_end),
                ("total", end - start)):
    print(f"{name:9s} us: mean {v.mean()/100:.2f} p50 {np.median(v)/100:.2f} p99 "
          f"{np.percentile(v, 99)/100:.2f} max {v.max()/100:.2f} (bucket {v.argmax()}, size {size[v.argmax()]})")
print("start offsets us: p50 %.1f max %.1f" % (np.median(start - t0) / 100, (start - t0).max() / 100))
big = np.argsort(size)[-5:]
for b in big:
    print("bucket", b, "size", size[b], "A", (a_end[b]-start[b])/100, "lb", (lb_end[b]-a_end[b])/100,
          "rest", (end[b]-lb_end[b])/100, "start", (start[b]-t0)/100)
