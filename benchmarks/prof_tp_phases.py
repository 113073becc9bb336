#!/usr/bin/env python3
"""Per-phase shader-clock durations of the tp bucket kernel (tploc.hip TP_MARK):
average over workgroups of (mark k - mark k-1), one 65,536 x 39 Criteo minibatch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from parameter_server_amd.ops.localize import Localizer  # noqa: E402
from parameter_server_amd.ops.synthetic import criteo_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
keys, _ = criteo_batch(B, seed=3, row0=0, num_features=10 ** 9, device="cuda")
L = Localizer(B * 39, 30, "cuda", mode="tp")
L.tp_prof = torch.zeros(4096 * 12, dtype=torch.int64, device="cuda")
for _ in range(3):
    L(keys)
torch.cuda.synchronize()
p = L.tp_prof.view(-1, 12)[:, :7].cpu()
nb = int((p[:, 0] != 0).sum())
p = p[:nb].double()
d = p[:, 1:] - p[:, :-1]
names = ["toff+scan", "gather+insert", "compact", "ranksort", "starts", "assign"]
tot = (p[:, 6] - p[:, 0])
print(f"buckets {nb}: cycles per workgroup mean {tot.mean():.0f} max {tot.max():.0f}")
for i, n in enumerate(names):
    print(f"  {n:10s} mean {d[:, i].mean():8.0f}  max {d[:, i].max():8.0f}")
