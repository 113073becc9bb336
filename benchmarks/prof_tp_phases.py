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
full = L.tp_prof.view(-1, 12).cpu()
p = full[:, :8]
nb = int((p[:, 0] != 0).sum())
p = p[:nb].double()
d = p[:, 1:] - p[:, :-1]
names = ["toff+scan", "gather+insert", "compact+publish", "ranksort", "look-back",
         "uniq/starts", "entries"]
tot = (p[:, 7] - p[:, 0])
print(f"buckets {nb}: cycles per workgroup mean {tot.mean():.0f} max {tot.max():.0f}")
for i, n in enumerate(names):
    print(f"  {n:15s} mean {d[:, i].mean():8.0f}  max {d[:, i].max():8.0f}")
rt0, rt1 = full[:nb, 8].double(), full[:nb, 9].double()  # 100 MHz realtime
t0 = rt0.min()
print(f"  wall (realtime, us): last start {(rt0.max() - t0) / 100:.1f}, "
      f"last end {(rt1.max() - t0) / 100:.1f}, mean duration {((rt1 - rt0) / 100).mean():.1f}")

# ---- fused forward + backward (tploc.hip tp_fwd_bwd FB_MARK) ----
from parameter_server_amd.ops.linear import AUC_BINS, linear_fwd_bwd, new_accum  # noqa: E402
from parameter_server_amd.ops.native import hipops  # noqa: E402

labels = (torch.rand(B, device="cuda") < 0.3).float()
L2 = Localizer(B * 39, 30, "cuda", mode="tp", lazy_cols=True)
loc = L2(keys)
w = torch.randn(int(loc.uniq.numel()), device="cuda") * 0.01
met, hist = new_accum("cuda"), torch.zeros(8 * 2 * AUC_BINS, dtype=torch.int32, device="cuda")
cf = torch.empty(B, device="cuda")
T = (B * 39 + 8191) // 8192
prof = torch.zeros(T * 16, dtype=torch.int64, device="cuda")


def run():
    hipops().tp_fb_set_prof(None)
    for _ in range(5):
        linear_fwd_bwd(loc, w, labels, B=B, width=39, coef=cf, metrics=met, hist=hist)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(50):
        linear_fwd_bwd(loc, w, labels, B=B, width=39, coef=cf, metrics=met, hist=hist)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 50 * 1e3
    hipops().tp_fb_set_prof(prof)
    for _ in range(3):
        linear_fwd_bwd(loc, w, labels, B=B, width=39, coef=cf, metrics=met, hist=hist)
    torch.cuda.synchronize()
    hipops().tp_fb_set_prof(None)
    p = prof.view(T, 16).cpu()
    ph = p[:, :7].double()
    d = ph[:, 1:] - ph[:, :-1]
    names = ["loads", "forward", "hist+zero", "atomics", "atomics-drain", "psum"]
    tot = ph[:, 6] - ph[:, 0]
    print(f"fused: {us:.1f} us per fwd+bwd (+ entry scan); "
          f"tiles {T}: cycles per workgroup mean {tot.mean():.0f} max {tot.max():.0f}")
    for i, n in enumerate(names):
        print(f"  {n:13s} mean {d[:, i].mean():8.0f}  max {d[:, i].max():8.0f}")
    rt0, rt1 = p[:, 8].double(), p[:, 9].double()  # 100 MHz realtime
    t0 = rt0.min()
    print(f"  wall (realtime, us): last start {(rt0.max() - t0) / 100:.1f}, "
          f"last end {(rt1.max() - t0) / 100:.1f}, mean duration {((rt1 - rt0) / 100).mean():.1f}")


run()
