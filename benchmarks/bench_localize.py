#!/usr/bin/env python3
"""Localisation + backward of one 65,536 x 39 Criteo-shaped minibatch: radix-sort +
RLE (sort32.hip) vs partition + LDS bitmaps (bucketloc.hip) vs the sort-free hash
dedup (hashloc.hip), per-call microseconds."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from parameter_server_amd.ops.linear import (AUC_BINS, linear_backward, linear_forward,  # noqa: E402
                                             linear_fwd_bwd, new_accum)
from parameter_server_amd.ops.localize import Localizer  # noqa: E402
from parameter_server_amd.ops.synthetic import criteo_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
BITS = int(os.environ.get("PSAMD_LOC_BITS", "30"))  # 34: 10^10 features
keys, labels = criteo_batch(B, seed=3, row0=0, num_features=10 ** 10 if BITS > 32 else 10 ** 9,
                       device="cuda")
coef = torch.randn(B, device="cuda")


def t(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


for mode in os.environ.get("PSAMD_LOC_MODES", "sort,part,tp").split(","):
    L = Localizer(B * 39, BITS, "cuda", mode=mode)
    loc = L(keys)
    us_loc = t(lambda: L(keys))
    us_bwd = t(lambda: linear_backward(loc, coef, B=B, width=39))
    out = {"mode": mode, "bits": BITS, "digit_bits": getattr(L, "digit_bits", None), "B": B,
           "unique": loc.num_unique(), "localize_us": us_loc, "backward_us": us_bwd}
    # forward + backward of the step (w_local, loss, metrics, AUC histogram)
    w = torch.randn(loc.num_unique(), device="cuda") * 0.05
    met, hist = new_accum("cuda"), torch.zeros(8 * 2 * AUC_BINS, dtype=torch.int32, device="cuda")
    cf = torch.empty(B, device="cuda")

    def unfused():
        linear_forward(loc.local_col, w, labels, B=B, width=39, coef=cf, metrics=met, hist=hist)
        linear_backward(loc, cf, B=B, width=39)
    out["fwd_bwd_us"] = t(unfused)
    if mode == "tp":
        Lz = Localizer(B * 39, BITS, "cuda", mode=mode, lazy_cols=True)
        lz = Lz(keys)
        out["localize_lazy_cols_us"] = t(lambda: Lz(keys))
        out["fused_fwd_bwd_us"] = t(lambda: linear_fwd_bwd(lz, w, labels, B=B, width=39, coef=cf,
                                                           metrics=met, hist=hist))
    print(json.dumps(out), flush=True)
