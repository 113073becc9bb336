#!/usr/bin/env python3
"""Fused sparse-LR forward / backward / KV resolve / update microbenchmark on one
65,536 x 39 Criteo-shaped minibatch (per-call microseconds, CUDA events)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from parameter_server_amd.ops.kv_table import KVTable, UpdateRule  # noqa: E402
from parameter_server_amd.ops.linear import (AUC_BINS, linear_backward, linear_forward,  # noqa: E402
                                             new_accum)
from parameter_server_amd.ops.localize import Localizer  # noqa: E402
from parameter_server_amd.ops.native import hipops  # noqa: E402
from parameter_server_amd.ops.synthetic import criteo_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
dev = "cuda"
keys, labels = criteo_batch(B, seed=3, row0=0, num_features=10 ** 9, device=dev)
L = Localizer(B * 39, 30, dev)
loc = L(keys)
U = loc.num_unique()
table = KVTable(1 << 28, dev, key_range=(0, 1 << 30))
slot = torch.empty(B * 39, dtype=torch.int64, device=dev)
w = torch.zeros(B * 39, dtype=torch.float32, device=dev)
metrics = new_accum(dev)  # striped, as the trainers use them
stats = new_accum(dev)
metrics1 = torch.zeros(8, dtype=torch.float64, device=dev)  # single-address layout
stats1 = torch.zeros(3, dtype=torch.float64, device=dev)
hist = torch.zeros(2 * AUC_BINS, dtype=torch.int32, device=dev)
coef = torch.empty(B, device=dev)
rule = UpdateRule("ftrl", "decay", 0.01, 10.0, 10.0, 1.0)


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


H = hipops()
it_, iv, isd, seed = table.init.args()


def first_touch():  # resolve of keys never seen (every key inserted), CUDA events
    tab = KVTable(1 << 28, dev, key_range=(0, 1 << 30))
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    H.kv_resolve(tab.slots, loc.uniq, loc.n_uniq, slot, w, True, it_, iv, isd, seed, tab._err,
                 tab._inserted, tab.home_base, tab.home_m)
    e.record()
    torch.cuda.synchronize()
    del tab
    return s.elapsed_time(e) * 1e3


res = {
    "B": B, "unique": U,
    "resolve_insert_us": first_touch(),
    "resolve_us": t(lambda: H.kv_resolve(table.slots, loc.uniq, loc.n_uniq, slot, w, True, it_, iv,
                                         isd, seed, table._err, table._inserted, table.home_base,
                                         table.home_m)),
    "forward_us": t(lambda: linear_forward(loc.local_col, w, labels, B=B, width=39, coef=coef,
                                           metrics=metrics, hist=hist)),
    "forward_nohist_us": t(lambda: linear_forward(loc.local_col, w, labels, B=B, width=39,
                                                  coef=coef, metrics=metrics, hist=None)),
    "forward_unstriped_us": t(lambda: linear_forward(loc.local_col, w, labels, B=B, width=39,
                                                     coef=coef, metrics=metrics1, hist=hist)),
    "update_unstriped_us": t(lambda: H.kv_update(table.slots, slot, loc.grad, loc.n_uniq,
                                                 *rule.args(), stats1)),
    "backward_us": t(lambda: linear_backward(loc, coef, B=B, width=39)),
    "update_us": t(lambda: H.kv_update(table.slots, slot, loc.grad, loc.n_uniq, *rule.args(),
                                       stats)),
}
print(json.dumps(res), flush=True)
