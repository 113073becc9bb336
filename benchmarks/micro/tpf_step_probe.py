#!/usr/bin/env python3
"""What bounds the flat step kernel (csrc/hip/tploc.hip tpf_step / tpf_step2)? Times, on
one localised 65,536 x 39 Criteo-shaped minibatch after a few training steps: the pull
half, the update half, both in one launch, an empty launch (all counts 0), and the
compact path's kv_resolve of the same distinct keys, for table capacities 2^22 / 2^26 /
2^31 (the bench's: 64 GiB of slots) -- a TLB / page-walk bound would show as time growing
with the table's span at a fixed key count."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer  # noqa: E402
from parameter_server_amd.ops.native import hipops  # noqa: E402
from parameter_server_amd.ops.synthetic import criteo_batch  # noqa: E402

os.environ["PSAMD_FLAT"] = "1"
dev = torch.device("cuda")
H = hipops()
B = 65536


def timeit_list(add, it=30):
    """Device time per op of ``it`` copies of one op in a native launch list (validated
    once, issued from C++: the host issue cost of a Python binding call stays out)."""
    L = H.LaunchList()
    for _ in range(it):
        add(L)
    L.run()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    L.run()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def timeit(fn, it=30):
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


for lg in (22, 26, 31):
    cfg = SparseLRConfig(num_features=10 ** 9, minibatch=B, table_capacity=1 << lg)
    tr = SparseLRTrainer(cfg, device=dev)
    for t in range(4):
        k, lab = criteo_batch(B, seed=5, row0=t * B, num_features=cfg.num_features, device=dev)
        tr.step(k, lab, width=39)
    k, lab = criteo_batch(B, seed=5, row0=4 * B, num_features=cfg.num_features, device=dev)
    loc = tr.localize(k, buf=0)
    tr.step(k, lab, width=39, loc=loc)  # psum / slot_u of this minibatch are valid now
    torch.cuda.synchronize()
    n, bits, tb = loc.nnz, loc.bits, tr.table
    it_, iv, isd, seed = tb.init.args()
    common = (tb.slots, it_, iv, isd, seed, tb._err, tb._inserted, tb.home_base, tb.home_m,
              *tr.rule.args(), tr.stats)
    zero = tuple(torch.zeros_like(x) if i == 0 else x for i, x in enumerate(loc.bufs))
    row = {"table_log2": lg}
    for v1 in ("1", "0"):
        os.environ["PSAMD_TPF_STEP2"] = "0" if v1 == "1" else "1"
        tag = "v1" if v1 == "1" else "v2"
        row[f"pull_{tag}"] = timeit_list(lambda L: L.add_tpf_step(
            n, bits, None, None, loc.bufs, loc.w_ent, *common, None, None, None))
        row[f"update_{tag}"] = timeit_list(lambda L: L.add_tpf_step(
            n, bits, loc.bufs, loc.psum, None, None, *common, None, None, None))
        row[f"both_{tag}"] = timeit_list(lambda L: L.add_tpf_step(
            n, bits, loc.bufs, loc.psum, loc.bufs, loc.w_ent, *common, None, None, None))
        row[f"empty_{tag}"] = timeit_list(lambda L: L.add_tpf_step(
            n, bits, zero, loc.psum, zero, loc.w_ent, *common, None, None, None))
    row["fwd_bwd"] = timeit_list(lambda L: L.add_tp_fwd_bwd(
        loc.rep, loc.dcnt, None, n, 39, None, loc.w_ent, lab, B, 0, tr.coef[:B], tr.metrics,
        tr.hist, 2048, loc.psum, None, None, None, None, False))
    lz = tr._localizers[0]
    f = lz.flat
    row["localize_tpf"] = timeit_list(lambda L: L.add_localize_tpf(
        k, n, bits, lz.ptemp, f.dcnt, f.rep, f.uniqf, f.ent_pos, f.ent_j, f.cnt, f.err, False))
    uk = loc.unique_keys().to(dev)
    row["distinct_keys"] = int(uk.numel())
    row["kv_resolve_same_keys"] = timeit(lambda: tb.resolve(uk, insert=False, with_w=True))
    perm = uk[torch.randperm(uk.numel(), device=dev)]
    row["kv_resolve_shuffled"] = timeit(lambda: tb.resolve(perm, insert=False, with_w=True))
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in row.items()}),
          flush=True)
    del tr, tb
    torch.cuda.empty_cache()
