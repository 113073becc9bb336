#!/usr/bin/env python3
"""Per-kernel device time of one data preparation + fused forward/backward at a given
minibatch size (argv[1], default 65,536): run under rocprofv3 --kernel-trace --stats to
split localize_tpf into its tile and bucket kernels. B = 53,760 gives 256 tiles of 8,192
occurrences (one per CU), B = 65,536 gives 313 (57 CUs hold two): whether the per-tile
kernels (tile, fused forward/backward) pay for the second round."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from parameter_server_amd.models import SparseLRConfig, SparseLRTrainer  # noqa: E402
from parameter_server_amd.ops.native import hipops  # noqa: E402
from parameter_server_amd.ops.synthetic import criteo_batch  # noqa: E402

os.environ["PSAMD_FLAT"] = "1"
B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
dev = torch.device("cuda")
H = hipops()
cfg = SparseLRConfig(num_features=10 ** 9, minibatch=B, table_capacity=1 << 26)
tr = SparseLRTrainer(cfg, device=dev)
for t in range(3):
    k, lab = criteo_batch(B, seed=5, row0=t * B, num_features=cfg.num_features, device=dev)
    tr.step(k, lab, width=39)
loc = tr.localize(k, buf=0)
tr.step(k, lab, width=39, loc=loc)
torch.cuda.synchronize()
n, bits = loc.nnz, loc.bits
lz = tr._localizers[0]
f = lz.flat
L = H.LaunchList()
for _ in range(30):
    L.add_criteo_gen(5, 0, B, B, cfg.num_features, 1.1, k, lab)
    L.add_localize_tpf(k, n, bits, lz.ptemp, f.dcnt, f.rep, f.uniqf, f.ent_pos, f.ent_j, f.cnt,
                       f.err, False)
    L.add_tp_fwd_bwd(loc.rep, loc.dcnt, None, n, 39, None, loc.w_ent, lab, B, 0, tr.coef[:B],
                     tr.metrics, tr.hist, 2048, loc.psum, None, None, None, None, False)
L.run()
torch.cuda.synchronize()
print("B", B, "occurrences", n, "tiles", -(-n // 8192), flush=True)
