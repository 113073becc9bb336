"""Debug: repeated tp_fwd_bwd on one compact localisation -- which psum entries differ."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from parameter_server_amd.ops.linear import linear_fwd_bwd
from parameter_server_amd.ops.localize import Localizer
from parameter_server_amd.ops.synthetic import criteo_batch
DEV = torch.device("cuda")
B, width = 65536, 39
keys, labels = criteo_batch(B, seed=9, row0=0, num_features=10 ** 9, device=DEV)
n = keys.numel()
L = Localizer(n, 30, DEV, mode="tp", lazy_cols=True)(keys)
U = int(L.n_uniq.item())
w = torch.randn(U, device=DEV) * 0.05
parts = []
for r in range(4):
    linear_fwd_bwd(L, w, labels, B=B, width=width, coef=torch.empty(B, device=DEV))
    torch.cuda.synchronize()
    parts.append(L.tile.psum.clone())
T = (n + 8191) // 8192
dc = L.tile.dcnt[:T].cpu()
for r in range(1, 4):
    d = (parts[r] != parts[0]).nonzero().flatten().cpu()
    tiles = sorted(set((d // 8192).tolist()))
    inside = [(int(i) % 8192) < int(dc[int(i) // 8192]) for i in d[:2000]]
    print(f"run {r}: {d.numel()} differing psum entries, tiles {tiles[:20]} (#{len(tiles)}), "
          f"inside dcnt: {sum(inside)}/{len(inside)}", flush=True)
    if d.numel():
        i = int(d[0]); print("  e.g.", i, parts[0][i].item(), parts[r][i].item(), "dcnt", int(dc[i // 8192]))
