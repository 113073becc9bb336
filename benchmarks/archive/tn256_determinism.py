import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from parameter_server_amd.ops.native import hipops
from parameter_server_amd.ops import gemm as GM
H = hipops()
for (M, N, K) in [(256, 2496, 1024), (1024, 4992, 16384), (256, 512, 1024)]:
    S = GM.tn256_splits(M, N, K)
    g = torch.Generator(device="cuda").manual_seed(1)
    A = (torch.rand(K, M, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(K, N, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    ref = A.float().t() @ B.float()
    part = torch.empty(S * M * N, device="cuda")
    outs = []
    for it in range(20):
        C = torch.zeros(M, N, device="cuda")
        H.gemm_tn256(A, B, M, N, K, S, part, C, 0.0)
        outs.append(C)
    torch.cuda.synchronize()
    nd = sum(int(not torch.equal(outs[0], o)) for o in outs)
    err = ((outs[0] - ref).abs().max()).item()
    print("shape", M, N, K, "S", S, "nondeterministic runs", nd, "max abs err", err, flush=True)
