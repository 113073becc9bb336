#!/usr/bin/env python3
"""One W&D forward product (16384 x 1024 x 4992, K-major bf16) through each own 256x256
variant and hipBLASLt, a few calls each: a target for rocprofv3 --pmc passes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from parameter_server_amd.ops.native import hipops  # noqa: E402

M, N, K = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (16384, 1024, 4992)))
A = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
B = (torch.rand(N, K, device="cuda") * 2 - 1).to(torch.bfloat16)
C = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
for _ in range(5):
    for v in (0, 2):
        hipops().gemm_nt256(A, B, M, N, K, None, False, C, None, v)
    torch.mm(A, B.t())
torch.cuda.synchronize()
