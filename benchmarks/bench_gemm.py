#!/usr/bin/env python3
"""TFLOP/s of the hand-written bf16 MFMA GEMM (csrc/hip/gemm.hip) on the wide & deep
MLP shapes and a square reference shape, vs torch.matmul (hipBLASLt) for context."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from parameter_server_amd.ops import gemm as G  # noqa: E402


def t(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e-3


rows = []
for name, (M, N, K, ak, bk) in {
    "fwd 16384x1024x4992": (16384, 1024, 4992, True, True),
    "dX 16384x4992x1024": (16384, 4992, 1024, True, False),
    "dW 1024x4992x16384": (1024, 4992, 16384, False, False),
    "fwd 16384x512x1024": (16384, 512, 1024, True, True),
    "square 4096": (4096, 4096, 4096, True, True),
    "square 8192": (8192, 8192, 8192, True, True),
}.items():
    A = (torch.rand((M, K) if ak else (K, M), device="cuda") * 2 - 1).to(torch.bfloat16)
    B = (torch.rand((N, K) if bk else (K, N), device="cuda") * 2 - 1).to(torch.bfloat16)
    ours = t(lambda: G.gemm(A, ak, B, bk, M, N, K))
    a = A if ak else A.t()
    b = B if bk else B.t()
    ref = t(lambda: a @ b.t())
    fl = 2.0 * M * N * K
    rows.append({"shape": name, "ours_tflops": fl / ours / 1e12, "torch_tflops": fl / ref / 1e12})
    print(json.dumps(rows[-1]), flush=True)

if "--wd-sweep" in sys.argv:
    # weight-gradient split-K sweep on the wide & deep shapes (fp32 output, beta 0)
    for N, K in ((1024, 4992), (512, 1024), (256, 512)):
        Bn = 16384
        dZ = (torch.rand(Bn, N, device="cuda") - 0.5).to(torch.bfloat16)
        X = (torch.rand(Bn, K, device="cuda") - 0.5).to(torch.bfloat16)
        out = torch.empty(N, K, device="cuda")
        for sk in (1, 2, 4, 8, 16, 32):
            dt = t(lambda: G.gemm(dZ, False, X, False, N, K, Bn, out_bf16=False, out_f32=out,
                                  splitk=sk))
            print(json.dumps({"dW": f"{N}x{K}x{Bn}", "splitk": sk, "us": dt * 1e6,
                              "tflops": 2.0 * N * K * Bn / dt / 1e12,
                              "auto": G.auto_splitk(N, K, Bn)}), flush=True)

if "--wd-backends" in sys.argv:
    # each wide & deep layer product: own kernel (fused epilogue) vs hipBLASLt
    Bn = 16384
    for K, N in ((4992, 1024), (1024, 512), (512, 256)):
        X = (torch.rand(Bn, K, device="cuda") - 0.5).to(torch.bfloat16)
        W = ((torch.rand(N, K, device="cuda") - 0.5) * 0.05).to(torch.bfloat16)
        b = torch.rand(N, device="cuda")
        bb = b.to(torch.bfloat16)
        dZ = (torch.rand(Bn, N, device="cuda") - 0.5).to(torch.bfloat16)
        cs = torch.zeros(K, device="cuda")
        dW = torch.empty(N, K, device="cuda")
        fl = 2.0 * Bn * N * K
        res = {
            "fwd own (bias+relu)": t(lambda: G.linear_forward(X, W, b, relu=True)),
            "fwd addmm+relu_": t(lambda: torch.addmm(bb, X, W.t()).relu_()),
            "fwd _addmm_activation": t(lambda: torch._addmm_activation(bb, X, W.t())),
            "dX own (mask+colsum)": t(lambda: G.linear_input_grad(dZ, W, mask=X, colsum=cs)),
            "dX own plain": t(lambda: G.linear_input_grad(dZ, W)),
            "dX mm": t(lambda: torch.mm(dZ, W)),
            "dW own split": t(lambda: G.linear_weight_grad(dZ, X, out=dW)),
            "dW mm fp32": t(lambda: torch.mm(dZ.t(), X, out_dtype=torch.float32)),
            "dW transpose+mm NT": t(lambda: torch.mm(dZ.t().contiguous(), X.t().contiguous().t(),
                                                     out_dtype=torch.float32)),
            "dW transpose only": t(lambda: (dZ.t().contiguous(), X.t().contiguous())),
            "dW transpose+own NT": t(lambda: G.gemm(dZ.t().contiguous(), True,
                                                    X.t().contiguous(), True, N, K, Bn,
                                                    out_bf16=False, out_f32=dW)),
        }
        for k, v in res.items():
            print(json.dumps({"layer": f"{K}->{N}", "op": k, "us": v * 1e6,
                              "tflops": fl / v / 1e12}), flush=True)
