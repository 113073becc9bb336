"""bf16 MFMA GEMM (csrc/hip/gemm.hip) and the Linear-layer products built on it.

``gemm(A, a_kmajor, B, b_kmajor, M, N, K)``: C[m, n] = sum_k A(m, k) B(n, k) with
A(m, k) = A[m, k] (K-major, row-major [M, K]) or A[k, m] (MN-major, row-major
[K, M]); B likewise. fp32 accumulation; fused epilogues (bias, ReLU, ReLU-mask
of an auxiliary tensor); bf16 and / or fp32 outputs.

For a layer with weights ``W [N_out, K_in]`` (bf16) and input ``X [B, K_in]``:
* forward      ``Z = X W^T``      -> A = X (K-major), B = W (K-major)
* input grad   ``dX = dZ W``      -> A = dZ (K-major), B = W (MN-major)
* weight grad  ``dW = dZ^T X``    -> A = dZ (MN-major), B = X (MN-major)
CPU tensors use the same math in fp32 PyTorch (the numerics reference).
"""
from __future__ import annotations

import torch

from .native import hipops, is_gpu

EPI_BIAS, EPI_RELU, EPI_MASK, EPI_COLSUM = 1, 2, 4, 8


def _view(t: torch.Tensor, kmajor: bool, rows: int, K: int) -> torch.Tensor:
    return t.reshape(rows, K) if kmajor else t.reshape(K, rows).t()


def auto_splitk(M: int, N: int, K: int, target_blocks: int = 1024) -> int:
    """K splits so that a small-output / long-K product (the weight gradient) still
    puts >= ~4 blocks on each of the 256 CUs; each split keeps >= 16 K-tiles."""
    tiles = -(-M // 128) * -(-N // 128)
    # measured (benchmarks/bench_gemm.py --wd-sweep, K = 16384): 1024x4992 best at 4
    # splits, 512x1024 at 16 (32: +50 % from the fp32 atomics), 256x512 at 16-32
    return max(1, min(-(-target_blocks // tiles), K // 1024))


def gemm(A, a_kmajor: bool, B, b_kmajor: bool, M: int, N: int, K: int, *, bias=None,
         relu: bool = False, mask=None, out_bf16: bool = True, out_f32=None, beta: float = 0.0,
         splitk: int = 1, colsum=None):
    """Returns the bf16 output (or None when ``out_bf16`` is False and ``out_f32`` given).
    ``splitk > 1`` (fp32 output only, beta 0 or 1) splits K over blocks and adds the
    partial products atomically. ``colsum`` [N] fp32 += the output's column sums
    (of the bf16 values when there is a bf16 output)."""
    epi = (EPI_BIAS if bias is not None else 0) | (EPI_RELU if relu else 0) | \
        (EPI_MASK if mask is not None else 0) | (EPI_COLSUM if colsum is not None else 0)
    if is_gpu(A):
        C = torch.empty(M, N, dtype=torch.bfloat16, device=A.device) if out_bf16 else None
        lda = K if a_kmajor else M
        ldb = K if b_kmajor else N
        hipops().gemm_bf16(A, a_kmajor, lda, B, b_kmajor, ldb, M, N, K, epi, bias, mask, N, C, N,
                           out_f32, N, beta, splitk, colsum)
        return C
    a = _view(A, a_kmajor, M, K).float()
    b = _view(B, b_kmajor, N, K).float()
    x = a @ b.t()
    if bias is not None:
        x = x + bias.float()
    if relu:
        x = x.clamp_min(0)
    if mask is not None:
        x = x * (mask.reshape(M, N).float() > 0)
    if colsum is not None:
        colsum += (x.to(torch.bfloat16).float() if out_bf16 else x).sum(0)
    if out_f32 is not None:
        o = out_f32.view(M, N)
        o.copy_(x + beta * o if beta != 0.0 else x)
    return x.to(torch.bfloat16) if out_bf16 else None


# Layer products on the GPU: "mfma" = the hand-written kernels (forward products with
# K % 64 == 0 and N >= 256 on the 256x256 LDS-DMA kernels of gemm256.hip, the rest on
# the 128x128 kernel above with fused epilogues); "hipblaslt" = the vendor library GEMM
# (torch.mm / addmm with its own bias + ReLU epilogue) + separate elementwise kernels;
# "auto" = per product, the faster of the two as measured on MI355X
# (benchmarks/bench_gemm256.py, B = 16384, uniform random bf16,
# profiles/r4_gemm256_ring.log): the library for the plain long-K products -- the
# layer-0 forward (K = 4992: 1441 vs 1270 TFLOP/s for the best own variant) and the
# unmasked input gradient (1125 vs 803) -- and the own kernels where their fused
# epilogues save passes (masked input gradient + bias-gradient column sums, the short-K
# forwards with their fused bias + ReLU: 1024 -> 512 604 own (128x128) vs 644 library,
# 512 -> 256 312 vs 222) and for every weight gradient (TN 256x256 split-K: 668 vs 542,
# 362 vs 167, 127 vs 45 TFLOP/s).
BACKENDS = ("mfma", "hipblaslt", "auto")


def _nt256_variant(K: int) -> int:
    """gemm256.hip NT variant: the one-barrier kernel (0). The 4-slot LDS ring (4) is
    faster in isolation (1270 vs 1156 TFLOP/s at K = 4992, profiles/r4_gemm256_ring.log)
    but not inside the wide & deep step (gemm="mfma": 1.041 vs 1.029 ms, gpurun r4n),
    where the other stream's kernels share the CUs; PSAMD_GEMM_NT256 selects one."""
    import os

    v = os.environ.get("PSAMD_GEMM_NT256")
    return int(v) if v is not None else 0
_addmm_act = getattr(torch, "_addmm_activation", None)


def linear_forward(X, W, bias=None, relu=False, backend: str = "mfma", bias16=None):
    """X [B, K] bf16, W [N, K] bf16 -> act(X W^T + b) [B, N] bf16 (``bias16``: a bf16
    copy of ``bias`` for the library path)."""
    Bn, K = X.shape
    N = W.shape[0]
    if backend == "auto":
        backend = "hipblaslt" if K >= 1024 else "mfma"
    if backend == "hipblaslt" and is_gpu(X):
        if bias is None:
            Z = torch.mm(X, W.t())
            return Z.relu_() if relu else Z
        b = bias16 if bias16 is not None else bias.to(X.dtype)
        if relu and _addmm_act is not None:
            return _addmm_act(b, X, W.t())
        Z = torch.addmm(b, X, W.t())
        return Z.relu_() if relu else Z
    if is_gpu(X) and K % 64 == 0 and -(-Bn // 256) * -(-N // 256) >= 256 and \
            X.is_contiguous() and W.is_contiguous():
        # 256x256 LDS-DMA kernel (gemm256.hip) once its tiles fill the 256 CUs: 1085 vs
        # 739 TFLOP/s for the 128x128 kernel on 16384 x 1024 x 4992; with fewer tiles
        # (16384 x 512) the 128x128 kernel wins (profiles/r2_gemm256.log)
        Z = torch.empty(Bn, N, dtype=torch.bfloat16, device=X.device)
        hipops().gemm_nt256(X, W, Bn, N, K, bias, relu, Z, None, _nt256_variant(K))
        return Z
    return gemm(X, True, W, True, Bn, N, K, bias=bias, relu=relu)


def linear_input_grad(dZ, W, mask=None, backend: str = "mfma", colsum=None):
    """dZ [B, N], W [N, K] -> dZ W [B, K] (times the ReLU mask of ``mask`` [B, K]);
    ``colsum`` [K] += its column sums (the bias gradient of the layer below)."""
    Bn, N = dZ.shape
    K = W.shape[1]
    if backend == "auto":
        backend = "hipblaslt" if mask is None and colsum is None and K >= 1024 else "mfma"
    if backend == "hipblaslt" and is_gpu(dZ):
        import os

        if os.environ.get("PSAMD_DX_WT", "1") == "1" and W.is_contiguous() and N % 64 == 0 \
                and K % 64 == 0:
            # both operands K-major (the forward's layout) through a transposed weight copy
            # (~5 us): the library's NT kernel beats its NN one on the layer-0 input
            # gradient, wide & deep step 0.956-0.958 -> 0.939-0.948 ms
            # (profiles/r4_wide_deep_fusion_ab.log); PSAMD_DX_WT=0: the plain product
            Wt = torch.empty(K, N, dtype=W.dtype, device=W.device)
            hipops().transpose_bf16(W, Wt)
            dX = torch.mm(dZ, Wt.t())
        else:
            dX = torch.mm(dZ, W)
        if mask is not None:
            dX.mul_(mask > 0)
        if colsum is not None:
            hipops().colsum_bf16(dX, colsum)
        return dX
    if is_gpu(dZ) and mask is None and colsum is None and N % 64 == 0 and \
            -(-Bn // 256) * -(-K // 256) >= 256 and dZ.is_contiguous():
        # unmasked long-N input gradient (layer 0): the 256x256 LDS-DMA kernel on a
        # transposed weight copy (10 MB for 1024 x 4992) beats the MN-major 128x128
        # kernel: 750 vs 628 TFLOP/s on 16384 x 4992 x 1024 (profiles/r2_gemm256.log)
        if N % 64 == 0 and K % 64 == 0 and W.is_contiguous():
            Wt = torch.empty(K, N, dtype=torch.bfloat16, device=W.device)
            hipops().transpose_bf16(W, Wt)  # (~5 us; torch's strided copy ~50 us)
        else:
            Wt = W.t().contiguous()
        dX = torch.empty(Bn, K, dtype=torch.bfloat16, device=dZ.device)
        hipops().gemm_nt256(dZ, Wt, Bn, K, N, None, False, dX, None, _nt256_variant(N))
        return dX
    return gemm(dZ, True, W, False, Bn, K, N, mask=mask, colsum=colsum)


def linear_weight_grad(dZ, X, out=None, beta: float = 0.0, backend: str = "mfma",
                       deferred=None):
    """dZ [B, N], X [B, K] -> dW = dZ^T X [N, K] fp32 (``out`` accumulates with ``beta``).
    ``deferred`` (a list): where the 256x256 TN kernel runs, only its GEMM is issued and
    the split-K reduce is appended to the list as a callable for the caller to issue
    later (on the same stream), so the next layer's GEMM is not queued behind it."""
    Bn, N = dZ.shape
    K = X.shape[1]
    out = torch.empty(N, K, dtype=torch.float32, device=dZ.device) if out is None else out
    if backend == "auto":  # (PSAMD_DW_LIB=1: the library for the weight gradients, A/B)
        import os

        backend = "hipblaslt" if os.environ.get("PSAMD_DW_LIB", "0") == "1" else "mfma"
    if backend == "hipblaslt" and is_gpu(dZ):
        r = torch.mm(dZ.t(), X, out_dtype=torch.float32)
        if beta == 0.0:
            out.copy_(r)
        elif beta == 1.0:
            out.add_(r)
        else:
            out.mul_(beta).add_(r)
        return out
    if is_gpu(dZ) and tn256_ok(N, K, Bn) and dZ.is_contiguous() and X.is_contiguous() and \
            out.is_contiguous():
        # 256x256 kernel reading both MN-major operands through transposed LDS reads
        # (gemm256.hip gemm_tn256), split-K partials summed in a fixed order
        S = tn256_splits(N, K, Bn)
        part = torch.empty(S * N * K, dtype=torch.float32, device=dZ.device)
        if deferred is not None:
            H = hipops()
            H.gemm_tn256(dZ, X, N, K, Bn, S, part, out, float(beta), 1)
            deferred.append(lambda: H.gemm_tn256(dZ, X, N, K, Bn, S, part, out, float(beta), 2))
            return out
        if S > 1 and _TN_FUSED_REDUCE:
            # the split-K reduce inside the GEMM (the last split of each tile sums the
            # partials in split order: bitwise the two-launch result, no separate pass)
            hipops().gemm_tn256(dZ, X, N, K, Bn, S, part, out, float(beta), 3,
                                _tile_counters(dZ.device, -(-N // 256) * -(-K // 256)))
            return out
        hipops().gemm_tn256(dZ, X, N, K, Bn, S, part, out, float(beta))
        return out
    sk = auto_splitk(N, K, Bn) if beta in (0.0, 1.0) else 1
    gemm(dZ, False, X, False, N, K, Bn, out_bf16=False, out_f32=out, beta=beta, splitk=sk)
    return out


# PSAMD_TN_FUSED_REDUCE=1 (A/B, off): the split-K reduce inside the TN GEMM's last split
# per tile. Bitwise equal, but the W&D step measured 3.77 ms (all layers) / 1.14-1.16 ms
# (S <= 4 only) vs 0.936-0.939 with the separate reduce pass: the reduce then runs on one
# workgroup per 256 x 256 tile (profiles/r5_tn_fused_reduce_ab.log)
_TN_FUSED_REDUCE = __import__("os").environ.get("PSAMD_TN_FUSED_REDUCE", "0") == "1"
_TILE_CTRS: dict = {}


def _tile_counters(dev, n: int):
    """Zeroed int32 per-tile counters of gemm_tn256's in-kernel split-K reduce (each
    launch leaves them zeroed; one buffer per device and stream ordering keeps launches
    apart: a side-stream and a main-stream TN GEMM never run at once here)."""
    key = (str(dev), torch.cuda.current_stream(dev).cuda_stream)
    t = _TILE_CTRS.get(key)
    if t is None or t.numel() < n:
        t = torch.zeros(max(n, 1024), dtype=torch.int32, device=dev)
        _TILE_CTRS[key] = t
    return t


def tn256_ok(M: int, N: int, K: int) -> bool:
    """gemm_tn256 takes the weight gradient [M, N] over K batch rows when both output
    sides fill 256-wide tiles and the batch is a multiple of 64 (>= 8 K-steps)."""
    import os

    if os.environ.get("PSAMD_TN256", "1") == "0":
        return False
    return M >= 256 and N >= 256 and M % 8 == 0 and N % 8 == 0 and K % 64 == 0 and K >= 512


def tn256_splits(M: int, N: int, K: int) -> int:
    """K splits: enough workgroups for the 256 CUs (one 128 KB workgroup each, so at most
    256 in one round), each split >= 8 K-steps (512 rows)."""
    tiles = -(-M // 256) * -(-N // 256)
    return max(1, min(256 // tiles if tiles <= 256 else 1, K // 512))
