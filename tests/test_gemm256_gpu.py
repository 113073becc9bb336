"""256x256 LDS-DMA bf16 GEMM (csrc/hip/gemm256.hip) against an fp32 PyTorch reference:
full and ragged tiles (rows clamped on load, masked on store), bias / ReLU epilogue,
bf16 (LDS-staged 16-B stores on full tiles) and fp32 outputs, and the forward layer
product that uses it."""
import pytest
import torch

from parameter_server_amd.ops import gemm as GM
from parameter_server_amd.ops.native import hipops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(A, B, bias, relu):
    x = A.float() @ B.float().t()
    if bias is not None:
        x = x + bias
    return x.clamp_min(0) if relu else x


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 128), (300, 1000, 192),
                                   (1024, 4992, 1024), (4097, 260, 640), (64, 64, 64)])
@pytest.mark.parametrize("epi", ["none", "bias_relu"])
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6])
def test_gemm256_matches_fp32(M, N, K, epi, variant):
    g = torch.Generator(device=DEV).manual_seed(M * 7 + N + K)
    A = (torch.rand(M, K, device=DEV, generator=g) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, K, device=DEV, generator=g) * 2 - 1).to(torch.bfloat16)
    bias = torch.randn(N, device=DEV) if epi != "none" else None
    relu = epi != "none"
    C = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
    Cf = torch.full((M, N), float("nan"), dtype=torch.float32, device=DEV)
    hipops().gemm_nt256(A, B, M, N, K, bias, relu, C, None, variant)
    hipops().gemm_nt256(A, B, M, N, K, bias, relu, None, Cf, variant)
    ref = _ref(A, B, bias, relu)
    torch.testing.assert_close(Cf, ref, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(C.float(), ref, rtol=1e-2, atol=2e-2)


def test_gemm256_pingpong_repeatable_long_k():
    """The ping-pong schedule's counted waits: a long-K product repeated many times is
    bit-identical every time and equals the one-barrier kernel's fp32 output
    (a stale LDS-DMA read would show up as a differing tile)."""
    M, N, K = 2048, 2048, 4096
    g = torch.Generator(device=DEV).manual_seed(5)
    A = (torch.rand(M, K, device=DEV, generator=g) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, K, device=DEV, generator=g) * 2 - 1).to(torch.bfloat16)
    ref = torch.empty(M, N, device=DEV)
    hipops().gemm_nt256(A, B, M, N, K, None, False, None, ref, 0)
    out = torch.empty(M, N, device=DEV)
    for v in (1, 4):  # (4: the 4-slot ring's counted waits)
        for _ in range(10):
            hipops().gemm_nt256(A, B, M, N, K, None, False, None, out, v)
            assert torch.equal(out, ref)


def test_gemm256_rejects_bad_k():
    A = torch.zeros(256, 100, dtype=torch.bfloat16, device=DEV)
    B = torch.zeros(256, 100, dtype=torch.bfloat16, device=DEV)
    with pytest.raises(ValueError):
        hipops().gemm_nt256(A, B, 256, 256, 100, None, False,
                            torch.empty(256, 256, dtype=torch.bfloat16, device=DEV), None)


def test_linear_forward_mfma_uses_256_tile_kernel():
    X = torch.randn(2048, 4992, device=DEV).to(torch.bfloat16)
    W = (torch.randn(1024, 4992, device=DEV) * 0.02).to(torch.bfloat16)
    b = torch.randn(1024, device=DEV)
    Z = GM.linear_forward(X, W, b, relu=True, backend="mfma")
    torch.testing.assert_close(Z.float(), _ref(X, W, b, True), rtol=2e-2, atol=3e-2)
