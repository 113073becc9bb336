"""bf16 MFMA GEMM (csrc/hip/gemm.hip) vs fp32 PyTorch of the same bf16 inputs."""
import pytest
import torch

from parameter_server_amd.ops import gemm as G
from parameter_server_amd.ops.native import hipops

pytestmark = pytest.mark.gpu


def _ref(A, ak, B, bk, M, N, K):
    a = (A.reshape(M, K) if ak else A.reshape(K, M).t()).float()
    b = (B.reshape(N, K) if bk else B.reshape(K, N).t()).float()
    return a @ b.t()


@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, False), (False, True)])
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (200, 136, 72), (1024, 512, 4992),
                                   (8, 8, 8), (4096, 1024, 256)])
def test_gemm_layouts_match_fp32(ak, bk, M, N, K):
    torch.manual_seed(M + N + K)
    A = torch.randn((M, K) if ak else (K, M), device="cuda").to(torch.bfloat16)
    B = torch.randn((N, K) if bk else (K, N), device="cuda").to(torch.bfloat16)
    C = G.gemm(A, ak, B, bk, M, N, K)
    ref = _ref(A, ak, B, bk, M, N, K)
    torch.testing.assert_close(C.float(), ref, rtol=1e-2, atol=2e-2 * K ** 0.5)
    Cf = torch.full((M, N), 3.0, device="cuda")
    G.gemm(A, ak, B, bk, M, N, K, out_bf16=False, out_f32=Cf, beta=0.5)
    torch.testing.assert_close(Cf, ref + 1.5, rtol=1e-4, atol=1e-3 * K ** 0.5)


@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_gemm_split_k(beta):
    torch.manual_seed(1)
    M, N, K = 256, 384, 8192
    A = torch.randn(K, M, device="cuda").to(torch.bfloat16)
    B = torch.randn(K, N, device="cuda").to(torch.bfloat16)
    Cf = torch.full((M, N), 2.0, device="cuda")
    G.gemm(A, False, B, False, M, N, K, out_bf16=False, out_f32=Cf, beta=beta, splitk=7)
    ref = _ref(A, False, B, False, M, N, K) + 2.0 * beta
    torch.testing.assert_close(Cf, ref, rtol=1e-4, atol=1e-2)


def test_gemm_asymmetric_identity():
    """A = I with an asymmetric B catches a transposed C-write (guide §3)."""
    M = N = K = 128
    A = torch.eye(M, device="cuda").to(torch.bfloat16)
    B = (torch.arange(N * K, device="cuda").reshape(N, K) % 97).to(torch.bfloat16)
    C = G.gemm(A, True, B, True, M, N, K)
    assert torch.equal(C.float(), B.float().t())


def test_linear_layer_products_and_epilogues():
    torch.manual_seed(0)
    Bn, K, N = 384, 4992, 1024
    X = torch.randn(Bn, K, device="cuda").to(torch.bfloat16)
    W = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    b = torch.randn(N, device="cuda")
    H = G.linear_forward(X, W, b, relu=True)
    ref = torch.relu(X.float() @ W.float().t() + b)
    torch.testing.assert_close(H.float(), ref, rtol=2e-2, atol=2e-2)
    dH = torch.randn(Bn, N, device="cuda").to(torch.bfloat16)
    dZ = G.gemm(dH, True, torch.eye(N, device="cuda").to(torch.bfloat16), True, Bn, N, N, mask=H)
    torch.testing.assert_close(dZ.float(), dH.float() * (H.float() > 0), rtol=0, atol=0)
    dX = G.linear_input_grad(dZ, W)
    torch.testing.assert_close(dX.float(), dZ.float() @ W.float(), rtol=2e-2, atol=2e-2)
    dW = G.linear_weight_grad(dZ, X)
    torch.testing.assert_close(dW, dZ.float().t() @ X.float(), rtol=1e-2, atol=5e-2)
    # CPU path = same math
    Hc = G.linear_forward(X.cpu(), W.cpu(), b.cpu(), relu=True)
    torch.testing.assert_close(Hc.float(), H.cpu().float(), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("M,N,K", [(384, 1024, 512), (200, 136, 72), (16384, 256, 512)])
def test_input_grad_colsum_epilogue(M, N, K):
    """EPI_COLSUM: the masked input gradient's column sums (bias gradient of the
    layer below) accumulate into colsum, equal to summing the bf16 output."""
    torch.manual_seed(M + N)
    dZ = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    W = (torch.randn(K, N, device="cuda") * 0.05).to(torch.bfloat16)
    mask = torch.relu(torch.randn(M, N, device="cuda")).to(torch.bfloat16)
    cs = torch.full((N,), 1.0, device="cuda")
    dX = G.linear_input_grad(dZ, W, mask=mask, colsum=cs)
    torch.testing.assert_close(cs - 1.0, dX.float().sum(0), rtol=1e-4, atol=1e-2)
    ref = (dZ.float() @ W.float()) * (mask.float() > 0)
    torch.testing.assert_close(dX.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("M,N,K,S,beta", [(256, 256, 512, 1, 0.0), (512, 1024, 4096, 7, 1.0),
                                          (1024, 4992, 2048, 3, 1.0), (264, 520, 1024, 2, 0.5),
                                          (256, 512, 16384, 32, 0.0)])
def test_gemm_tn256_weight_grad(M, N, K, S, beta):
    """TN 256x256 kernel (transposed LDS reads of MN-major operands, split-K partials with
    uneven splits, fixed-order reduce) against fp32: C = beta C + A^T B."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K + S)
    A = (torch.rand(K, M, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(K, N, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    C = torch.randn(M, N, device="cuda", generator=g)
    ref = A.float().t() @ B.float() + beta * C
    part = torch.full((S * M * N,), float("nan"), device="cuda")
    C0 = C.clone()
    hipops().gemm_tn256(A, B, M, N, K, S, part, C, beta)
    torch.testing.assert_close(C, ref, rtol=1e-4, atol=1e-3 * K ** 0.5)
    # the reduce inside the GEMM (phase 3: the last split of each tile sums the partials
    # in split order): bitwise the two-launch result, and the tile counters end zeroed
    ctr = torch.zeros(((M + 255) // 256) * ((N + 255) // 256), dtype=torch.int32, device="cuda")
    for _ in range(3):
        C3 = C0.clone()
        part.fill_(float("nan"))
        hipops().gemm_tn256(A, B, M, N, K, S, part, C3, beta, 3, ctr)
        assert torch.equal(C3, C)
        assert int(ctr.abs().sum()) == 0


def test_linear_weight_grad_routes_to_tn256():
    from parameter_server_amd.ops import gemm as GM

    torch.manual_seed(3)
    Bn, N, K = 4096, 512, 1024
    dZ = torch.randn(Bn, N, device="cuda").to(torch.bfloat16)
    X = torch.randn(Bn, K, device="cuda").to(torch.bfloat16)
    assert GM.tn256_ok(N, K, Bn)
    out = torch.ones(N, K, device="cuda")
    GM.linear_weight_grad(dZ, X, out=out, beta=1.0, backend="mfma")
    ref = dZ.float().t() @ X.float() + 1.0
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-3 * Bn ** 0.5)
    out2 = torch.ones(N, K, device="cuda")
    GM.linear_weight_grad(dZ, X, out=out2, beta=1.0, backend="mfma")
    assert torch.equal(out, out2)  # fixed-order split-K sum


@pytest.mark.parametrize("R,C", [(64, 64), (1024, 4992), (192, 640)])
def test_transpose_bf16(R, C):
    x = torch.randn(R, C, device="cuda").to(torch.bfloat16)
    y = torch.empty(C, R, dtype=torch.bfloat16, device="cuda")
    hipops().transpose_bf16(x, y)
    assert torch.equal(y, x.t().contiguous())
