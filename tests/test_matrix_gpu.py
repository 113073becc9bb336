"""HIP SpMV (csrc/hip/spmv.hip) behind SparseMatrix.times on the GPU, against a
plain fp64 PyTorch reference of the same product."""
import pytest
import torch

from parameter_server_amd.utils.matrix import SparseMatrix

pytestmark = pytest.mark.gpu


def _mat(rows, cols, density, seed, dtype):
    g = torch.Generator().manual_seed(seed)
    mask = torch.rand(rows, cols, generator=g) < density
    a = (torch.randn(rows, cols, generator=g, dtype=torch.float64) * mask)
    # a few long rows / columns and empty ones to exercise every lane-group width
    a[0, :] = torch.randn(cols, generator=g, dtype=torch.float64)
    a[rows // 2, :] = 0
    return a.to(dtype).to(torch.float64), a.to(dtype)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("index_dtype", [torch.int32, torch.int64])
@pytest.mark.parametrize("density", [0.002, 0.03, 0.2, 0.9])
@pytest.mark.parametrize("row_major", [True, False])
def test_spmv_matches_fp64(dtype, index_dtype, density, row_major):
    rows, cols = 3001, 1703
    ref, a = _mat(rows, cols, density, 7, dtype)
    m = SparseMatrix.from_dense(a, row_major=row_major, index_dtype=index_dtype).to("cuda")
    x = torch.randn(cols, dtype=torch.float64)
    z = torch.randn(rows, dtype=torch.float64)
    tol = dict(rtol=1e-4, atol=1e-3) if dtype == torch.float32 else dict(rtol=1e-10, atol=1e-10)
    y = m.times(x.to(dtype).cuda())
    torch.testing.assert_close(y.double().cpu(), ref @ x.to(dtype).double(), **tol)
    yt = m.trans_times(z.to(dtype).cuda())
    torch.testing.assert_close(yt.double().cpu(), ref.t() @ z.to(dtype).double(), **tol)
    y0 = torch.randn(rows, dtype=dtype, device="cuda")
    y1 = y0.clone()
    m.times(x.to(dtype).cuda(), y1, alpha=-1.5, beta=0.25)
    torch.testing.assert_close(y1.double().cpu(),
                               -1.5 * (ref @ x.to(dtype).double()) + 0.25 * y0.double().cpu(),
                               **tol)


def test_spmv_binary_and_blocks():
    rows, cols = 5000, 900
    _, a = _mat(rows, cols, 0.05, 3, torch.float32)
    b = (a != 0).float()
    csr = SparseMatrix.from_dense(b).to("cuda")
    csr = SparseMatrix(csr.offset, csr.index, None, rows=rows, cols=cols)
    assert csr.binary
    x = torch.randn(cols, device="cuda")
    torch.testing.assert_close(csr.times(x).cpu(), b @ x.cpu(), rtol=1e-4, atol=1e-3)
    csc = csr.alter_storage()
    assert csc.device.type == "cuda" and not csc.row_major
    torch.testing.assert_close(csc.times(x).cpu(), b @ x.cpu(), rtol=1e-4, atol=1e-3)
    blk = csc.col_block(100, 700)
    xb = torch.randn(600, device="cuda")
    torch.testing.assert_close(blk.times(xb).cpu(), b[:, 100:700] @ xb.cpu(), rtol=1e-4,
                               atol=1e-3)
    rb = csr.row_block(1000, 3000)
    torch.testing.assert_close(rb.times(x).cpu(), b[1000:3000] @ x.cpu(), rtol=1e-4, atol=1e-3)


def test_spmv_rejects_bad_shapes():
    m = SparseMatrix.from_dense(torch.eye(4)).to("cuda")
    with pytest.raises(ValueError):
        m.times(torch.ones(5, device="cuda"))
    with pytest.raises(ValueError):
        m.times(torch.ones(4, device="cuda", dtype=torch.float64))


def test_sarray_on_gpu_matches_cpu():
    import numpy as np

    from parameter_server_amd.utils import sarray

    rng = np.random.default_rng(5)
    dst = np.unique(rng.integers(0, 1 << 62, 100_000, dtype=np.uint64))
    src = np.unique(np.concatenate([dst[::7], rng.integers(0, 1 << 62, 1000, dtype=np.uint64)]))
    sv = rng.standard_normal(src.size * 2).astype(np.float32)
    want, nw = sarray.ordered_match(src, sv, dst, 2, "PLUS")
    t = lambda a: torch.from_numpy(a.view(np.int64)).cuda()  # noqa: E731
    got, ng = sarray.ordered_match(t(src), torch.from_numpy(sv).cuda(), t(dst), 2, "PLUS")
    assert nw == ng
    torch.testing.assert_close(got.cpu(), torch.from_numpy(want))
    u = sarray.set_union(t(dst[:500]), t(src[:500]))
    assert np.array_equal(u.cpu().numpy().view(np.uint64),
                          np.union1d(dst[:500].view(np.int64), src[:500].view(np.int64)).view(np.uint64))
