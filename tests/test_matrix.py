"""SparseMatrix / DenseMatrix (reference src/util/sparse_matrix.h, dense_matrix.h)
against dense fp64 PyTorch references, on CPU tensors."""
import numpy as np
import pytest
import torch

from parameter_server_amd.utils.matrix import DenseMatrix, SparseMatrix


def rand_sparse(rows, cols, density, seed, binary=False, dtype=torch.float64):
    g = torch.Generator().manual_seed(seed)
    mask = torch.rand(rows, cols, generator=g) < density
    a = torch.randn(rows, cols, generator=g, dtype=dtype) * mask
    if binary:
        a = mask.to(dtype)
    return a


@pytest.mark.parametrize("row_major", [True, False])
@pytest.mark.parametrize("binary", [False, True])
def test_times_and_trans_times(row_major, binary):
    a = rand_sparse(37, 53, 0.15, 1, binary)
    m = SparseMatrix.from_dense(a, row_major=row_major)
    if binary:
        m = SparseMatrix(m.offset, m.index, None, rows=37, cols=53, row_major=row_major)
    assert m.binary == binary and m.nnz == int((a != 0).sum())
    x = torch.randn(53, dtype=torch.float64)
    torch.testing.assert_close(m.times(x), a @ x)
    z = torch.randn(37, dtype=torch.float64)
    torch.testing.assert_close(m.trans_times(z), a.t() @ z)
    y0 = torch.randn(37, dtype=torch.float64)
    y = y0.clone()
    m.times(x, y, alpha=2.0, beta=0.5)
    torch.testing.assert_close(y, 2 * (a @ x) + 0.5 * y0)


def test_alter_storage_and_blocks():
    a = rand_sparse(40, 30, 0.2, 2)
    csr = SparseMatrix.from_dense(a, row_major=True)
    csc = csr.alter_storage()
    assert not csc.row_major and csc.nnz == csr.nnz
    torch.testing.assert_close(csc.to_dense(), a)
    torch.testing.assert_close(csc.alter_storage().to_dense(), a)
    # column block of the CSC shares the nnz arrays (absolute offsets)
    cb = csc.col_block(7, 19)
    assert cb.index.data_ptr() == csc.index.data_ptr()
    torch.testing.assert_close(cb.to_dense(), a[:, 7:19])
    x = torch.randn(12, dtype=torch.float64)
    torch.testing.assert_close(cb.times(x), a[:, 7:19] @ x)
    rb = csr.row_block(5, 22)
    torch.testing.assert_close(rb.to_dense(), a[5:22])
    torch.testing.assert_close(rb.times(torch.ones(30, dtype=torch.float64)), a[5:22].sum(1))
    with pytest.raises(ValueError):
        csr.col_block(1, 3)
    t = csr.trans()
    assert t.rows == 30 and t.cols == 40 and not t.row_major
    torch.testing.assert_close(t.to_dense(), a.t())


def test_dot_times_and_bin_file(tmp_path):
    a = rand_sparse(20, 25, 0.3, 3)
    m = SparseMatrix.from_dense(a)
    sq = m.dot_times(m)
    torch.testing.assert_close(sq.to_dense(), a * a)
    name = str(tmp_path / "mat")
    m.col_block(0, 25).write_to_bin_file(name)
    r = SparseMatrix.read_from_bin_file(name)
    assert r.info == m.info
    torch.testing.assert_close(r.to_dense(), a)
    # binary: no .value file
    b = SparseMatrix(m.offset, m.index, None, rows=20, cols=25)
    b.write_to_bin_file(name + "b")
    rb = SparseMatrix.read_from_bin_file(name + "b")
    assert rb.binary and torch.equal(rb.to_dense(), (a != 0).float())


def test_validation_and_from_batch():
    with pytest.raises(ValueError):
        SparseMatrix([0, 3, 2], [0, 1, 2], rows=2, cols=3)
    with pytest.raises(ValueError):
        SparseMatrix([0, 1], [0, 1], rows=2, cols=3)
    rp = np.array([0, 2, 5])
    m = SparseMatrix.from_batch(rp, np.array([0, 3, 1, 2, 3]), cols=4)
    torch.testing.assert_close(m.times(torch.arange(4.0)), torch.tensor([3.0, 6.0]))


def test_dense_matrix():
    a = torch.randn(6, 4, dtype=torch.float64)
    for rm in (True, False):
        d = DenseMatrix(a, row_major=rm)
        x = torch.randn(4, dtype=torch.float64)
        torch.testing.assert_close(d.times(x), a @ x)
        torch.testing.assert_close(d.trans().logical(), a.t())
        torch.testing.assert_close(d.alter_storage().logical(), a)
        assert d.alter_storage().row_major != rm
        torch.testing.assert_close(d.col_block(1, 3).logical(), a[:, 1:3])
        torch.testing.assert_close(d.row_block(2, 5).logical(), a[2:5])
