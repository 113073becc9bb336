"""Sparse / dense matrices (reference src/util/matrix.h, sparse_matrix.h, dense_matrix.h).

The reference's ``Matrix<V>`` family is the CPU container the Darlin app reads
its training data into (``SlotReader`` -> ``SparseMatrix<uint32,V>``) and the
one its gradient path multiplies with (``times`` / ``trans``, sparse_matrix.h:
33-130). Here a matrix is a set of torch tensors that live on the CPU or in HBM;
products on a GPU tensor run the HIP kernels in ``csrc/hip/spmv.hip``
(lane-group gather for a row-reduce, hardware float/double atomics for a
scatter), products on CPU tensors use torch's ``index_add_`` / segment sums.

Layout (Yale/CSR-or-CSC, reference sparse_matrix.h:22-31):
* ``offset`` int64 [outer+1]  — ABSOLUTE positions into ``index``/``value``, so a
  column/row block is a view that shares the nnz arrays (reference colBlock /
  rowBlock, sparse_matrix.h:152-182);
* ``index`` int32 (localized) or int64 [nnz];
* ``value`` float32/float64 [nnz], or ``None`` for SPARSE_BINARY.

``MatrixInfo`` (reference proto/matrix.proto) is a small dataclass; binary
files follow writeToBinFile (sparse_matrix.h:48-53): ``name.info`` (JSON instead
of a text proto), ``name.offset``, ``name.index``, ``name.value`` raw arrays.
"""
from __future__ import annotations

import json
from dataclasses import asdict, dataclass, replace

import numpy as np
import torch

from ..ops.native import hipops, is_gpu

DENSE, SPARSE, SPARSE_BINARY = 1, 2, 3


@dataclass
class MatrixInfo:
    type: int = SPARSE
    row_major: bool = True
    row: tuple = (0, 0)   # [begin, end) of the global row range
    col: tuple = (0, 0)   # [begin, end) of the global column range
    nnz: int = 0
    sizeof_index: int = 4
    sizeof_value: int = 4

    @property
    def rows(self) -> int:
        return self.row[1] - self.row[0]

    @property
    def cols(self) -> int:
        return self.col[1] - self.col[0]


class Matrix:
    """Common interface (reference matrix.h:27-128)."""

    info: MatrixInfo

    @property
    def rows(self) -> int:
        return self.info.rows

    @property
    def cols(self) -> int:
        return self.info.cols

    @property
    def row_major(self) -> bool:
        return self.info.row_major

    @property
    def nnz(self) -> int:
        return self.info.nnz

    @property
    def outer_size(self) -> int:
        return self.rows if self.row_major else self.cols

    @property
    def inner_size(self) -> int:
        return self.cols if self.row_major else self.rows

    def empty(self) -> bool:
        return self.nnz == 0

    def debug_string(self) -> str:
        return f"{type(self).__name__}({asdict(self.info)})"

    __repr__ = debug_string


class SparseMatrix(Matrix):
    def __init__(self, offset, index, value=None, *, rows: int, cols: int, row_major=True,
                 row0: int = 0, col0: int = 0, validate: bool = True):
        self.offset = torch.as_tensor(offset, dtype=torch.int64)
        self.index = torch.as_tensor(index)
        if self.index.dtype not in (torch.int32, torch.int64):
            self.index = self.index.to(torch.int64)
        self.value = None if value is None else torch.as_tensor(value)
        if self.value is not None and self.value.dtype not in (torch.float32, torch.float64):
            self.value = self.value.to(torch.float32)
        outer = rows if row_major else cols
        if self.offset.numel() != outer + 1:
            raise ValueError(f"offset has {self.offset.numel()} entries, expected {outer + 1}")
        if self.value is not None and self.value.numel() != self.index.numel():
            raise ValueError("value / index length mismatch")
        if validate and outer > 0:
            o = self.offset.cpu()
            if bool((o[1:] < o[:-1]).any()) or int(o[0]) < 0 or int(o[-1]) > self.index.numel():
                raise ValueError("offset must be non-decreasing within [0, nnz]")
        nnz = int(self.offset[-1] - self.offset[0]) if outer > 0 else 0
        self.info = MatrixInfo(
            type=SPARSE_BINARY if self.value is None else SPARSE, row_major=row_major,
            row=(row0, row0 + rows), col=(col0, col0 + cols), nnz=nnz,
            sizeof_index=self.index.element_size(),
            sizeof_value=0 if self.value is None else self.value.element_size())

    # ---------------------------------------------------------------- builders
    @classmethod
    def from_coo(cls, row, col, value=None, *, rows: int, cols: int, row_major=True,
                 index_dtype=torch.int32, device=None):
        """Build CSR (row_major) or CSC from COO triplets (any order)."""
        row = torch.as_tensor(row, dtype=torch.int64, device=device)
        col = torch.as_tensor(col, dtype=torch.int64, device=device)
        major, minor = (row, col) if row_major else (col, row)
        outer = rows if row_major else cols
        order = torch.sort(major * max(1, (cols if row_major else rows)) + minor, stable=True)[1]
        counts = torch.bincount(major, minlength=outer)
        offset = torch.zeros(outer + 1, dtype=torch.int64, device=major.device)
        offset[1:] = torch.cumsum(counts, 0)
        v = None if value is None else torch.as_tensor(value, device=major.device)[order]
        return cls(offset, minor[order].to(index_dtype), v, rows=rows, cols=cols,
                   row_major=row_major)

    @classmethod
    def from_dense(cls, a, row_major=True, index_dtype=torch.int32):
        a = torch.as_tensor(a)
        r, c = torch.nonzero(a, as_tuple=True)
        return cls.from_coo(r, c, a[r, c], rows=a.shape[0], cols=a.shape[1],
                            row_major=row_major, index_dtype=index_dtype, device=a.device)

    @classmethod
    def from_batch(cls, row_ptr, keys, vals=None, *, cols: int, index_dtype=torch.int32):
        """A localized CSR minibatch (data.ExampleBatch row_ptr / local ids)."""
        rp = torch.as_tensor(row_ptr, dtype=torch.int64)
        return cls(rp, torch.as_tensor(keys).to(index_dtype), vals, rows=rp.numel() - 1,
                   cols=cols, row_major=True)

    def to(self, device) -> "SparseMatrix":
        out = SparseMatrix.__new__(SparseMatrix)
        out.offset = self.offset.to(device)
        out.index = self.index.to(device)
        out.value = None if self.value is None else self.value.to(device)
        out.info = replace(self.info)
        return out

    @property
    def device(self):
        return self.index.device

    @property
    def binary(self) -> bool:
        return self.info.type == SPARSE_BINARY

    def mem_size(self) -> int:
        v = 0 if self.value is None else self.value.numel() * self.value.element_size()
        return v + self.index.numel() * self.index.element_size() + self.offset.numel() * 8

    # -------------------------------------------------------------- structure
    def _view(self, offset, info) -> "SparseMatrix":
        out = SparseMatrix.__new__(SparseMatrix)
        out.offset, out.index, out.value, out.info = offset, self.index, self.value, info
        return out

    def trans(self) -> "SparseMatrix":
        """Transpose without copying: flip the storage order and swap the ranges
        (reference trans / tranposeInfo, sparse_matrix.h:37-41)."""
        return self._view(self.offset, replace(self.info, row_major=not self.row_major,
                                               row=self.info.col, col=self.info.row))

    def row_block(self, begin: int, end: int) -> "SparseMatrix":
        """Rows [begin, end) (local numbering) of a row-major matrix (sparse_matrix.h:170-182)."""
        if not self.row_major:
            raise ValueError("row_block needs a row-major matrix")
        off = self.offset[begin:end + 1]
        r0 = self.info.row[0]
        return self._view(off, replace(self.info, row=(r0 + begin, r0 + end),
                                       nnz=int(off[-1] - off[0]) if end > begin else 0))

    def col_block(self, begin: int, end: int) -> "SparseMatrix":
        """Columns [begin, end) of a column-major matrix (sparse_matrix.h:152-168); a
        row-major matrix only supports the full range, like the reference."""
        if self.row_major:
            if (begin, end) != (0, self.cols):
                raise ValueError("col_block on a row-major matrix needs the full column range")
            return self._view(self.offset, replace(self.info))
        off = self.offset[begin:end + 1]
        c0 = self.info.col[0]
        return self._view(off, replace(self.info, col=(c0 + begin, c0 + end),
                                       nnz=int(off[-1] - off[0]) if end > begin else 0))

    def _major_ids(self) -> torch.Tensor:
        counts = self.offset[1:] - self.offset[:-1]
        return torch.repeat_interleave(
            torch.arange(self.outer_size, device=self.offset.device), counts)

    def _compact(self):
        """(offset rebased to 0, index, value) restricted to this view's nnz range."""
        p0, p1 = int(self.offset[0]), int(self.offset[-1])
        v = None if self.value is None else self.value[p0:p1]
        return self.offset - p0, self.index[p0:p1], v

    def alter_storage(self) -> "SparseMatrix":
        """CSR <-> CSC with the same logical matrix (sparse_matrix.h:185-241)."""
        off, idx, val = self._compact()
        inner = self.inner_size
        major = torch.repeat_interleave(torch.arange(self.outer_size, device=off.device),
                                        off[1:] - off[:-1])
        order = torch.sort(idx.to(torch.int64), stable=True)[1]
        counts = torch.bincount(idx.to(torch.int64), minlength=inner)
        new_off = torch.zeros(inner + 1, dtype=torch.int64, device=off.device)
        new_off[1:] = torch.cumsum(counts, 0)
        out = SparseMatrix(new_off, major[order].to(self.index.dtype),
                           None if val is None else val[order], rows=self.rows, cols=self.cols,
                           row_major=not self.row_major, row0=self.info.row[0],
                           col0=self.info.col[0], validate=False)
        return out

    def dot_times(self, other: "SparseMatrix") -> "SparseMatrix":
        """Element-wise product with a matrix of identical structure (sparse_matrix.h:132-150)."""
        if (self.rows, self.cols, self.nnz) != (other.rows, other.cols, other.nnz):
            raise ValueError("dot_times needs matrices of the same shape and nnz")
        a = self.value if self.value is not None else None
        b = other.value if other.value is not None else None
        if a is None and b is None:
            return self._view(self.offset, replace(self.info))
        v = b if a is None else (a if b is None else a * b)
        out = self._view(self.offset, replace(self.info, type=SPARSE,
                                              sizeof_value=v.element_size()))
        out.value = v
        return out

    def to_dense(self) -> torch.Tensor:
        off, idx, val = self._compact()
        dt = torch.float32 if val is None else val.dtype
        d = torch.zeros(self.outer_size, self.inner_size, dtype=dt, device=off.device)
        major = torch.repeat_interleave(torch.arange(self.outer_size, device=off.device),
                                        off[1:] - off[:-1])
        d.index_put_((major, idx.to(torch.int64)),
                     torch.ones_like(major, dtype=dt) if val is None else val, accumulate=True)
        return d if self.row_major else d.t().contiguous()

    # ---------------------------------------------------------------- products
    def times(self, x, y=None, *, alpha: float = 1.0, beta: float = 0.0) -> torch.Tensor:
        """y = alpha * A x + beta * y (reference times / templateTimes)."""
        x = torch.as_tensor(x)
        if x.numel() != self.cols:
            raise ValueError(f"x has {x.numel()} entries, matrix has {self.cols} columns")
        dt = x.dtype if x.dtype in (torch.float32, torch.float64) else torch.float32
        x = x.to(dt).contiguous()
        if self.value is not None and self.value.dtype != dt:
            raise ValueError("x dtype must match the matrix value dtype")
        if y is None:
            y = torch.zeros(self.rows, dtype=dt, device=x.device)
            beta = 0.0
        if y.numel() != self.rows or y.dtype != dt:
            raise ValueError("y must be [rows] with the dtype of x")
        if is_gpu(x):
            hipops().spmv(not self.row_major, self.offset, self.index, self.value, x, y,
                          float(alpha), float(beta))
            return y
        off, idx, val = self._compact()
        major = torch.repeat_interleave(torch.arange(self.outer_size), off[1:] - off[:-1])
        idx = idx.to(torch.int64)
        if self.row_major:
            contrib = x[idx] if val is None else x[idx] * val
            ax = torch.zeros(self.rows, dtype=dt).index_add_(0, major, contrib)
        else:
            contrib = x[major] if val is None else x[major] * val
            ax = torch.zeros(self.rows, dtype=dt).index_add_(0, idx, contrib)
        if beta == 0.0:
            y.copy_(alpha * ax)
        else:
            y.mul_(beta).add_(alpha * ax)
        return y

    def trans_times(self, x, y=None, **kw) -> torch.Tensor:
        """y = A^T x without materialising the transpose."""
        return self.trans().times(x, y, **kw)

    # ---------------------------------------------------------------- file io
    def write_to_bin_file(self, name: str) -> None:
        info = asdict(self.info)
        info["index_dtype"] = str(self.index.dtype).replace("torch.", "")
        info["value_dtype"] = None if self.value is None else str(self.value.dtype).replace(
            "torch.", "")
        off, idx, val = self._compact()
        with open(name + ".info", "w") as f:
            json.dump(info, f)
        off.cpu().numpy().tofile(name + ".offset")
        idx.cpu().numpy().tofile(name + ".index")
        if val is not None:
            val.cpu().numpy().tofile(name + ".value")

    @classmethod
    def read_from_bin_file(cls, name: str, device=None) -> "SparseMatrix":
        with open(name + ".info") as f:
            info = json.load(f)
        off = np.fromfile(name + ".offset", dtype=np.int64)
        idx = np.fromfile(name + ".index", dtype=np.dtype(info["index_dtype"]))
        val = None
        if info.get("value_dtype"):
            val = torch.from_numpy(np.fromfile(name + ".value", dtype=np.dtype(info["value_dtype"])))
        rows, cols = info["row"][1] - info["row"][0], info["col"][1] - info["col"][0]
        m = cls(torch.from_numpy(off), torch.from_numpy(idx), val, rows=rows, cols=cols,
                row_major=info["row_major"], row0=info["row"][0], col0=info["col"][0])
        return m if device is None else m.to(device)


class DenseMatrix(Matrix):
    """Row- or column-major dense block (reference dense_matrix.h); ``times`` is a
    GEMV (the reference CHECK-fails here; it is cheap to support)."""

    def __init__(self, value, row_major: bool = True):
        v = torch.as_tensor(value)
        if v.dim() != 2:
            raise ValueError("DenseMatrix needs a 2-D tensor")
        self.value = v.contiguous() if row_major else v.t().contiguous()
        rows, cols = v.shape
        self.info = MatrixInfo(type=DENSE, row_major=row_major, row=(0, rows), col=(0, cols),
                               nnz=rows * cols, sizeof_index=0, sizeof_value=v.element_size())

    def logical(self) -> torch.Tensor:
        return self.value if self.row_major else self.value.t()

    def times(self, x, y=None) -> torch.Tensor:
        r = self.logical() @ torch.as_tensor(x).to(self.value.dtype)
        if y is None:
            return r
        y.copy_(r)
        return y

    def trans(self) -> "DenseMatrix":
        return DenseMatrix(self.logical().t(), row_major=not self.row_major)

    def alter_storage(self) -> "DenseMatrix":
        return DenseMatrix(self.logical(), row_major=not self.row_major)

    def row_block(self, begin: int, end: int) -> "DenseMatrix":
        return DenseMatrix(self.logical()[begin:end], row_major=self.row_major)

    def col_block(self, begin: int, end: int) -> "DenseMatrix":
        return DenseMatrix(self.logical()[:, begin:end], row_major=self.row_major)

    def mem_size(self) -> int:
        return self.value.numel() * self.value.element_size()
