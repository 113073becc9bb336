// Sparse matrix x dense vector products for SparseMatrix (utils/matrix.py).
//
// Reference: SparseMatrix<I,V>::times / rangeTimes (src/util/sparse_matrix.h:73-130)
// walks the compressed major dimension on CPU threads; for a row-major matrix
// it reduces each row (y[r] = sum v*x[idx]); for a column-major matrix it scatters
// (y[idx] += v*x[c]) thread-locally. Here both storages map to two kernels:
//
//  * spmv_gather: a group of G lanes (G in 4..64, chosen on the host from the
//    average run length so a Criteo row of ~39 nnz uses 64 lanes and a 4-nnz row
//    uses 4) owns one major index, strides over its run with coalesced loads and
//    reduces with an xor butterfly inside the group; the G-lane groups pack a
//    wave64 densely, so short runs do not leave 60 of 64 lanes idle.
//  * spmv_scatter: the same lane groups, but each nnz is added into y with a
//    hardware float/double atomic (global_atomic_add_f32/f64 on gfx950).
//
// Index type int32 (localized, the common case — reference CHECKs localize
// happened before times) or int64; value type float or double; binary matrices
// pass val == nullptr (implicit 1). y = alpha * (A x) + beta * y.
#include "common.cuh"

namespace psamd {

namespace {

constexpr int kSpBlk = 256;

template <typename I, typename V, int G>
__global__ void __launch_bounds__(kSpBlk) spmv_gather_kernel(
    const int64_t* __restrict__ off, const I* __restrict__ idx, const V* __restrict__ val,
    int64_t n_major, int64_t nnz, const V* __restrict__ x, int64_t n_x, V alpha, V beta,
    V* __restrict__ y) {
  const int sub = threadIdx.x % G;
  const int64_t groups_per_grid = (int64_t)gridDim.x * (kSpBlk / G);
  for (int64_t r = (int64_t)blockIdx.x * (kSpBlk / G) + threadIdx.x / G; r < n_major;
       r += groups_per_grid) {
    const int64_t b = max(off[r], (int64_t)0), e = min(off[r + 1], nnz);  // clamp bad offsets
    V acc = 0;
    for (int64_t p = b + sub; p < e; p += G) {
      const int64_t c = (int64_t)idx[p];
      const V xv = in_range(c, n_x) ? x[c] : V(0);
      acc += val ? val[p] * xv : xv;
    }
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, G);
    if (sub == 0) y[r] = beta == V(0) ? alpha * acc : alpha * acc + beta * y[r];
  }
}

template <typename I, typename V, int G>
__global__ void __launch_bounds__(kSpBlk) spmv_scatter_kernel(
    const int64_t* __restrict__ off, const I* __restrict__ idx, const V* __restrict__ val,
    int64_t n_major, int64_t nnz, const V* __restrict__ x, V alpha, V* __restrict__ y,
    int64_t n_y) {
  const int sub = threadIdx.x % G;
  const int64_t groups_per_grid = (int64_t)gridDim.x * (kSpBlk / G);
  for (int64_t c = (int64_t)blockIdx.x * (kSpBlk / G) + threadIdx.x / G; c < n_major;
       c += groups_per_grid) {
    const V xc = alpha * x[c];
    if (xc == V(0)) continue;
    const int64_t b = max(off[c], (int64_t)0), e = min(off[c + 1], nnz);
    for (int64_t p = b + sub; p < e; p += G) {
      const int64_t r = (int64_t)idx[p];
      if (in_range(r, n_y)) unsafeAtomicAdd(&y[r], val ? val[p] * xc : xc);
    }
  }
}

__global__ void scale_kernel_f(float* y, int64_t n, float beta) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = beta == 0.f ? 0.f : y[i] * beta;
}
__global__ void scale_kernel_d(double* y, int64_t n, double beta) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    y[i] = beta == 0.0 ? 0.0 : y[i] * beta;
}
inline void scale(float* y, int64_t n, float b, hipStream_t st) {
  scale_kernel_f<<<grid_for(n, 256), 256, 0, st>>>(y, n, b);
}
inline void scale(double* y, int64_t n, double b, hipStream_t st) {
  scale_kernel_d<<<grid_for(n, 256), 256, 0, st>>>(y, n, b);
}

// Lanes per major index: smallest power of two >= the mean run length, in [4, 64].
inline int pick_group(int64_t nnz, int64_t n_major) {
  const int64_t avg = n_major > 0 ? (nnz + n_major - 1) / n_major : 1;
  int g = 4;
  while (g < 64 && g < avg) g <<= 1;
  return g;
}

template <typename I, typename V>
void gather_dispatch(const int64_t* off, const I* idx, const V* val, int64_t n_major, int64_t nnz,
                     const V* x, int64_t n_x, V alpha, V beta, V* y, hipStream_t st) {
  const int g = pick_group(nnz, n_major);
  const int grid = grid_for(n_major * g, kSpBlk, 8192);
#define PSAMD_SPMV_G(GG)                                                                  \
  case GG:                                                                                \
    spmv_gather_kernel<I, V, GG><<<grid, kSpBlk, 0, st>>>(off, idx, val, n_major, nnz, x, n_x, \
                                                          alpha, beta, y);                \
    break;
  switch (g) {
    PSAMD_SPMV_G(4) PSAMD_SPMV_G(8) PSAMD_SPMV_G(16) PSAMD_SPMV_G(32) default:
    PSAMD_SPMV_G(64)
  }
#undef PSAMD_SPMV_G
}

template <typename I, typename V>
void scatter_dispatch(const int64_t* off, const I* idx, const V* val, int64_t n_major, int64_t nnz,
                      const V* x, V alpha, V beta, V* y, int64_t n_y, hipStream_t st) {
  if (beta != V(1)) scale(y, n_y, beta, st);
  const int g = pick_group(nnz, n_major);
  const int grid = grid_for(n_major * g, kSpBlk, 8192);
#define PSAMD_SPMV_G(GG)                                                                     \
  case GG:                                                                                   \
    spmv_scatter_kernel<I, V, GG><<<grid, kSpBlk, 0, st>>>(off, idx, val, n_major, nnz, x, alpha, \
                                                           y, n_y);                          \
    break;
  switch (g) {
    PSAMD_SPMV_G(4) PSAMD_SPMV_G(8) PSAMD_SPMV_G(16) PSAMD_SPMV_G(32) default:
    PSAMD_SPMV_G(64)
  }
#undef PSAMD_SPMV_G
}

}  // namespace

// dtype codes: idx 4 = int32, 8 = int64; val 4 = float, 8 = double.
void spmv(bool scatter, const int64_t* off, const void* idx, int idx_bytes, const void* val,
          int val_bytes, int64_t n_major, int64_t nnz, const void* x, int64_t n_x, double alpha,
          double beta, void* y, int64_t n_y, hipStream_t st) {
  if (n_major <= 0) {
    if (scatter && val_bytes == 4) scale((float*)y, n_y, (float)beta, st);
    if (scatter && val_bytes == 8) scale((double*)y, n_y, beta, st);
    return;
  }
#define PSAMD_SPMV_CALL(I, V)                                                                  \
  if (scatter)                                                                                 \
    scatter_dispatch<I, V>(off, (const I*)idx, (const V*)val, n_major, nnz, (const V*)x,       \
                           (V)alpha, (V)beta, (V*)y, n_y, st);                                 \
  else                                                                                         \
    gather_dispatch<I, V>(off, (const I*)idx, (const V*)val, n_major, nnz, (const V*)x, n_x,   \
                          (V)alpha, (V)beta, (V*)y, st);
  if (idx_bytes == 4 && val_bytes == 4) {
    PSAMD_SPMV_CALL(int32_t, float)
  } else if (idx_bytes == 4) {
    PSAMD_SPMV_CALL(int32_t, double)
  } else if (val_bytes == 4) {
    PSAMD_SPMV_CALL(int64_t, float)
  } else {
    PSAMD_SPMV_CALL(int64_t, double)
  }
#undef PSAMD_SPMV_CALL
  PSAMD_HIP_CHECK(hipGetLastError());
}

}  // namespace psamd
