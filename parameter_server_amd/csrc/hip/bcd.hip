// Darlin block coordinate descent (L1-regularised logistic regression) on CDNA4.
//
// Reference hot loops (CPU, std::thread pools) this file replaces:
//   K11 worker block gradient G_j, U_j       src/app/linear_method/darlin.h:381-427
//   K13 server coordinate update + KKT filter + trust region
//                                             src/app/linear_method/darlin.h:206-246
//   K12 worker dual update dual_i *= exp(y_i dw_j x_ij)
//                                             src/app/linear_method/darlin.h:472-502
//   objective sum log(1 + 1/dual_i)           src/app/linear_method/darlin.h:504-511
//
// MI355X design:
//  * the training matrix of a rank is one CSC over the GLOBAL column space of a
//    feature group (columns = filtered keys, sorted); a feature block is a
//    contiguous column range [c0, c1) == contiguous nnz range [p0, p1).
//  * the reference keeps dual_i = exp(y_i x_i.w) and multiplies it; here the
//    margin ym_i = y_i x_i.w is kept in fp64 and updated additively with the
//    hardware fp64 global atomic add (log-space version of the same update; no
//    overflow of exp for large margins). tau_i = 1 / (1 + exp(ym_i)).
//  * the gradient is an nnz-parallel segmented reduction by column inside each
//    wave64 (Hillis-Steele over 64 lanes, fp64): columns that start and end
//    inside a wave are written with a plain store, only wave-spanning (head)
//    columns use atomics -> no per-column wave imbalance for power-law columns.
//  * every rank applies the (deterministic) server update to a replicated copy
//    of the block after an all-reduce of (G, U); there is no pull phase.
#include "common.cuh"

#include <algorithm>
#include <cmath>
#include <stdexcept>

namespace psamd {

namespace {

constexpr int kPartSeg = 16;  // segments of the row pass's two-stage partial reduce

__device__ __forceinline__ double softplus_neg(double m) {  // log(1 + exp(-m))
  return m > 0 ? log1p(exp(-m)) : -m + log1p(exp(m));
}

__device__ __forceinline__ double shfl_up_d(double v, int off) {
  return __shfl_up(v, off, 64);
}

// K11 -------------------------------------------------------------------------
// G[c - c0] = -sum_i y_i tau_i x_ic
// U[c - c0] =  sum_i min(tau_i (1 - tau_i) exp(|x_ic| delta_c), .25) x_ic^2
// (binary: x = 1 and the exp factor is exp(delta_c), darlin.h:408-418).
__global__ void __launch_bounds__(256)
bcd_grad_kernel(const int32_t* __restrict__ col, const int32_t* __restrict__ row,
                const float* __restrict__ val, int64_t p0, int64_t p1, int64_t c0, int64_t ncols,
                const double* __restrict__ ym, const float* __restrict__ y, int64_t nrows,
                const double* __restrict__ delta, const uint8_t* __restrict__ active,
                double* __restrict__ G, double* __restrict__ U) {
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = p0 + blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~63); i0 < p1;
       i0 += stride) {
    const int64_t i = i0 + lane;
    const bool valid = i < p1;
    int64_t c = -1;
    double g = 0, u = 0;
    if (valid) {
      c = (int64_t)col[i] - c0;
      if (c >= 0 && c < ncols && active[c0 + c]) {
        const int32_t r = row[i];
        if (in_range(r, nrows)) {
          const double tau = 1.0 / (1.0 + exp(ym[r]));
          const double yr = (double)y[r];
          const double t2 = tau * (1.0 - tau);
          const double dl = delta[c0 + c];
          if (val) {
            const double v = (double)val[i];
            g = -yr * tau * v;
            u = fmin(t2 * exp(fabs(v) * dl), 0.25) * v * v;
          } else {
            g = -yr * tau;
            u = fmin(t2 * exp(dl), 0.25);
          }
        }
      } else if (c < 0 || c >= ncols) {
        c = -1;  // out-of-block element (corrupt input): contributes nothing
      }
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const double go = shfl_up_d(g, off);
      const double uo = shfl_up_d(u, off);
      const int64_t co = __shfl_up(c, off, 64);
      if (lane >= off && co == c) { g += go; u += uo; }
    }
    const int64_t c_next = __shfl_down(c, 1, 64);
    const int64_t c_lane0 = __shfl(c, 0, 64);
    int64_t prev0 = -2;
    if (lane == 0 && i0 > p0) prev0 = (int64_t)col[i0 - 1] - c0;
    prev0 = __shfl(prev0, 0, 64);
    const bool tail = valid && c >= 0 && (lane == 63 || c_next != c || i + 1 >= p1);
    if (tail) {
      const bool starts_inside = (c != c_lane0) || (prev0 != c);
      bool ends_inside = true;
      if (lane == 63 && i + 1 < p1) ends_inside = ((int64_t)col[i + 1] - c0) != c;
      if (starts_inside && ends_inside) {
        G[c] = g;
        U[c] = u;
      } else {
        unsafeAtomicAdd(&G[c], g);
        unsafeAtomicAdd(&U[c], u);
      }
    }
  }
}

// K13 -------------------------------------------------------------------------
// Per-coordinate proximal Newton step with trust region and KKT filter
// (darlin.h:206-246). dw receives the applied change (0 if inactive; filtered: 0, or
// NaN with nan_filtered = the reference server's NaN mark, darlin.h:228-231, which
// tells the replicas of a sharded server to drop the column from their active set).
// Violation is max-reduced as the bit pattern of a non-negative double.
// the coordinate step of one active column k (bcd_update_kernel, and the fused update at
// the end of a small narrow block's row-order gradient)
// (wk / dk: w[k] / delta[k], loaded by the caller)
__device__ __forceinline__ double bcd_update_col(int64_t k, double gj, double uj, double wk,
                                                 double dk, double* __restrict__ w,
                                                 double* __restrict__ delta,
                                                 uint8_t* __restrict__ active, double eta,
                                                 double lambda, double delta_max, double kkt_thr,
                                                 int nan_filtered, double& vmax) {
  double d = 0;
  const double g = gj, u = uj / eta + 1e-10;
  const double gp = g + lambda, gn = g - lambda;
  double vio = 0;
  bool filtered = false;
  if (wk == 0) {
    if (gp < 0) vio = -gp;
    else if (gn > 0) vio = gn;
    else if (gp > kkt_thr && gn < -kkt_thr) filtered = true;
  }
  if (filtered) {
    active[k] = 0;
    if (nan_filtered) d = __builtin_nan("");
  } else {
    vmax = fmax(vmax, vio);
    d = -wk;
    if (gp <= u * wk) d = -gp / u;
    else if (gn >= u * wk) d = -gn / u;
    d = fmin(dk, fmax(-dk, d));
    delta[k] = fmin(delta_max, 2 * fabs(d) + .1);
    w[k] = wk + d;
  }
  return d;
}

// wave max -> one atomic per wave (violation as the bits of a non-negative double)
__device__ __forceinline__ void bcd_vio_max(double vmax, unsigned long long* vio_bits) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) vmax = fmax(vmax, __shfl_xor(vmax, off, 64));
  if ((threadIdx.x & 63) == 0 && vmax > 0)
    atomicMax(vio_bits, (unsigned long long)__double_as_longlong(vmax));
}

__global__ void __launch_bounds__(256)
bcd_update_kernel(int64_t c0, int64_t ncols, double* __restrict__ G, double* __restrict__ U,
                  double* __restrict__ w, double* __restrict__ delta,
                  uint8_t* __restrict__ active, double* __restrict__ dw, double eta, double lambda,
                  double delta_max, double kkt_thr, unsigned long long* __restrict__ vio_bits,
                  int consume, int nan_filtered, const long long* __restrict__ part2, int k2) {
  double vmax = 0;
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < ncols;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = c0 + j;
    double d = 0;
    double gj, uj;
    if (part2) {  // a narrow row pass's segment sums (bcd_part_reduce2's arithmetic)
      long long sg = 0, su = 0;
#pragma unroll
      for (int q = 0; q < kPartSeg; ++q) {
        sg += part2[(int64_t)q * 2 * ncols + j];
        su += part2[(int64_t)q * 2 * ncols + ncols + j];
      }
      gj = (double)sg * ldexp(1.0, -k2);
      uj = (double)su * ldexp(1.0, -k2);
    } else {
      gj = G[j];
      uj = U[j];
    }
    if (consume && !part2) {  // leave G / U zeroed for the block's next gradient (no memsets)
      G[j] = 0;
      U[j] = 0;
    }
    if (active[k]) d = bcd_update_col(k, gj, uj, w[k], delta[k], w, delta, active, eta, lambda,
                                      delta_max, kkt_thr, nan_filtered, vmax);
    dw[j] = d;
  }
  bcd_vio_max(vmax, vio_bits);
}

// Sharded server, replica side: the owners' updates of a block arrive as one
// all-gathered dw (NaN = KKT-filtered). Every rank replays them on its replica of
// w / delta / active outside its own slice [own0, own1) with the owner's exact
// arithmetic (the replicas stay bitwise equal), and turns NaN marks into 0 for the
// dual update.
__global__ void __launch_bounds__(256)
bcd_replica_kernel(int64_t c0, int64_t ncols, int64_t own0, int64_t own1, double* __restrict__ dw,
                   double* __restrict__ w, double* __restrict__ delta,
                   uint8_t* __restrict__ active, double delta_max) {
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < ncols;
       j += (int64_t)gridDim.x * blockDim.x) {
    const double d = dw[j];
    const bool mine = j >= own0 && j < own1;
    if (d != d) {
      dw[j] = 0;
      if (!mine) active[c0 + j] = 0;
    } else if (!mine && active[c0 + j]) {
      const int64_t k = c0 + j;
      delta[k] = fmin(delta_max, 2 * fabs(d) + .1);
      w[k] = w[k] + d;
    }
  }
}

// K12 -------------------------------------------------------------------------
// ym_i += y_i * dw_c * x_ic for every nnz of the block with dw_c != 0.
// kUnique: every row occurs at most once in the block's range (one key per example
// and feature group, the Criteo / TERAFEA slot layout; checked at preprocessing), so
// the update is a plain read-modify-write of ym (no fp64 atomics); otherwise one
// atomic per entry (rows sorted within the block: coalesced, uncontended).
template <bool kUnique>
__global__ void __launch_bounds__(256)
bcd_dual_kernel(const int32_t* __restrict__ col, const int32_t* __restrict__ row,
                const float* __restrict__ val, int64_t p0, int64_t p1, int64_t c0, int64_t ncols,
                const double* __restrict__ dw, const float* __restrict__ y, double* __restrict__ ym,
                int64_t nrows) {
  // kR entries per thread per round with their loads in flight together (entry ->
  // dw[col] and entry -> row -> y / ym are dependent chains)
  constexpr int kR = 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = p0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i0 < p1;
       i0 += (int64_t)kR * stride) {
    int64_t cc[kR];
    int32_t rr[kR];
#pragma unroll
    for (int q = 0; q < kR; ++q) {
      const int64_t i = i0 + q * stride;
      cc[q] = -1;
      rr[q] = -1;
      if (i < p1) {
        const int64_t c = (int64_t)col[i] - c0;
        cc[q] = (c >= 0 && c < ncols) ? c : -1;
        rr[q] = row[i];
      }
    }
    double d[kR];
#pragma unroll
    for (int q = 0; q < kR; ++q) {
      d[q] = (cc[q] >= 0 && in_range(rr[q], nrows)) ? dw[cc[q]] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < kR; ++q) {
      if (d[q] == 0) continue;
      const int32_t r = rr[q];
      const double x = val ? (double)val[i0 + q * stride] : 1.0;
      if (kUnique) ym[r] += (double)y[r] * d[q] * x;
      else unsafeAtomicAdd(&ym[r], (double)y[r] * d[q] * x);
    }
  }
}

// K11, load-balanced: the block's CSC range is cut ONCE on the host (the matrix
// does not change between passes) into chunks of two kinds, one wavefront each:
//  * small: whole columns of <= 64 entries packed into <= 64 entries: the in-wave
//    segmented scan above, every column stored with a plain store;
//  * hot: <= kHotChunk entries of ONE column (> 64 entries): lanes accumulate
//    their strided entries (independent iterations, loads in flight), one wave
//    sum, one fp64 atomic per chunk.
// The flat kernel above sends one atomic per 64 entries of a wave-spanning
// column: a column present in every example (4 M entries) serialises ~62 k
// same-address fp64 atomics (~1.5 ms for the block); here it is 4 M / 4096.
// Measured and not kept (5.55 ms/pass, 4 M rows): interleaving {ym, y} per row
// for the random row gather (5.55, no change: the rows live in L2 / MALL) and
// forcing 8 waves/SIMD with __launch_bounds__(256, 8) (6.33: 12 VGPRs spill).
constexpr int64_t kHotBit = int64_t(1) << 62;
constexpr int64_t kSkipBit = int64_t(1) << 61;

__device__ __forceinline__ void bcd_gu(int64_t i, int64_t c, int64_t c0,
                                       const int32_t* __restrict__ row,
                                       const float* __restrict__ val,
                                       const double* __restrict__ ym, const float* __restrict__ y,
                                       int64_t nrows, double dl, double& g, double& u) {
  const int32_t r = row[i];
  if (!in_range(r, nrows)) return;
  const double tau = 1.0 / (1.0 + exp(ym[r]));
  const double yr = (double)y[r];
  const double t2 = tau * (1.0 - tau);
  if (val) {
    const double v = (double)val[i];
    g += -yr * tau * v;
    u += fmin(t2 * exp(fabs(v) * dl), 0.25) * v * v;
  } else {
    g += -yr * tau;
    u += fmin(t2 * exp(dl), 0.25);
  }
}

// rowq[i] = {-y_i tau_i, tau_i (1 - tau_i)}: the per-example factors of G / U packed in
// one 16-B record, recomputed per wide block (bcd_rowq_kernel, a 4 M-row stream), so the
// random per-entry gather fetches ONE line instead of two (ym and y) and skips the
// exp: the wide blocks' gradient is bound by these gathers.
// rows (optional): the block's distinct examples (a block of the CTR-log group layout
// touches ~1/15 of them: packing all 4 M rows per block cost 17.5 us, its list ~2 us).
__global__ void __launch_bounds__(256)
bcd_rowq_kernel(const double* __restrict__ ym, const float* __restrict__ y, int64_t n,
                const int32_t* __restrict__ rows, int64_t nrows, double2* __restrict__ rowq) {
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = rows ? rows[q] : q;
    if (!in_range(i, nrows)) continue;
    const double tau = 1.0 / (1.0 + exp(ym[i]));
    rowq[i] = make_double2(-(double)y[i] * tau, tau * (1.0 - tau));
  }
}

__device__ __forceinline__ void bcd_gu_q(int64_t i, const int32_t* __restrict__ row,
                                         const float* __restrict__ val,
                                         const double2* __restrict__ rowq, int64_t nrows,
                                         double dl, double& g, double& u) {
  const int32_t r = row[i];
  if (!in_range(r, nrows)) return;
  const double2 q = rowq[r];
  if (val) {
    const double v = (double)val[i];
    g += q.x * v;
    u += fmin(q.y * exp(fabs(v) * dl), 0.25) * v * v;
  } else {
    g += q.x;
    u += fmin(q.y * dl, 0.25);  // binary: dl is exp(delta) here
  }
}

template <bool kQ>
__global__ void __launch_bounds__(256)
bcd_grad_chunk_kernel(const int32_t* __restrict__ col, const int32_t* __restrict__ row,
                      const float* __restrict__ val, const int64_t* __restrict__ chunks,
                      int64_t nchunks, int64_t c0, int64_t ncols,
                      const double* __restrict__ ym, const float* __restrict__ y, int64_t nrows,
                      const double* __restrict__ delta, const uint8_t* __restrict__ active,
                      const double2* __restrict__ rowq,
                      double* __restrict__ G, double* __restrict__ U) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t k = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); k < nchunks;
       k += nw) {
    const int64_t e0 = chunks[k], e1 = chunks[k + 1];
    if (e0 & kSkipBit) continue;  // a column summed by the row pass (hot in LDS)
    const bool hot = (e0 & kHotBit) != 0;
    const int64_t a = e0 & ~(kHotBit | kSkipBit), b = e1 & ~(kHotBit | kSkipBit);
    if (hot) {
      const int64_t c = (int64_t)col[a] - c0;  // wave-uniform
      if (c < 0 || c >= ncols || !active[c0 + c]) continue;
      const double dl = delta[c0 + c];
      double g = 0, u = 0;
      if (kQ) {
        const double dq = val ? dl : exp(dl);
#pragma unroll 4
        for (int64_t i = a + lane; i < b; i += 64) bcd_gu_q(i, row, val, rowq, nrows, dq, g, u);
      } else {
#pragma unroll 4
        for (int64_t i = a + lane; i < b; i += 64) bcd_gu(i, c, c0, row, val, ym, y, nrows, dl, g, u);
      }
      g = wave_allsum(g);
      u = wave_allsum(u);
      if (lane == 0) {
        unsafeAtomicAdd(&G[c], g);
        unsafeAtomicAdd(&U[c], u);
      }
      continue;
    }
    const int64_t i = a + lane;
    const bool valid = i < b;
    int64_t c = -1;
    double g = 0, u = 0;
    if (valid) {
      c = (int64_t)col[i] - c0;
      if (c < 0 || c >= ncols) c = -1;
      else if (active[c0 + c]) {
        if (kQ) {
          const double dl = delta[c0 + c];
          bcd_gu_q(i, row, val, rowq, nrows, val ? dl : exp(dl), g, u);
        } else {
          bcd_gu(i, c, c0, row, val, ym, y, nrows, delta[c0 + c], g, u);
        }
      }
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const double go = shfl_up_d(g, off);
      const double uo = shfl_up_d(u, off);
      const int64_t co = __shfl_up(c, off, 64);
      if (lane >= off && co == c) { g += go; u += uo; }
    }
    const int64_t c_next = __shfl_down(c, 1, 64);
    if (valid && c >= 0 && (lane == 63 || i + 1 >= b || c_next != c)) {
      G[c] = g;  // whole column inside the chunk
      U[c] = u;
    }
  }
}

// K11, row order, for NARROW blocks (ncols <= kRowCols: the integer slots and the
// low-cardinality categorical slots of CTR data). The block's entries come from the
// row-sorted copy the dual update uses, so the per-row reads of ym / y stream
// sequentially instead of gathering one random 64-B line per entry (the column-order
// kernel's cost: ~106 us per 4 M-entry block, profiles/r3_darlin_prof.log). G / U
// accumulate per column in LDS as 64-bit FIXED POINT with integer LDS atomics
// (ds_add_u64 ~15 cycles vs ~195 for a float LDS atomic on gfx950), in `copies`
// replicas (copies x ncols <= 2048; 50 KB of LDS: 3 workgroups of 512 per CU) so that
// lanes of different waves on a hot column serialise less; each
// workgroup writes its exact partial sums, and bcd_rows_reduce adds the W partials of
// every column in a fixed order: the result is deterministic. Scale 2^k (host: the
// block's entry count x the largest |addend| < 2^(61-k), so the partials AND their
// sum are exact int64 sums).
constexpr int kRowCols = 2048;

// Fused coordinate update (upd.dw != null, one rank): the workgroups add their column
// sums into the block's accumulator (part) and the last one to finish (a device counter,
// reset by that workgroup) applies the update to every column, writing dw for the
// block's later dual update, and zeroes the accumulator. The
// block's columns are touched by no other block, so updating them when the gradient
// lands instead of tau blocks later changes nothing (kkt_thr is fixed within a pass).
struct RowsUpd {
  double* w;
  double* delta;   // (the kernel reads delta through its const view before the update)
  uint8_t* active;
  double* dw;
  unsigned long long* vio_bits;
  unsigned int* counter;
  double eta, lambda, delta_max, kkt_thr;
};

template <bool kVal>
__global__ void __launch_bounds__(512)
bcd_grad_rows_kernel(const int32_t* __restrict__ col, const int32_t* __restrict__ row,
                     const float* __restrict__ val, int64_t p0, int64_t p1, int64_t c0,
                     int ncols, int copies, const double* __restrict__ ym,
                     const float* __restrict__ y, int64_t nrows, const double* delta,
                     const uint8_t* active, int k2,
                     long long* __restrict__ part, RowsUpd upd) {
  __shared__ long long acc[2 * kRowCols];  // [copies][2][ncols] (G, U), copies*ncols <= 2048
  __shared__ double cdl[kRowCols];            // per column: exp(delta) (binary) or delta
  __shared__ uint8_t cact[kRowCols];
  const int t = threadIdx.x;
  const int stride = 2 * ncols;
  for (int i = t; i < copies * stride; i += blockDim.x) acc[i] = 0;
  for (int c = t; c < ncols; c += blockDim.x) {
    const double dl = delta[c0 + c];
    cdl[c] = kVal ? dl : exp(dl);
    cact[c] = active[c0 + c];
  }
  // fused update: every workgroup holds w / delta of "its" update columns (j = t + 512 q)
  // from the start, so the last one's update waits on no load but the sums
  constexpr int kUq = kRowCols / 512;
  double uw[kUq], ud[kUq];
  if (upd.dw) {
#pragma unroll
    for (int q = 0; q < kUq; ++q) {
      const int j = t + q * 512;
      uw[q] = j < ncols ? upd.w[c0 + j] : 0.0;
      ud[q] = j < ncols ? delta[c0 + j] : 0.0;
    }
  }
  __syncthreads();
  const int64_t n = p1 - p0;
  const int64_t per = (n + gridDim.x - 1) / gridDim.x;
  const int64_t a = p0 + per * blockIdx.x, b = min(p1, a + per);
  long long* my = acc + (int64_t)((t >> 6) % copies) * stride;
  const double sc = ldexp(1.0, k2);
  // kR entries per thread per round, every load of a round in flight before the math
  // (entries -> rows -> ym / y is a two-deep dependent chain)
  constexpr int kR = 8;
  for (int64_t i0 = a + t; i0 < b; i0 += (int64_t)kR * blockDim.x) {
    int cc[kR];
    int32_t rr[kR];
#pragma unroll
    for (int q = 0; q < kR; ++q) {
      const int64_t i = i0 + (int64_t)q * blockDim.x;
      cc[q] = -1;
      rr[q] = -1;
      if (i < b) {
        const int c = col[i] - (int)c0;
        cc[q] = (c >= 0 && c < ncols) ? c : -1;
        rr[q] = row[i];
      }
    }
    double ymv[kR];
    float yv[kR];
#pragma unroll
    for (int q = 0; q < kR; ++q) {
      const bool ok = cc[q] >= 0 && in_range(rr[q], nrows);
      ymv[q] = ok ? ym[rr[q]] : 0.0;
      yv[q] = ok ? y[rr[q]] : 0.f;
      if (!ok) cc[q] = -1;
    }
#pragma unroll
    for (int q = 0; q < kR; ++q) {
      const int c = cc[q];
      if (c < 0 || !cact[c]) continue;
      const double tau = 1.0 / (1.0 + exp(ymv[q]));
      const double yr = (double)yv[q];
      const double t2 = tau * (1.0 - tau);
      double g, u;
      if (kVal) {
        const double v = (double)val[i0 + (int64_t)q * blockDim.x];
        g = -yr * tau * v;
        u = fmin(t2 * exp(fabs(v) * cdl[c]), 0.25) * v * v;
      } else {
        g = -yr * tau;
        u = fmin(t2 * cdl[c], 0.25);
      }
      atomicAdd(reinterpret_cast<unsigned long long*>(&my[c]),
                (unsigned long long)__double2ll_rn(g * sc));
      atomicAdd(reinterpret_cast<unsigned long long*>(&my[ncols + c]),
                (unsigned long long)__double2ll_rn(u * sc));
    }
  }
  __syncthreads();
  if (!upd.dw) {
    long long* out = part + (int64_t)blockIdx.x * stride;
    for (int i = t; i < stride; i += blockDim.x) {
      long long s = 0;
      for (int q = 0; q < copies; ++q) s += acc[q * stride + i];
      out[i] = s;
    }
    return;
  }
  // fused update: part is the block's [G | U] fixed-point accumulator (2 x ncols int64,
  // zero between uses); the nonzero workgroup sums go in by int64 atomics (exact: the
  // result does not depend on their order)
  for (int i = t; i < stride; i += blockDim.x) {
    long long s = 0;
    for (int q = 0; q < copies; ++q) s += acc[q * stride + i];
    if (s) atomicAdd(reinterpret_cast<unsigned long long*>(part + i), (unsigned long long)s);
  }
  __shared__ unsigned int last;
  __threadfence();  // this workgroup's sums visible device-wide before it counts
  __syncthreads();
  if (t == 0) {
    const unsigned int prev = atomicAdd(upd.counter, 1u);
    last = prev == gridDim.x - 1;
    if (last) upd.counter[0] = 0;  // (every other workgroup has counted: reuse)
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  const double isc = ldexp(1.0, -k2);
  double vmax = 0;
#pragma unroll
  for (int q = 0; q < kUq; ++q) {
    const int j = t + q * 512;
    if (j >= ncols) break;
    // (other workgroups' atomics: device-coherent loads), then zero for the next use
    const long long sg = __hip_atomic_load(part + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const long long su =
        __hip_atomic_load(part + ncols + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    part[j] = 0;
    part[ncols + j] = 0;
    const int64_t k = c0 + j;
    double d = 0;
    if (cact[j])
      d = bcd_update_col(k, (double)sg * isc, (double)su * isc, uw[q], ud[q], upd.w, upd.delta,
                         upd.active, upd.eta, upd.lambda, upd.delta_max, upd.kkt_thr, 0, vmax);
    upd.dw[j] = d;
  }
  bcd_vio_max(vmax, upd.vio_bits);
}

// G[c] / U[c] = sum over the W workgroup partials x 2^-k: one workgroup per output, its
// threads strided over the partials, then a wave / block sum (int64: exact, so the
// order does not matter and the result is deterministic).
__global__ void __launch_bounds__(256)
bcd_rows_reduce_kernel(const long long* __restrict__ part, int W, int ncols, int k2,
                       double* __restrict__ G, double* __restrict__ U,
                       const int32_t* __restrict__ cols = nullptr) {
  __shared__ long long ws[4];
  const int i = blockIdx.x;  // output 0 .. 2*ncols-1
  long long s = 0;
  for (int w = threadIdx.x; w < W; w += blockDim.x) s += part[(int64_t)w * 2 * ncols + i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const long long tot = ws[0] + ws[1] + ws[2] + ws[3];
    const double v = (double)tot * ldexp(1.0, -k2);
    const int c = i < ncols ? i : i - ncols;
    const int o = cols ? cols[c] : c;  // (hot-column sums of a wide block: their columns)
    if (i < ncols) G[o] = v;
    else U[o] = v;
  }
}

// Row pass over DENSE per-row block layouts (blocks with at most one entry per example,
// the slot layout of CTR data): dcol[i] = column of example i's entry relative to the
// block's c0 (-1: none), dval[i] its value (null: binary). 4 B per example instead of a
// (col, row) pair per entry, read in example order. One pass applies the PENDING dual
// update of block j (ym_i += y_i dw_c x_ic, the update that ran last on the stream) and
// then, on the updated margin, the gradient of the NEXT block k: the dual update of a
// block is always followed by the next block's gradient in the BCD loop, so the pair
// fuses without changing the order of anything (bitwise equal to bcd_dual + grad).
//   bcd_rowpass_grad_kernel: k narrow (ncols <= kRowCols): fixed-point LDS column sums
//     as bcd_grad_rows_kernel (W partials, then bcd_rows_reduce);
//   bcd_rowpass_q_kernel: k wide: writes rowq[i] for the examples of block k (what
//     bcd_rowq_kernel wrote for all of them) for the chunked column-order gradient;
//     without a grad block it is the dense dual update alone.
constexpr int kColdRow = 1 << 30;  // row pass: the example's entry is in a cold column

struct RowDual {
  const int32_t* dcol;  // null: no pending dual update
  const float* dval;
  const double* dw;
  int ncols;
};

// tau_i = 1 / (1 + exp(ym_i)) in the row passes: kF32 computes it in fp32 (v_exp_f32 +
// v_rcp_f32, ~1e-7 relative) instead of fp64 exp + divide (~50 VALU ops per example,
// what made the narrow pass VALU-bound: profiles/r3_darlin_rowpass.log); the factors
// -y tau, tau (1 - tau) and the G / U sums stay fp64 / 64-bit fixed point.
template <bool kF32>
__device__ __forceinline__ double rp_tau(double m) {
  if (kF32) {
    const float e = __expf(fminf((float)m, 80.f));  // exp(80) < FLT_MAX: no inf / NaN
    return (double)__builtin_amdgcn_rcpf(1.f + e);
  }
  return 1.0 / (1.0 + exp(m));
}

template <bool kF32>
__device__ __forceinline__ double rp_exp(double x) {
  return kF32 ? (double)__expf(fminf((float)x, 80.f)) : exp(x);
}

__device__ __forceinline__ double rp_dual_delta(const RowDual& d, int c, uint32_t i, double dwc,
                                                double yr) {
  const double x = d.dval ? (double)d.dval[i] : 1.0;
  return yr * dwc * x;  // the bcd_dual_kernel expression: (y * dw) * x
}

// kHot (wide block k): the LDS sums cover the block's hottest columns only, hcols[h] =
// column of LDS slot h (ncols = their count); dcol[i] >= 0 marks a COLD entry (its
// factors go to rowq[i] for the chunked column-order kernel over the cold columns),
// dcol[i] <= -2 the hot slot -2 - dcol[i], -1 no entry.
template <bool kDual, bool kHot, bool kF32>
__global__ void __launch_bounds__(512)
bcd_rowpass_grad_kernel(int64_t n, double* __restrict__ ym, const float* __restrict__ y,
                        RowDual dj, const int32_t* __restrict__ dcol, const float* __restrict__ dval,
                        int64_t c0, int ncols, int copies, const double* __restrict__ delta,
                        const uint8_t* __restrict__ active, int k2, long long* __restrict__ part,
                        const int32_t* __restrict__ hcols, double2* __restrict__ rowq) {
  __shared__ long long acc[2 * kRowCols];  // [copies][2][ncols] (G, U)
  __shared__ double cdl[kRowCols];
  __shared__ uint8_t cact[kRowCols];
  const int t = threadIdx.x;
  const int stride = 2 * ncols;
  for (int i = t; i < copies * stride; i += blockDim.x) acc[i] = 0;
  for (int c = t; c < ncols; c += blockDim.x) {
    const int64_t k = c0 + (kHot ? hcols[c] : c);
    const double dl = delta[k];
    cdl[c] = dval ? dl : exp(dl);
    cact[c] = active[k];
  }
  __syncthreads();
  // 32-bit example offsets (the host checks n < 2^31): zero-extended VGPR offsets from
  // the arrays' SGPR bases, no 64-bit address arithmetic per access
  const uint32_t per = (uint32_t)((n + gridDim.x - 1) / gridDim.x);
  const uint32_t a = per * blockIdx.x, b = (uint32_t)min<int64_t>(n, (int64_t)a + per);
  long long* my = acc + (int64_t)((t >> 6) % copies) * stride;
  const double sc = ldexp(1.0, k2);
  constexpr int kR = 8;  // examples per thread per round, loads in flight together
  for (uint32_t i0 = a + t; i0 < b; i0 += (uint32_t)kR * blockDim.x) {
    int ck[kR], cj[kR];
    double m[kR];
    float yv[kR];
    // two batches of unconditional loads at clamped in-range indices (a guarded load per
    // example compiled to a branch + s_waitcnt each: ~kR serialised round trips), then
    // selects: the column codes, then margins and labels
    int cr[kR], dr[kR];
#pragma unroll
    for (int q = 0; q < kR; ++q) {
      const uint32_t i = i0 + (uint32_t)q * blockDim.x;
      const uint32_t ic = i < b ? i : a;
      cr[q] = dcol[ic];
      dr[q] = kDual ? dj.dcol[ic] : -1;
    }
#pragma unroll
    for (int q = 0; q < kR; ++q) {
      const uint32_t i = i0 + (uint32_t)q * blockDim.x;
      const bool in = i < b;
      const int c = cr[q];
      if (kHot) ck[q] = !in ? -1 : c >= 0 ? kColdRow : (c <= -2 && -2 - c < ncols) ? -2 - c : -1;
      else ck[q] = (in && c >= 0 && c < ncols) ? c : -1;
      cj[q] = (kDual && in && dr[q] >= 0 && dr[q] < dj.ncols) ? dr[q] : -1;
      const uint32_t im = (ck[q] != -1 || cj[q] >= 0) ? i : a;
      m[q] = ym[im];
      yv[q] = y[im];
    }
#pragma unroll
    for (int q = 0; q < kR; ++q)
      if (!(ck[q] != -1 || cj[q] >= 0)) {
        m[q] = 0;
        yv[q] = 0.f;
      }
    if (kDual) {
      double dwv[kR];
#pragma unroll
      for (int q = 0; q < kR; ++q) dwv[q] = cj[q] >= 0 ? dj.dw[cj[q]] : 0.0;
#pragma unroll
      for (int q = 0; q < kR; ++q) {
        if (dwv[q] == 0) continue;
        const uint32_t i = i0 + (uint32_t)q * blockDim.x;
        m[q] += rp_dual_delta(dj, cj[q], i, dwv[q], (double)yv[q]);
        ym[i] = m[q];
      }
    }
#pragma unroll
    for (int q = 0; q < kR; ++q) {
      const int c = ck[q];
      if (kHot && c == kColdRow) {  // cold entry: factors for the column-order kernel
        const double tau = rp_tau<kF32>(m[q]);
        rowq[i0 + (uint32_t)q * blockDim.x] = make_double2(-(double)yv[q] * tau, tau * (1.0 - tau));
        continue;
      }
      if (c < 0 || !cact[c]) continue;
      const double tau = rp_tau<kF32>(m[q]);
      const double yr = (double)yv[q];
      const double t2 = tau * (1.0 - tau);
      double g, u;
      if (dval) {
        const double v = (double)dval[i0 + (uint32_t)q * blockDim.x];
        g = -yr * tau * v;
        u = fmin(t2 * rp_exp<kF32>(fabs(v) * cdl[c]), 0.25) * v * v;
      } else {
        g = -yr * tau;
        u = fmin(t2 * cdl[c], 0.25);
      }
      atomicAdd(reinterpret_cast<unsigned long long*>(&my[c]),
                (unsigned long long)__double2ll_rn(g * sc));
      atomicAdd(reinterpret_cast<unsigned long long*>(&my[ncols + c]),
                (unsigned long long)__double2ll_rn(u * sc));
    }
  }
  __syncthreads();
  long long* out = part + (int64_t)blockIdx.x * stride;
  for (int i = t; i < stride; i += blockDim.x) {
    long long s = 0;
    for (int q = 0; q < copies; ++q) s += acc[q * stride + i];
    out[i] = s;
  }
}

template <bool kDual, bool kQ, bool kF32>
__global__ void __launch_bounds__(256)
bcd_rowpass_q_kernel(int64_t n, double* __restrict__ ym, const float* __restrict__ y, RowDual dj,
                     const int32_t* __restrict__ dcol, int ncols, double2* __restrict__ rowq) {
  constexpr int kR = 8;
  const uint32_t stride = gridDim.x * blockDim.x;  // (n < 2^31: 32-bit offsets)
  for (uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x; i0 < (uint64_t)n;
       i0 += (uint32_t)kR * stride) {
    int ck[kR], cj[kR];
    double m[kR];
    float yv[kR];
#pragma unroll
    for (int q = 0; q < kR; ++q) {
      const uint32_t i = i0 + q * stride;
      ck[q] = -1;
      cj[q] = -1;
      m[q] = 0;
      yv[q] = 0.f;
      if (i < n) {
        if (kQ) {
          const int c = dcol[i];
          ck[q] = (c >= 0 && c < ncols) ? c : -1;
        }
        if (kDual) {
          const int d = dj.dcol[i];
          cj[q] = (d >= 0 && d < dj.ncols) ? d : -1;
        }
      }
    }
    double dwv[kR];
#pragma unroll
    for (int q = 0; q < kR; ++q) {  // (margin loads beside the dw gather, not behind it)
      const uint32_t i = i0 + q * stride;
      if (ck[q] >= 0 || cj[q] >= 0) {
        m[q] = ym[i];
        yv[q] = y[i];
      }
      dwv[q] = kDual && cj[q] >= 0 ? dj.dw[cj[q]] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < kR; ++q) {
      const uint32_t i = i0 + q * stride;
      if (kDual && dwv[q] != 0) {
        m[q] += rp_dual_delta(dj, cj[q], i, dwv[q], (double)yv[q]);
        ym[i] = m[q];
      }
      if (kQ && ck[q] >= 0) {
        const double tau = rp_tau<kF32>(m[q]);
        rowq[i] = make_double2(-(double)yv[q] * tau, tau * (1.0 - tau));
      }
    }
  }
}

// Coalesced two-stage sum of the row pass's W workgroup partials part[w][i] (i < n2 =
// 2 x LDS columns): stage 1, one workgroup per 64 outputs x one of S segments of the
// partials, every load a 512-B run of one partial row (a thread per output striding
// over w read one 8-B word per 64-B line: ~35 us for 768 x 4096 partials); stage 2 adds
// the S segment sums and stores G / U (through the hot-column map). Exact int64 sums:
// deterministic in any order.
__global__ void __launch_bounds__(256)
bcd_part_reduce1_kernel(const long long* __restrict__ part, int W, int n2,
                        long long* __restrict__ part2) {
  __shared__ long long ws[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  const int w0 = (int)((int64_t)blockIdx.y * W / kPartSeg);
  const int w1 = (int)((int64_t)(blockIdx.y + 1) * W / kPartSeg);
  long long s = 0;
  if (i < n2)
    for (int w = w0 + wv; w < w1; w += 4) s += part[(int64_t)w * n2 + i];
  ws[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && i < n2)
    part2[(int64_t)blockIdx.y * n2 + i] = ws[0][lane] + ws[1][lane] + ws[2][lane] + ws[3][lane];
}

__global__ void __launch_bounds__(256)
bcd_part_reduce2_kernel(const long long* __restrict__ part2, int ncols, int k2,
                        double* __restrict__ G, double* __restrict__ U,
                        const int32_t* __restrict__ cols) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int n2 = 2 * ncols;
  if (i >= n2) return;
  long long s = 0;
#pragma unroll
  for (int q = 0; q < kPartSeg; ++q) s += part2[(int64_t)q * n2 + i];
  const double v = (double)s * ldexp(1.0, -k2);
  const int c = i < ncols ? i : i - ncols;
  const int o = cols ? cols[c] : c;
  if (i < ncols) G[o] = v;
  else U[o] = v;
}

// objective: out[0] += sum_i log(1 + exp(-ym_i))
__global__ void __launch_bounds__(256)
bcd_objective_kernel(const double* __restrict__ ym, int64_t n, double* __restrict__ out) {
  __shared__ double lds[4];
  double s = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    s += softplus_neg(ym[i]);
  const double t = block_sum_f64(s, lds);
  if (threadIdx.x == 0) unsafeAtomicAdd(out, t);
}

// server stats over [c0, c1): out[0] += sum |w| (w != 0), out[1] += nnz(w),
// out[2] += |active set|
__global__ void __launch_bounds__(256)
bcd_server_stats_kernel(const double* __restrict__ w, const uint8_t* __restrict__ active,
                        int64_t c0, int64_t c1, double* __restrict__ out) {
  __shared__ double lds[4];
  double a = 0, nz = 0, na = 0;
  for (int64_t k = c0 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < c1;
       k += (int64_t)gridDim.x * blockDim.x) {
    const double wk = w[k];
    if (wk != 0 && wk == wk) { a += fabs(wk); nz += 1; }
    na += active[k] ? 1 : 0;
  }
  a = block_sum_f64(a, lds);
  __syncthreads();
  nz = block_sum_f64(nz, lds);
  __syncthreads();
  na = block_sum_f64(na, lds);
  if (threadIdx.x == 0) {
    unsafeAtomicAdd(&out[0], a);
    unsafeAtomicAdd(&out[1], nz);
    unsafeAtomicAdd(&out[2], na);
  }
}

}  // namespace

void bcd_grad(const int32_t* col, const int32_t* row, const float* val, int64_t p0, int64_t p1,
              int64_t c0, int64_t ncols, const double* ym, const float* y, int64_t nrows,
              const double* delta, const uint8_t* active, double* G, double* U, hipStream_t st) {
  fill_async<double>(G, ncols, 0.0, st);
  fill_async<double>(U, ncols, 0.0, st);
  if (p1 <= p0) return;
  bcd_grad_kernel<<<grid_for(p1 - p0, 256, 4096), 256, 0, st>>>(
      col, row, val, p0, p1, c0, ncols, ym, y, nrows, delta, active, G, U);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void bcd_grad_chunked(const int32_t* col, const int32_t* row, const float* val,
                      const int64_t* chunks, int64_t nchunks, int64_t c0, int64_t ncols,
                      const double* ym, const float* y, int64_t nrows, const double* delta,
                      const uint8_t* active, double* rowq, double* G, double* U, bool zeroed,
                      bool rowq_ready, const int32_t* urows, int64_t nurows, hipStream_t st) {
  if (!zeroed) {
    fill_async<double>(G, ncols, 0.0, st);
    fill_async<double>(U, ncols, 0.0, st);
  }
  if (nchunks <= 0) return;
  if (rowq) {
    if (!rowq_ready) {  // (ready: a row pass wrote the block's examples' factors)
      const int64_t n = urows ? nurows : nrows;
      if (n > 0)
        bcd_rowq_kernel<<<grid_for(n, 256, 4096), 256, 0, st>>>(ym, y, n, urows, nrows,
                                                                 (double2*)rowq);
      PSAMD_HIP_CHECK(hipGetLastError());
    }
    bcd_grad_chunk_kernel<true><<<grid_for(nchunks, 4, 16384), 256, 0, st>>>(
        col, row, val, chunks, nchunks, c0, ncols, ym, y, nrows, delta, active,
        (const double2*)rowq, G, U);
  } else {
    bcd_grad_chunk_kernel<false><<<grid_for(nchunks, 4, 16384), 256, 0, st>>>(
        col, row, val, chunks, nchunks, c0, ncols, ym, y, nrows, delta, active, nullptr, G, U);
  }
  PSAMD_HIP_CHECK(hipGetLastError());
}

int bcd_rows_max_cols() { return kRowCols; }
int bcd_part_segments() { return kPartSeg; }

void bcd_grad_rows(const int32_t* col, const int32_t* row, const float* val, int64_t p0,
                   int64_t p1, int64_t c0, int64_t ncols, const double* ym, const float* y,
                   int64_t nrows, double* delta, uint8_t* active, int k2, int W,
                   long long* part, double* G, double* U, double* w, double* dw,
                   unsigned long long* vio_bits, unsigned int* counter, double eta, double lambda,
                   double delta_max, double kkt_thr, hipStream_t st) {
  if (ncols <= 0) return;
  if (ncols > kRowCols) throw std::runtime_error("bcd_grad_rows: ncols > 2048");
  const int copies = std::max(1, std::min(8, kRowCols / (int)ncols));
  // dw given: part is the block's 2 x ncols accumulator and the coordinate update runs in
  // the gradient's last workgroup (no reduce launch, no update launch)
  const RowsUpd upd{w, delta, active, dw, vio_bits, counter, eta, lambda, delta_max, kkt_thr};
  if (p1 > p0 || dw) {
    if (val)
      bcd_grad_rows_kernel<true><<<W, 512, 0, st>>>(col, row, val, p0, p1, c0, (int)ncols, copies,
                                                    ym, y, nrows, delta, active, k2, part, upd);
    else
      bcd_grad_rows_kernel<false><<<W, 512, 0, st>>>(col, row, val, p0, p1, c0, (int)ncols, copies,
                                                     ym, y, nrows, delta, active, k2, part, upd);
    PSAMD_HIP_CHECK(hipGetLastError());
  } else {
    fill_async<long long>(part, (int64_t)W * 2 * ncols, 0, st);
  }
  if (dw) return;
  bcd_rows_reduce_kernel<<<(unsigned)(2 * ncols), 256, 0, st>>>(part, W, (int)ncols, k2, G, U);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void bcd_update(int64_t c0, int64_t ncols, double* G, double* U, double* w, double* delta,
                uint8_t* active, double* dw, double eta, double lambda, double delta_max,
                double kkt_thr, unsigned long long* vio_bits, bool consume, bool nan_filtered,
                const long long* part2, int k2, hipStream_t st) {
  if (ncols <= 0) return;
  bcd_update_kernel<<<grid_for(ncols, 256, 4096), 256, 0, st>>>(
      c0, ncols, G, U, w, delta, active, dw, eta, lambda, delta_max, kkt_thr, vio_bits,
      consume ? 1 : 0, nan_filtered ? 1 : 0, part2, k2);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void bcd_replica(int64_t c0, int64_t ncols, int64_t own0, int64_t own1, double* dw, double* w,
                 double* delta, uint8_t* active, double delta_max, hipStream_t st) {
  if (ncols <= 0) return;
  bcd_replica_kernel<<<grid_for(ncols, 256, 4096), 256, 0, st>>>(c0, ncols, own0, own1, dw, w,
                                                                  delta, active, delta_max);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void bcd_dual(const int32_t* col, const int32_t* row, const float* val, int64_t p0, int64_t p1,
              int64_t c0, int64_t ncols, const double* dw, const float* y, double* ym,
              int64_t nrows, bool unique_rows, hipStream_t st) {
  if (p1 <= p0) return;
  if (unique_rows)
    bcd_dual_kernel<true><<<grid_for(p1 - p0, 256, 4096), 256, 0, st>>>(
        col, row, val, p0, p1, c0, ncols, dw, y, ym, nrows);
  else
    bcd_dual_kernel<false><<<grid_for(p1 - p0, 256, 4096), 256, 0, st>>>(
        col, row, val, p0, p1, c0, ncols, dw, y, ym, nrows);
  PSAMD_HIP_CHECK(hipGetLastError());
}

// Row pass (see bcd_rowpass_grad_kernel): pending dual of block j (jcol null: none), then
// block k's gradient: narrow (part != null: LDS fixed point, W partials + reduce into G / U)
// or rowq (wide; kcol null: the dense dual alone).
void bcd_rowpass(int64_t n, double* ym, const float* y, const int32_t* jcol, const float* jval,
                 const double* jdw, int64_t jncols, const int32_t* kcol, const float* kval,
                 int64_t c0, int64_t ncols, const double* delta, const uint8_t* active, int k2,
                 int W, long long* part, double* G, double* U, double* rowq,
                 const int32_t* hcols, int64_t nhot, long long* part2_out, bool tau32,
                 hipStream_t st) {
  if (n <= 0) return;
  if (n >= ((int64_t)1 << 31)) throw std::runtime_error("bcd_rowpass: >= 2^31 examples per rank");
  const RowDual dj{jcol, jval, jdw, (int)jncols};
  if (part) {  // gradient of block k in LDS: narrow (all columns) or wide (hot columns)
    const int nl = (int)(hcols ? nhot : ncols);  // LDS column slots
    if (nl <= 0) return;
    if (nl > kRowCols) throw std::runtime_error("bcd_rowpass: > 2048 LDS columns");
    const int copies = std::max(1, std::min(8, kRowCols / nl));
    auto q = reinterpret_cast<double2*>(rowq);
#define PSAMD_RP(D, H)                                                                       \
  do {                                                                                        \
    if (tau32)                                                                                \
      bcd_rowpass_grad_kernel<D, H, true><<<W, 512, 0, st>>>(n, ym, y, dj, kcol, kval, c0, nl, \
                                                             copies, delta, active, k2, part,  \
                                                             hcols, q);                        \
    else                                                                                      \
      bcd_rowpass_grad_kernel<D, H, false><<<W, 512, 0, st>>>(n, ym, y, dj, kcol, kval, c0,    \
                                                              nl, copies, delta, active, k2,   \
                                                              part, hcols, q);                 \
  } while (0)
    if (jcol && hcols) PSAMD_RP(true, true);
    else if (jcol) PSAMD_RP(true, false);
    else if (hcols) PSAMD_RP(false, true);
    else PSAMD_RP(false, false);
#undef PSAMD_RP
    PSAMD_HIP_CHECK(hipGetLastError());
    // [kPartSeg][2 nl] segment sums: after the partials, or (part2_out) the block's own
    // buffer that its coordinate update reads directly (no second stage)
    long long* part2 = part2_out ? part2_out : part + (int64_t)W * 2 * nl;
    bcd_part_reduce1_kernel<<<dim3((unsigned)((2 * nl + 63) / 64), kPartSeg), 256, 0, st>>>(
        part, W, 2 * nl, part2);
    PSAMD_HIP_CHECK(hipGetLastError());
    if (part2_out) return;
    bcd_part_reduce2_kernel<<<(unsigned)((2 * nl + 255) / 256), 256, 0, st>>>(part2, nl, k2, G, U,
                                                                            hcols);
    PSAMD_HIP_CHECK(hipGetLastError());
    return;
  }
  const unsigned grid = (unsigned)grid_for(n, 256 * 8, 4096);
  auto q = reinterpret_cast<double2*>(rowq);
#define PSAMD_RQ(D, K)                                                                      \
  do {                                                                                       \
    if (tau32)                                                                               \
      bcd_rowpass_q_kernel<D, K, true><<<grid, 256, 0, st>>>(n, ym, y, dj, kcol, (int)ncols, q); \
    else                                                                                     \
      bcd_rowpass_q_kernel<D, K, false><<<grid, 256, 0, st>>>(n, ym, y, dj, kcol, (int)ncols,  \
                                                              q);                            \
  } while (0)
  if (jcol && kcol) PSAMD_RQ(true, true);
  else if (kcol) PSAMD_RQ(false, true);
  else if (jcol) PSAMD_RQ(true, false);
  else return;
#undef PSAMD_RQ
  PSAMD_HIP_CHECK(hipGetLastError());
}

void bcd_objective(const double* ym, int64_t n, double* out, hipStream_t st) {
  if (n <= 0) return;
  bcd_objective_kernel<<<grid_for(n, 256, 1024), 256, 0, st>>>(ym, n, out);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void bcd_server_stats(const double* w, const uint8_t* active, int64_t c0, int64_t c1, double* out,
                      hipStream_t st) {
  if (c1 <= c0) return;
  bcd_server_stats_kernel<<<grid_for(c1 - c0, 256, 1024), 256, 0, st>>>(w, active, c0, c1, out);
  PSAMD_HIP_CHECK(hipGetLastError());
}

}  // namespace psamd
