// bf16 MFMA GEMM for the dense (MLP) blocks of the wide & deep model.
//
//   C[m, n] = sum_k A(m, k) * B(n, k)           (fp32 accumulation)
//   A(m, k) = A[m * lda + k]  (A_KMAJOR)  or  A[k * lda + m]
//   B(n, k) = B[n * ldb + k]  (B_KMAJOR)  or  B[k * ldb + n]
//
// The three products of a Linear layer with weights W[N_out, K_in] (bf16, the
// torch layout) and activations X[B, K_in] all map onto it without any
// transposed copy: forward X.W^T (A, B K-major), input gradient dZ.W (A
// K-major, B MN-major), weight gradient dZ^T.X (both MN-major).
//
// CDNA4 design: 256 threads = 4 wave64 in 2x2, a 128x128 block tile, BK = 64;
// each wave owns 64x64 = 4x4 tiles of v_mfma_f32_16x16x32_bf16 (lane l holds
// A[row l&15][k 8(l>>4)..+7], B[k 8(l>>4)..+7][col l&15]; C col = l&15,
// row = 4(l>>4)+j). Operands are staged global -> registers -> LDS as
// [rows][BK+8] K-contiguous images (144-B row stride: the 16 lanes of a
// ds_read_b128 group hit 16 distinct 16-B bank slots); an MN-major operand keeps
// its global layout in LDS ([BK][BM+16], coalesced 16-B loads and stores) and its
// fragments are read with the gfx950 hardware transpose ds_read_b64_tr_b16.
// Double-buffered LDS with the next tile's global loads in
// flight during the current tile's MFMAs (one barrier per K-step). The block
// index is remapped so consecutive tiles of one A panel share an XCD's L2.
//
// Fused epilogues: + bias[n], ReLU, multiply by the ReLU mask of an auxiliary
// bf16 tensor (backward through an activation), bf16 and/or fp32 stores, and the
// output's column sums (the input-gradient GEMM of layer i emits dZ of layer i-1,
// whose column sums are that layer's bias gradient: no second pass over dZ).
#include "common.cuh"

#include <hip/hip_bf16.h>
#include <algorithm>

namespace psamd {

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 128, BN = 128, BK = 64, LDS_K = BK + 8;  // padded row (elements)
constexpr int LDS_M = BM + 16;  // MN-major image row: [BK][BM + 16] (288-B stride)
constexpr int THREADS = 256;
constexpr int LDS_ELEMS = BM * LDS_K > BK * LDS_M ? BM * LDS_K : BK * LDS_M;
static_assert(BM == BN, "square block tile");

typedef short v4i16 __attribute__((ext_vector_type(4)));

// MN-major image: element (k, m) at [k][m ^ 64 * ((k >> 3) & 1)]; rows 8 apart then
// land on disjoint 32-B bank windows for the transposed reads below.
__device__ __forceinline__ int mn_off(int k, int m) { return k * LDS_M + (m ^ (((k >> 3) & 1) << 6)); }

enum Epi : int {
  EPI_NONE = 0,      // C = acc
  EPI_BIAS = 1,      // + bias[n]
  EPI_RELU = 2,      // max(., 0)
  EPI_MASK = 4,      // * (aux[m, n] > 0)   (backward through ReLU)
  EPI_COLSUM = 8,    // colsum[n] += sum_m C[m, n]  (bias gradient of the layer below)
  EPI_VEC = 16,      // (set by the host) vectorised epilogue through LDS, see below
};
constexpr int EPI_LDS = 68;  // fp32 row stride of a wave's 64 x 64 staging tile

__device__ __forceinline__ int xcd_swizzle(int bid, int nwg) {
  // bijective remap: the blocks that land on one XCD (bid % 8) get a contiguous range
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / 8;
}

// Stage one operand tile [rows r0.., k k0..] into registers.
template <bool KMAJOR>
struct Stage {
  uint4 v[4];
  __device__ __forceinline__ void load(const __bf16* __restrict__ p, int ld, int rows, int K,
                                       int r0, int k0, int tid) {
    if (KMAJOR) {
      // 128 rows x 8 chunks of 8 k -> 4 chunks per thread
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = tid + i * THREADS;
        const int row = c >> 3, kc = (c & 7) * 8;
        const int gr = r0 + row, gk = k0 + kc;
        if (gr < rows && gk < K)
          v[i] = *reinterpret_cast<const uint4*>(p + (int64_t)gr * ld + gk);
        else
          v[i] = make_uint4(0, 0, 0, 0);
      }
    } else {
      // 64 k-rows x 16 chunks of 8 m -> 4 chunks per thread (16 lanes = 256 B per row)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = tid + i * THREADS;
        const int kk = c >> 4, mc = (c & 15) * 8;
        const int gr = r0 + mc, gk = k0 + kk;
        if (gr < rows && gk < K)
          v[i] = *reinterpret_cast<const uint4*>(p + (int64_t)gk * ld + gr);
        else
          v[i] = make_uint4(0, 0, 0, 0);
      }
    }
  }
  __device__ __forceinline__ void store(__bf16* __restrict__ lds, int tid) const {
    if (KMAJOR) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = tid + i * THREADS;
        const int row = c >> 3, kc = (c & 7) * 8;
        *reinterpret_cast<uint4*>(lds + row * LDS_K + kc) = v[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = tid + i * THREADS;
        const int kk = c >> 4, mc = (c & 15) * 8;
        *reinterpret_cast<uint4*>(lds + mn_off(kk, mc)) = v[i];
      }
    }
  }
};

// 16x16x32 operand fragment of rows [rb, rb+16), k [ks, ks+32): lane l gets
// X[rb + (l & 15)][ks + 8 (l >> 4) + j], j = 0..7.
template <bool KMAJOR>
__device__ __forceinline__ bf16x8 load_frag(const __bf16* __restrict__ img, int rb, int ks,
                                            int lane) {
  if (KMAJOR)
    return *reinterpret_cast<const bf16x8*>(img + (rb + (lane & 15)) * LDS_K + ks +
                                            8 * (lane >> 4));
  // [k][m] image: two hardware transposed reads (ds_read_b64_tr_b16) of 4 k-rows x 16
  // m-columns; lane 4r+p of each 16-lane group addresses row r, columns 4p..4p+3.
  const int q = lane >> 4, li = lane & 15, r = li >> 2, pc = li & 3;
  const int k1 = ks + 8 * q + r;
  typedef __attribute__((address_space(3))) v4i16 lds_v4;
  const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_v4*)(img + mn_off(k1, rb + 4 * pc)));
  const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (lds_v4*)(img + mn_off(k1 + 4, rb + 4 * pc)));
  const v4i16 both[2] = {lo, hi};
  return *reinterpret_cast<const bf16x8*>(both);
}

template <bool A_KMAJOR, bool B_KMAJOR>
__global__ void __launch_bounds__(THREADS)
gemm_bf16_kernel(const __bf16* __restrict__ A, int lda, const __bf16* __restrict__ B, int ldb,
                 int M, int N, int K, int epi, const float* __restrict__ bias,
                 const __bf16* __restrict__ aux, int ldaux, __bf16* __restrict__ C, int ldc,
                 float* __restrict__ Cf, int ldcf, float beta, int kchunk,
                 float* __restrict__ colsum) {
  __shared__ __attribute__((aligned(16))) __bf16 lds[2][2][LDS_ELEMS];  // [buf][A|B]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int bid = xcd_swizzle(blockIdx.x, tiles_m * tiles_n);
  const int m0 = (bid / tiles_n) * BM, n0 = (bid % tiles_n) * BN;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  Stage<A_KMAJOR> sa;
  Stage<B_KMAJOR> sb;
  // split-K: blockIdx.y owns k in [kbeg, kend); partial sums are added atomically
  const int kbeg = blockIdx.y * kchunk;
  const int kend = min(K, kbeg + kchunk);
  const bool split = gridDim.y > 1;
  const int nk = (kend - kbeg + BK - 1) / BK;
  sa.load(A, lda, M, kend, m0, kbeg, tid);
  sb.load(B, ldb, N, kend, n0, kbeg, tid);
  sa.store(lds[0][0], tid);
  sb.store(lds[0][1], tid);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + 1 < nk;
    if (more) {  // next tile's global loads stay in flight during the MFMAs below
      sa.load(A, lda, M, kend, m0, kbeg + (kt + 1) * BK, tid);
      sb.load(B, ldb, N, kend, n0, kbeg + (kt + 1) * BK, tid);
    }
#pragma unroll
    for (int ks = 0; ks < BK; ks += 32) {
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i] = load_frag<A_KMAJOR>(lds[cur][0], wm * 64 + i * 16, ks, lane);
        b[i] = load_frag<B_KMAJOR>(lds[cur][1], wn * 64 + i * 16, ks, lane);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      sa.store(lds[cur ^ 1][0], tid);
      sb.store(lds[cur ^ 1][1], tid);
    }
    __syncthreads();
    cur ^= 1;
  }

  if ((epi & EPI_VEC) && !split) {
    // Vectorised epilogue: the MFMA layout gives a lane 4 rows of ONE column per
    // 16x16 tile, so direct stores are 2-byte scatters (and the ReLU-mask reads
    // 2-byte gathers). Stage the wave's 64 x 64 fp32 tile in LDS (free after the
    // main loop's last barrier; 4 x 17 KB <= 72 KB), then each lane owns 8
    // consecutive columns of 8 rows: 16-B mask loads, 16-B bf16 stores, 32-B fp32
    // stores, and column sums reduced over the 8 row lanes with 3 shuffles.
    float* W = reinterpret_cast<float*>(&lds[0][0][0]) + wid * (64 * EPI_LDS);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          W[(i * 16 + 4 * (lane >> 4) + r) * EPI_LDS + j * 16 + (lane & 15)] = acc[i][j][r];
    __syncthreads();
    const int cg = lane & 7, rr = lane >> 3;
    const int n = n0 + wn * 64 + cg * 8;
    const bool nok = n < N;  // host guarantees N % 8 == 0
    float bn[8], cs[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      bn[q] = ((epi & EPI_BIAS) && nok) ? bias[n + q] : 0.f;
      cs[q] = 0.f;
    }
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int row = it * 8 + rr;
      const int m = m0 + wm * 64 + row;
      if (m >= M || !nok) continue;
      const float4 x0 = *reinterpret_cast<const float4*>(&W[row * EPI_LDS + cg * 8]);
      const float4 x1 = *reinterpret_cast<const float4*>(&W[row * EPI_LDS + cg * 8 + 4]);
      float x[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        x[q] += bn[q];
        if (epi & EPI_RELU) x[q] = fmaxf(x[q], 0.f);
      }
      if (epi & EPI_MASK) {
        const bf16x8 mv = *reinterpret_cast<const bf16x8*>(aux + (int64_t)m * ldaux + n);
#pragma unroll
        for (int q = 0; q < 8; ++q) x[q] = ((float)mv[q] > 0.f) ? x[q] : 0.f;
      }
      if (C) {
        bf16x8 o;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          o[q] = (__bf16)x[q];
          cs[q] += (float)o[q];
        }
        *reinterpret_cast<bf16x8*>(C + (int64_t)m * ldc + n) = o;
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) cs[q] += x[q];
      }
      if (Cf) {
        float4* p = reinterpret_cast<float4*>(Cf + (int64_t)m * ldcf + n);
        float4 y0 = make_float4(x[0], x[1], x[2], x[3]), y1 = make_float4(x[4], x[5], x[6], x[7]);
        if (beta != 0.f) {
          const float4 o0 = p[0], o1 = p[1];
          y0.x += beta * o0.x; y0.y += beta * o0.y; y0.z += beta * o0.z; y0.w += beta * o0.w;
          y1.x += beta * o1.x; y1.y += beta * o1.y; y1.z += beta * o1.z; y1.w += beta * o1.w;
        }
        p[0] = y0;
        p[1] = y1;
      }
    }
    if (epi & EPI_COLSUM) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        cs[q] += __shfl_xor(cs[q], 8, 64);
        cs[q] += __shfl_xor(cs[q], 16, 64);
        cs[q] += __shfl_xor(cs[q], 32, 64);
      }
      // every lane of column group cg now holds its 8 sums: lane (rr, cg) adds
      // column n + rr, so ONE atomic instruction covers the wave's 64 columns
      float v = cs[0];
#pragma unroll
      for (int q = 1; q < 8; ++q) v = rr == q ? cs[q] : v;
      if (nok) unsafeAtomicAdd(colsum + n + rr, v);
    }
    return;
  }

  // epilogue: lane holds rows 4(l>>4)+r, col l&15 of every 16x16 tile
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + j * 16 + (lane & 15);
    float cs = 0.f;  // this lane's part of the tile column sum (EPI_COLSUM)
    if (n < N) {
      const float bn = (epi & EPI_BIAS) ? bias[n] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = m0 + wm * 64 + i * 16 + 4 * (lane >> 4) + r;
          if (m >= M) continue;
          float x = acc[i][j][r] + bn;
          if (epi & EPI_RELU) x = fmaxf(x, 0.f);
          if (epi & EPI_MASK) x = ((float)aux[(int64_t)m * ldaux + n] > 0.f) ? x : 0.f;
          if (split) {  // fp32 output only (host pre-scales Cf by beta)
            unsafeAtomicAdd(Cf + (int64_t)m * ldcf + n, x);
            cs += x;
            continue;
          }
          const __bf16 xb = (__bf16)x;
          if (C) C[(int64_t)m * ldc + n] = xb;
          cs += C ? (float)xb : x;  // the sum of what the next GEMM reads
          if (Cf) {
            float* p = Cf + (int64_t)m * ldcf + n;
            *p = beta != 0.f ? x + beta * *p : x;
          }
        }
      }
    }
    if (epi & EPI_COLSUM) {  // block-uniform: the 4 lanes of a column, one atomic
      cs += __shfl_xor(cs, 16, 64);
      cs += __shfl_xor(cs, 32, 64);
      if (n < N && lane < 16) unsafeAtomicAdd(colsum + n, cs);
    }
  }
}

// Zero the fp32 output of a split-K GEMM: a kernel, not hipMemset2DAsync (measured on
// the W&D weight-gradient stream: 129 us for the 1024 x 4992 dW, ~5 us as a kernel of
// 16-B stores; a memset node inside a captured graph may also leave the stream order).
__global__ void __launch_bounds__(256)
zero_rows_kernel(float* __restrict__ p, int64_t ld, int M, int N, int vec) {
  for (int m = blockIdx.y; m < M; m += gridDim.y) {
    float* r = p + (int64_t)m * ld;
    if (vec) {
      float4* r4 = reinterpret_cast<float4*>(r);
      for (int n = blockIdx.x * blockDim.x + threadIdx.x; n < N / 4; n += gridDim.x * blockDim.x)
        r4[n] = make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
      for (int n = blockIdx.x * blockDim.x + threadIdx.x; n < N; n += gridDim.x * blockDim.x)
        r[n] = 0.f;
    }
  }
}

}  // namespace

void gemm_bf16(bool a_kmajor, bool b_kmajor, const void* A, int lda, const void* B, int ldb,
               int M, int N, int K, int epi, const float* bias, const void* aux, int ldaux,
               void* C, int ldc, float* Cf, int ldcf, float beta, int splitk, float* colsum,
               hipStream_t st) {
  if (M <= 0 || N <= 0) return;
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (splitk < 1) splitk = 1;
  // k chunks are whole BK tiles; a split GEMM accumulates fp32 partials atomically
  const int kchunk = ((K + splitk * BK - 1) / (splitk * BK)) * BK;
  splitk = (K + kchunk - 1) / kchunk;
  if (splitk > 1) {
    if (beta == 0.f) {
      const int vec = (N % 4 == 0 && ldcf % 4 == 0 && (reinterpret_cast<uintptr_t>(Cf) & 15) == 0);
      const int per = vec ? N / 4 : N;
      const dim3 zg((unsigned)std::min(8, (per + 255) / 256), (unsigned)std::min(M, 2048));
      zero_rows_kernel<<<zg, 256, 0, st>>>(Cf, ldcf, M, N, vec);
      PSAMD_HIP_CHECK(hipGetLastError());
    }
    else if (beta != 1.f)
      throw std::runtime_error("split-K GEMM supports beta 0 or 1");
  }
  const dim3 grid(tiles, splitk);
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (splitk == 1 && N % 8 == 0 && (!C || (ldc % 8 == 0 && al16(C))) &&
      (!Cf || (ldcf % 4 == 0 && al16(Cf))) && (!(epi & EPI_MASK) || (ldaux % 8 == 0 && al16(aux))))
    epi |= EPI_VEC;
  auto a = reinterpret_cast<const __bf16*>(A);
  auto b = reinterpret_cast<const __bf16*>(B);
  auto x = reinterpret_cast<const __bf16*>(aux);
  auto c = reinterpret_cast<__bf16*>(C);
#define PSAMD_GEMM(AK, BKM)                                                               \
  gemm_bf16_kernel<AK, BKM><<<grid, THREADS, 0, st>>>(a, lda, b, ldb, M, N, K, epi, bias, x, \
                                                      ldaux, c, ldc, Cf, ldcf, beta, kchunk, \
                                                      colsum)
  if (a_kmajor && b_kmajor) PSAMD_GEMM(true, true);
  else if (a_kmajor) PSAMD_GEMM(true, false);
  else if (b_kmajor) PSAMD_GEMM(false, true);
  else PSAMD_GEMM(false, false);
#undef PSAMD_GEMM
  PSAMD_HIP_CHECK(hipGetLastError());
}

}  // namespace psamd
