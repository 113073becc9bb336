// 256 x 256-tile bf16 MFMA GEMM for K-major operands ("NT": C = A B^T):
//
//   C[m, n] = act(sum_k A[m * lda + k] * B[n * ldb + k] + bias[n])   (fp32 accumulate)
//
// The wide & deep forward products X W^T (X [B, K_in], W [N_out, K_in], the torch
// layout) and, with the transposed weight copy, the input gradients dZ W take this
// form. The 128 x 128 register-staged kernel of gemm.hip measured 684 TFLOP/s on the
// 16384 x 1024 x 4992 forward; this one is built for the long-K products:
//
// * 512 threads = 8 wave64 as 2 (M) x 4 (N); a wave owns a 128 x 64 output = 8 x 4
//   v_mfma_f32_16x16x32_bf16 tiles (lane l: A[row l&15][k 8(l>>4)..+7],
//   B[k 8(l>>4)..+7][col l&15]; C col l&15, rows 4(l>>4)+j), 64 MFMAs per K-step.
// * operands go global -> LDS by LDS-DMA (global_load_lds_dwordx4: no VGPR round
//   trip, 4 instructions per operand per thread per 256 x 64 tile); two 64 KiB
//   buffers (A | B), the next K-step's DMA in flight while the MFMAs of this one run,
//   one counted wait + one barrier per K-step; all LDS in one __shared__ array.
// * LDS image [256 rows][64 k] of 128-B rows with the 16-B chunk c of row r stored at
//   c ^ ((r >> 1) & 7): the 16 lanes of a ds_read_b128 lane group (rows r..r+15, one
//   logical chunk) then cover all 64 banks. LDS-DMA writes lane-linear, so the
//   swizzle is applied to the per-lane GLOBAL source address.
// * bijective XCD remap of the block index: the tiles of one A panel run on one XCD
//   (its 4 MiB L2 keeps the panel for all its N tiles).
// * fused epilogue: + bias[n], ReLU, bf16 and / or fp32 stores.
// Requirements (checked by the binding): K % 64 == 0, lda / ldb multiples of 8
// (16-B rows), 16-B aligned operands. Rows past M / N are clamped on load and
// masked on store.
#include "common.cuh"

#include <hip/hip_bf16.h>

#include <stdexcept>

namespace psamd {

namespace g256 {
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int BM = 256, BN = 256, BK = 64, TH = 512;
constexpr int TILE_BYTES = BM * BK * 2;   // 32 KiB per operand tile
constexpr int BUF_BYTES = 2 * TILE_BYTES; // A | B
}  // namespace g256

__device__ __forceinline__ int g256_swz(int r, int c) { return c ^ ((r >> 1) & 7); }

__device__ __forceinline__ int g256_xcd(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = bid % 8;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + bid / 8;
}

// LDS-DMA of one 256 x 64 operand tile (rows r0.., k k0..) into the image at dst:
// wave-instruction wi fills bytes [wi*1024, +1024) = rows wi*8 .. wi*8+7.
__device__ __forceinline__ void g256_stage(const __bf16* __restrict__ p, int64_t ld, int rows,
                                           int r0, int k0, char* dst, int wave, int lane) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int wi = q * 8 + wave;
    const int row = wi * 8 + (lane >> 3);
    const int c = g256_swz(row, lane & 7);
    int gr = r0 + row;
    gr = gr < rows ? gr : rows - 1;
    const __bf16* src = p + (int64_t)gr * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)src,
                                     (__attribute__((address_space(3))) void*)(dst + wi * 1024),
                                     16, 0, 0);
  }
}

// kFine: the fragment reads of a sub-step interleaved with its MFMAs (B fragments and
// A fragment 0 first, then A fragment i+1 in flight while the 4 MFMAs of fragment i
// issue, the next sub-step's B fragments during the last row), pinned by scheduling
// group barriers: the compiler's own schedule waits for all 12 reads (lgkmcnt(0))
// before the first of 32 MFMAs of every sub-step, and with 2 waves per SIMD that
// wait is only covered when the other wave happens to be in its MFMA run.
template <bool kFine>
__global__ void __launch_bounds__(g256::TH)
gemm_nt256_kernel(const __bf16* __restrict__ A, int64_t lda, const __bf16* __restrict__ B,
                  int64_t ldb, int M, int N, int K, const float* __restrict__ bias, int relu,
                  __bf16* __restrict__ C, int64_t ldc, float* __restrict__ Cf, int64_t ldcf,
                  int tiles_n) {
  using namespace g256;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF_BYTES];  // 128 KiB
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int id = g256_xcd(blockIdx.x, gridDim.x);
  const int tm = id / tiles_n, tn = id - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = K / BK;
  g256_stage(A, lda, M, m0, 0, smem, wave, lane);
  g256_stage(B, ldb, N, n0, 0, smem + TILE_BYTES, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const char* cur = smem + (kt & 1) * BUF_BYTES;
    if (kt + 1 < nk) {  // next K-step's DMA in flight during this one's MFMAs
      char* nxt = smem + ((kt + 1) & 1) * BUF_BYTES;
      g256_stage(A, lda, M, m0, (kt + 1) * BK, nxt, wave, lane);
      g256_stage(B, ldb, N, n0, (kt + 1) * BK, nxt + TILE_BYTES, wave, lane);
    }
    if (kFine) {
      auto rd_b = [&](int ks, int j) {
        const int c = ks * 4 + (lane >> 4), r = wc * 64 + j * 16 + (lane & 15);
        return *reinterpret_cast<const bf16x8*>(cur + TILE_BYTES + r * 128 + g256_swz(r, c) * 16);
      };
      auto rd_a = [&](int ks, int i) {
        const int c = ks * 4 + (lane >> 4), r = wr * 128 + i * 16 + (lane & 15);
        return *reinterpret_cast<const bf16x8*>(cur + r * 128 + g256_swz(r, c) * 16);
      };
      bf16x8 b[2][4], a[2];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[0][j] = rd_b(0, j);
      a[0] = rd_a(0, 0);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          // in flight during the 4 MFMAs of row i: A fragment i+1 (or the next sub-step's
          // first), and in the last row of sub-step 0 the next sub-step's B fragments
          if (i < 7) a[(i + 1) & 1] = rd_a(ks, i + 1);
          else if (ks == 0) a[(i + 1) & 1] = rd_a(1, 0);
          if (ks == 0 && i == 7) {
#pragma unroll
            for (int j = 0; j < 4; ++j) b[1][j] = rd_b(1, j);
          }
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i & 1], b[ks][j], acc[i][j], 0,
                                                                0, 0);
        }
      }
      // schedule: [B x4, A0] then per row {A next (+ B x4 of sub-step 1 at row 7), 4 MFMA}
#define G256_SG(mask, n) __builtin_amdgcn_sched_group_barrier(mask, n, 0)
#define G256_ROW(nr) G256_SG(0x100, nr); G256_SG(0x008, 4)
      G256_SG(0x100, 5);
      G256_ROW(1); G256_ROW(1); G256_ROW(1); G256_ROW(1);  // sub-step 0, rows 0-3
      G256_ROW(1); G256_ROW(1); G256_ROW(1); G256_ROW(5);  // rows 4-7 (+ next B)
      G256_ROW(1); G256_ROW(1); G256_ROW(1); G256_ROW(1);  // sub-step 1
      G256_ROW(1); G256_ROW(1); G256_ROW(1); G256_SG(0x008, 4);
#undef G256_ROW
#undef G256_SG
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c = ks * 4 + (lane >> 4);
        bf16x8 a[8], b[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = wc * 64 + j * 16 + (lane & 15);
          b[j] = *reinterpret_cast<const bf16x8*>(cur + TILE_BYTES + r * 128 + g256_swz(r, c) * 16);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int r = wr * 128 + i * 16 + (lane & 15);
          a[i] = *reinterpret_cast<const bf16x8*>(cur + r * 128 + g256_swz(r, c) * 16);
        }
        __builtin_amdgcn_s_setprio(1);  // MFMA cluster at raised priority (guide T5)
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next K-step has landed
    __syncthreads();                                   // ... and this one is read
  }
  // epilogue: C[m][n], m = m0 + wr*128 + i*16 + 4*(lane>>4) + r, n = n0 + wc*64 + j*16 + (lane&15)
  if (C && !Cf && (ldc & 7) == 0 && m0 + BM <= M && n0 + BN <= N) {
    // full bf16 tile: stage the 256 x 256 tile in the (now free) LDS, then 16-B stores
    // of whole 512-B rows (fragment-order stores would be 32-B row pieces)
    __bf16* st = reinterpret_cast<__bf16*>(smem);  // [256][256] bf16 = 128 KiB
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nl = wc * 64 + j * 16 + (lane & 15);
      const float bv = bias ? bias[n0 + nl] : 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ml = wr * 128 + i * 16 + 4 * (lane >> 4) + r;
          float v = acc[i][j][r] + bv;
          if (relu) v = v > 0.f ? v : 0.f;
          st[ml * BN + nl] = (__bf16)v;
        }
    }
    __syncthreads();
#pragma unroll 4
    for (int q = 0; q < BM * BN / 8 / TH; ++q) {  // 16 chunks of 8 bf16 per thread
      const int ch = q * TH + t;
      const int ml = ch >> 5, nc = (ch & 31) * 8;
      *reinterpret_cast<uint4*>(C + (int64_t)(m0 + ml) * ldc + n0 + nc) =
          *reinterpret_cast<const uint4*>(st + ml * BN + nc);
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wc * 64 + j * 16 + (lane & 15);
    if (n >= N) continue;
    const float bv = bias ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * 128 + i * 16 + 4 * (lane >> 4) + r;
        if (m >= M) continue;
        float v = acc[i][j][r] + bv;
        if (relu) v = v > 0.f ? v : 0.f;
        if (C) C[(int64_t)m * ldc + n] = (__bf16)v;
        if (Cf) Cf[(int64_t)m * ldcf + n] = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Ping-pong variant: the K-step is cut into 4 phases (one 64 x 32 C-quadrant of every
// wave each, 16 MFMAs), a phase into a LOAD interval (issue one half-tile of the next
// K-step's LDS-DMA, ds_read the quadrant's fragments, retire them) and an MFMA
// interval, each closed by a raw s_barrier. The second wave row (waves 4-7: one per
// SIMD next to a first-row wave) runs one barrier behind, so on every SIMD one wave
// issues MFMAs while the other loads. Half-tiles: A rows by quadrant row
// (mq0 = rows {0-63, 128-191}, mq1 = {64-127, 192-255}), B rows by quadrant column
// (nq0 = n % 64 < 32, nq1 = the rest); quadrant order (0,0) (0,1) (1,1) (1,0) keeps one
// A and one B fragment set live. DMA order of K-step t+1 during t: A-mq0, B-nq0,
// B-nq1, A-mq1; counted waits (vmcnt(4) at the end of phases 0, 1, 3: everything but
// the last two half-tiles) retire every half-tile at least one barrier before any wave
// reads it, and every LOAD interval retires its own ds_reads (lgkmcnt(0)) before its
// barrier, so a region is re-staged >= 3 barriers after its last read.
__device__ __forceinline__ void gpp_stage_a(const __bf16* __restrict__ p, int64_t ld, int rows,
                                            int r0, int k0, char* img, int mq, int wave,
                                            int lane) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int wi = q * 8 + wave;                                 // 0..15
    const int rowb = mq * 64 + (wi >> 3) * 128 + (wi & 7) * 8;  // first of 8 image rows
    const int row = rowb + (lane >> 3);
    const int c = g256_swz(row, lane & 7);
    int gr = r0 + row;
    gr = gr < rows ? gr : rows - 1;
    __builtin_amdgcn_global_load_lds((const void*)(p + (int64_t)gr * ld + k0 + c * 8),
                                     (__attribute__((address_space(3))) void*)(img + rowb * 128),
                                     16, 0, 0);
  }
}
__device__ __forceinline__ void gpp_stage_b(const __bf16* __restrict__ p, int64_t ld, int rows,
                                            int r0, int k0, char* img, int nq, int wave,
                                            int lane) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int wi = q * 8 + wave;                                 // 0..15
    const int rowb = (wi >> 2) * 64 + nq * 32 + (wi & 3) * 8;
    const int row = rowb + (lane >> 3);
    const int c = g256_swz(row, lane & 7);
    int gr = r0 + row;
    gr = gr < rows ? gr : rows - 1;
    __builtin_amdgcn_global_load_lds((const void*)(p + (int64_t)gr * ld + k0 + c * 8),
                                     (__attribute__((address_space(3))) void*)(img + rowb * 128),
                                     16, 0, 0);
  }
}

#define GPP_BAR() __builtin_amdgcn_s_barrier()

__global__ void __launch_bounds__(g256::TH)
gemm_nt256pp_kernel(const __bf16* __restrict__ A, int64_t lda, const __bf16* __restrict__ B,
                    int64_t ldb, int M, int N, int K, const float* __restrict__ bias, int relu,
                    __bf16* __restrict__ C, int64_t ldc, float* __restrict__ Cf, int64_t ldcf,
                    int tiles_n) {
  using namespace g256;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF_BYTES];  // 128 KiB, one array
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int id = g256_xcd(blockIdx.x, gridDim.x);
  const int tm = id / tiles_n, tn = id - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = K / BK;
  // prologue: K-step 0, every half-tile, then one full barrier
  gpp_stage_a(A, lda, M, m0, 0, smem, 0, wave, lane);
  gpp_stage_b(B, ldb, N, n0, 0, smem + TILE_BYTES, 0, wave, lane);
  gpp_stage_b(B, ldb, N, n0, 0, smem + TILE_BYTES, 1, wave, lane);
  gpp_stage_a(A, lda, M, m0, 0, smem, 1, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (wr == 1) GPP_BAR();  // the second wave row runs one barrier behind
  bf16x8 af[4][2], bf[2][2];
  for (int kt = 0; kt < nk; ++kt) {
    const char* cur = smem + (kt & 1) * BUF_BYTES;
    char* nxt = smem + ((kt + 1) & 1) * BUF_BYTES;
    const bool more = kt + 1 < nk;
    const int kn = (kt + 1) * BK;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int mq = (p == 0 || p == 1) ? 0 : 1;
      const int nq = (p == 1 || p == 2) ? 1 : 0;
      // ---- LOAD interval: one half-tile of K-step kt+1, this quadrant's fragments
      if (more) {
        if (p == 0) gpp_stage_a(A, lda, M, m0, kn, nxt, 0, wave, lane);
        if (p == 1) gpp_stage_b(B, ldb, N, n0, kn, nxt + TILE_BYTES, 0, wave, lane);
        if (p == 2) gpp_stage_b(B, ldb, N, n0, kn, nxt + TILE_BYTES, 1, wave, lane);
        if (p == 3) gpp_stage_a(A, lda, M, m0, kn, nxt, 1, wave, lane);
      }
      if (p != 2) {  // B fragments of column quadrant nq (p2 reuses p1's)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int c = ks * 4 + (lane >> 4);
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const int r = wc * 64 + nq * 32 + j * 16 + (lane & 15);
            bf[ks][j] = *reinterpret_cast<const bf16x8*>(cur + TILE_BYTES + r * 128 +
                                                          g256_swz(r, c) * 16);
          }
        }
      }
      if (p == 0 || p == 2) {  // A fragments of row quadrant mq (p1 / p3 reuse them)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int c = ks * 4 + (lane >> 4);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int r = wr * 128 + mq * 64 + i * 16 + (lane & 15);
            af[i][ks] = *reinterpret_cast<const bf16x8*>(cur + r * 128 + g256_swz(r, c) * 16);
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (p != 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      GPP_BAR();
      // ---- MFMA interval
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[mq][nq][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][ks], bf[ks][j],
                                                                       acc[mq][nq][i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      GPP_BAR();
    }
  }
  if (wr == 0) GPP_BAR();  // match the second row's extra barrier
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  // epilogue: quadrant (mq, nq), tile (i, j): m = wr*128 + mq*64 + i*16 + 4(lane>>4) + r,
  // n = wc*64 + nq*32 + j*16 + (lane&15)
  if (C && !Cf && (ldc & 7) == 0 && m0 + BM <= M && n0 + BN <= N) {
    __bf16* st = reinterpret_cast<__bf16*>(smem);  // [256][256] bf16
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int nl = wc * 64 + nq * 32 + j * 16 + (lane & 15);
        const float bv = bias ? bias[n0 + nl] : 0.f;
#pragma unroll
        for (int mq = 0; mq < 2; ++mq)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int ml = wr * 128 + mq * 64 + i * 16 + 4 * (lane >> 4) + r;
              float v = acc[mq][nq][i][j][r] + bv;
              if (relu) v = v > 0.f ? v : 0.f;
              st[ml * BN + nl] = (__bf16)v;
            }
      }
    __syncthreads();
#pragma unroll 4
    for (int q = 0; q < BM * BN / 8 / TH; ++q) {
      const int ch = q * TH + t;
      const int ml = ch >> 5, nc = (ch & 31) * 8;
      *reinterpret_cast<uint4*>(C + (int64_t)(m0 + ml) * ldc + n0 + nc) =
          *reinterpret_cast<const uint4*>(st + ml * BN + nc);
    }
    return;
  }
#pragma unroll
  for (int nq = 0; nq < 2; ++nq)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wc * 64 + nq * 32 + j * 16 + (lane & 15);
      if (n >= N) continue;
      const float bv = bias ? bias[n] : 0.f;
#pragma unroll
      for (int mq = 0; mq < 2; ++mq)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = m0 + wr * 128 + mq * 64 + i * 16 + 4 * (lane >> 4) + r;
            if (m >= M) continue;
            float v = acc[mq][nq][i][j][r] + bv;
            if (relu) v = v > 0.f ? v : 0.f;
            if (C) C[(int64_t)m * ldc + n] = (__bf16)v;
            if (Cf) Cf[(int64_t)m * ldcf + n] = v;
          }
    }
}
#undef GPP_BAR

// ---------------------------------------------------------------------------
// Deep-prefetch variant (variant 2): the ping-pong structure above, but each half-tile
// region is re-staged for K-step t+2 as soon as its last read of K-step t retired, so
// every half-tile has ~7 phases (instead of 4) between its DMA and its first read. Reads
// per K-step: p0 A-mq0 + B-nq0 (the B-nq0 fragments stay in registers for p3), p1
// B-nq1, p2 A-mq1, p3 none; stages during K-step t (into the same buffer, K-step t+2):
// p1 A-mq0 + B-nq0, p2 B-nq1, p3 A-mq1. Counted waits (per wave, glds in issue order:
// A0B0 = 4, B1 = 2, A1 = 2 per K-step): p3(t) retires A0B0(t+1) (12 younger), p0(t)
// retires B1(t) (10 younger), p1(t) retires A1(t) (12 younger); each read follows its
// wait by at least one barrier of both wave rows (the second row runs one barrier
// behind), and each region is re-staged a phase after its last read was retired
// (lgkmcnt(0)) before a barrier both rows have passed.
#define GP8_BAR() __builtin_amdgcn_s_barrier()
#define GP8_VM(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

__global__ void __launch_bounds__(g256::TH)
gemm_nt256p8_kernel(const __bf16* __restrict__ A, int64_t lda, const __bf16* __restrict__ B,
                    int64_t ldb, int M, int N, int K, const float* __restrict__ bias, int relu,
                    __bf16* __restrict__ C, int64_t ldc, float* __restrict__ Cf, int64_t ldcf,
                    int tiles_n) {
  using namespace g256;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF_BYTES];  // 128 KiB, one array
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int id = g256_xcd(blockIdx.x, gridDim.x);
  const int tm = id / tiles_n, tn = id - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = K / BK;
  // prologue: K-steps 0 and 1, each in the steady-state order A0 B0 | B1 | A1
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    if (kt < nk) {
      char* buf = smem + kt * BUF_BYTES;
      gpp_stage_a(A, lda, M, m0, kt * BK, buf, 0, wave, lane);
      gpp_stage_b(B, ldb, N, n0, kt * BK, buf + TILE_BYTES, 0, wave, lane);
      gpp_stage_b(B, ldb, N, n0, kt * BK, buf + TILE_BYTES, 1, wave, lane);
      gpp_stage_a(A, lda, M, m0, kt * BK, buf, 1, wave, lane);
    }
  }
  if (nk > 1) GP8_VM(12); else GP8_VM(4);  // A0B0(0) landed
  GP8_BAR();
  if (wr == 1) GP8_BAR();  // the second wave row runs one barrier behind
  bf16x8 af[4][2], bf0[2][2], bf1[2][2];
  for (int kt = 0; kt < nk; ++kt) {
    char* cur = smem + (kt & 1) * BUF_BYTES;
    const bool s2 = kt + 2 < nk, s1 = kt + 1 < nk;
    const int k2 = (kt + 2) * BK;
    // ---- p0: read A-mq0, B-nq0; retire B1(kt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + (lane >> 4);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = wc * 64 + j * 16 + (lane & 15);
        bf0[ks][j] = *reinterpret_cast<const bf16x8*>(cur + TILE_BYTES + r * 128 + g256_swz(r, c) * 16);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wr * 128 + i * 16 + (lane & 15);
        af[i][ks] = *reinterpret_cast<const bf16x8*>(cur + r * 128 + g256_swz(r, c) * 16);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (s1) GP8_VM(10); else GP8_VM(2);
    GP8_BAR();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[0][0][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][ks], bf0[ks][j],
                                                                   acc[0][0][i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    GP8_BAR();
    // ---- p1: stage A0 B0 (kt+2); read B-nq1; retire A1(kt)
    if (s2) {
      gpp_stage_a(A, lda, M, m0, k2, cur, 0, wave, lane);
      gpp_stage_b(B, ldb, N, n0, k2, cur + TILE_BYTES, 0, wave, lane);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + (lane >> 4);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = wc * 64 + 32 + j * 16 + (lane & 15);
        bf1[ks][j] = *reinterpret_cast<const bf16x8*>(cur + TILE_BYTES + r * 128 + g256_swz(r, c) * 16);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (s2) GP8_VM(12); else if (s1) GP8_VM(8); else GP8_VM(0);
    GP8_BAR();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[0][1][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][ks], bf1[ks][j],
                                                                   acc[0][1][i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    GP8_BAR();
    // ---- p2: stage B1 (kt+2); read A-mq1
    if (s2) gpp_stage_b(B, ldb, N, n0, k2, cur + TILE_BYTES, 1, wave, lane);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wr * 128 + 64 + i * 16 + (lane & 15);
        af[i][ks] = *reinterpret_cast<const bf16x8*>(cur + r * 128 + g256_swz(r, c) * 16);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    GP8_BAR();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[1][1][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][ks], bf1[ks][j],
                                                                   acc[1][1][i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    GP8_BAR();
    // ---- p3: stage A1 (kt+2); no reads; retire A0B0(kt+1)
    if (s2) gpp_stage_a(A, lda, M, m0, k2, cur, 1, wave, lane);
    if (s2) GP8_VM(12); else if (s1) GP8_VM(4);
    GP8_BAR();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[1][0][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][ks], bf0[ks][j],
                                                                   acc[1][0][i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    GP8_BAR();
  }
  if (wr == 0) GP8_BAR();  // match the second row's extra barrier
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  if (C && !Cf && (ldc & 7) == 0 && m0 + BM <= M && n0 + BN <= N) {
    __bf16* st = reinterpret_cast<__bf16*>(smem);  // [256][256] bf16
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int nl = wc * 64 + nq * 32 + j * 16 + (lane & 15);
        const float bv = bias ? bias[n0 + nl] : 0.f;
#pragma unroll
        for (int mq = 0; mq < 2; ++mq)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int ml = wr * 128 + mq * 64 + i * 16 + 4 * (lane >> 4) + r;
              float v = acc[mq][nq][i][j][r] + bv;
              if (relu) v = v > 0.f ? v : 0.f;
              st[ml * BN + nl] = (__bf16)v;
            }
      }
    __syncthreads();
#pragma unroll 4
    for (int q = 0; q < BM * BN / 8 / TH; ++q) {
      const int ch = q * TH + t;
      const int ml = ch >> 5, nc = (ch & 31) * 8;
      *reinterpret_cast<uint4*>(C + (int64_t)(m0 + ml) * ldc + n0 + nc) =
          *reinterpret_cast<const uint4*>(st + ml * BN + nc);
    }
    return;
  }
#pragma unroll
  for (int nq = 0; nq < 2; ++nq)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wc * 64 + nq * 32 + j * 16 + (lane & 15);
      if (n >= N) continue;
      const float bv = bias ? bias[n] : 0.f;
#pragma unroll
      for (int mq = 0; mq < 2; ++mq)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = m0 + wr * 128 + mq * 64 + i * 16 + 4 * (lane >> 4) + r;
            if (m >= M) continue;
            float v = acc[mq][nq][i][j][r] + bv;
            if (relu) v = v > 0.f ? v : 0.f;
            if (C) C[(int64_t)m * ldc + n] = (__bf16)v;
            if (Cf) Cf[(int64_t)m * ldcf + n] = v;
          }
    }
}
#undef GP8_BAR
#undef GP8_VM

// ---------------------------------------------------------------------------
// "TN" 256 x 256 kernel for MN-major operands (the weight gradient dW = dZ^T X of a
// linear layer: both operands are [batch][features] with the reduction over the batch
// rows):
//
//   P[split][m][n] = sum_{k in the split} A[k * lda + m] * B[k * ldb + n]   (fp32)
//
// Same geometry as gemm_nt256_kernel (8 waves as 2 x 4, a wave owns 128 x 64, 64
// v_mfma_f32_16x16x32_bf16 per K-step, LDS-DMA double buffer, one counted wait + one
// barrier per K-step), but a tile is staged as it lies in memory, [64 k][256 m] with
// 512-B k-rows, and the MFMA fragments (8 consecutive k of one m per lane) come out of
// it with ds_read_b64_tr_b16: per 16-lane group, lane 4q+p addresses row q, columns
// 4p..4p+3 of a 4-row x 16-column block, and lane i receives column i of the 4 rows
// (guide T10); two reads give the 8 k of a fragment. The 16-B chunk c of k-row r sits
// at chunk c ^ f(r), f(r) = 2 (r & 3) + 8 ((r >> 3) & 1): the 8 rows a 32-lane half reads
// (two groups 8 rows apart) then cover all 64 banks (conflict-free). LDS-DMA writes
// lane-linear, so the swizzle is applied to the per-lane global source address.
// K is split over gridDim.y (K-steps shared out evenly, so any split count): every split
// writes its own fp32 partial tile (no atomics), gemm_splitk_reduce sums them in a fixed
// order. Requirements (binding): M, N multiples of 8, K a multiple of 64 with >= 1 K-step
// per split, 16-B aligned operands, lda / ldb multiples of 8.
__device__ __forceinline__ int gtn_swz(int r) { return ((r & 3) << 1) | (((r >> 3) & 1) << 3); }

// LDS-DMA of a [64 k][256 cols] tile (k rows k0.., columns c0..) into dst: wave
// instruction wi fills k-rows 2wi, 2wi+1 (lane l: row 2wi + l/32, chunk position l%32).
__device__ __forceinline__ void gtn_stage(const __bf16* __restrict__ p, int64_t ld, int cols,
                                          int c0, int k0, char* dst, int wave, int lane) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int wi = q * 8 + wave;
    const int r = 2 * wi + (lane >> 5);
    const int c = (lane & 31) ^ gtn_swz(r);
    int col = c0 + c * 8;
    col = col + 8 <= cols ? col : cols - 8;  // (clamped; the stores mask it)
    const __bf16* src = p + (int64_t)(k0 + r) * ld + col;
    __builtin_amdgcn_global_load_lds((const void*)src,
                                     (__attribute__((address_space(3))) void*)(dst + wi * 1024),
                                     16, 0, 0);
  }
}

typedef short gtn_s4 __attribute__((ext_vector_type(4)));

// one transposed read: 4 bf16 (k rows kr..kr+3) of column (cb + lane's i) of the image
__device__ __forceinline__ gtn_s4 gtn_tr(const char* img, int kr, int cb, int lane) {
  const int q = (lane & 15) >> 2, p = lane & 3;
  const int r = kr + q;
  const int col = cb + 4 * p;  // first of the 4 columns this lane addresses
  const int c = (col >> 3) ^ gtn_swz(r);
  const char* a = img + r * 512 + c * 16 + (col & 7) * 2;
  // (the builtin, not inline asm: the compiler then counts the read's lgkmcnt itself)
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) gtn_s4*)(const __attribute__((address_space(3))) char*)a);
}

__global__ void __launch_bounds__(g256::TH)
gemm_tn256_kernel(const __bf16* __restrict__ A, int64_t lda, const __bf16* __restrict__ B,
                  int64_t ldb, int M, int N, int K, float* P, int tiles_n,
                  float* __restrict__ Out, float beta, unsigned int* tile_ctr) {
  using namespace g256;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF_BYTES];  // 128 KiB
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wr = wave >> 2, wc = wave & 3;
  const int id = g256_xcd(blockIdx.x, gridDim.x);
  const int tm = id / tiles_n, tn = id - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  // split y of S takes K-steps [y * NK / S, (y+1) * NK / S) (any S: uneven by one step)
  const int NK = K / BK, S = gridDim.y;
  const int ks0 = (int)((int64_t)blockIdx.y * NK / S), ks1 = (int)((int64_t)(blockIdx.y + 1) * NK / S);
  const int kb = ks0 * BK;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = ks1 - ks0;
  gtn_stage(A, lda, M, m0, kb, smem, wave, lane);
  gtn_stage(B, ldb, N, n0, kb, smem + TILE_BYTES, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int g = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const char* cur = smem + (kt & 1) * BUF_BYTES;
    if (kt + 1 < nk) {
      char* nxt = smem + ((kt + 1) & 1) * BUF_BYTES;
      gtn_stage(A, lda, M, m0, kb + (kt + 1) * BK, nxt, wave, lane);
      gtn_stage(B, ldb, N, n0, kb + (kt + 1) * BK, nxt + TILE_BYTES, wave, lane);
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int kr = ks * 32 + 8 * g;
      bf16x8 a[8], b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cb = wc * 64 + j * 16;
        const gtn_s4 lo = gtn_tr(cur + TILE_BYTES, kr, cb, lane);
        const gtn_s4 hi = gtn_tr(cur + TILE_BYTES, kr + 4, cb, lane);
        b[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int cb = wr * 128 + i * 16;
        const gtn_s4 lo = gtn_tr(cur, kr, cb, lane);
        const gtn_s4 hi = gtn_tr(cur, kr + 4, cb, lane);
        a[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next K-step has landed
    __syncthreads();                                   // ... and this one is read
  }
  // C[m][n]: m = m0 + wr*128 + i*16 + 4*(lane>>4) + r, n = n0 + wc*64 + j*16 + (lane&15)
  float* out = P + (int64_t)blockIdx.y * M * N;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wc * 64 + j * 16 + (lane & 15);
    if (n >= N) continue;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * 128 + i * 16 + 4 * (lane >> 4) + r;
        if (m < M) out[(int64_t)m * N + n] = acc[i][j][r];
      }
  }
  if (!tile_ctr) return;
  // in-kernel split-K reduce (tile_ctr given): the last of the tile's S splits to finish
  // (a per-tile counter it resets) sums the S partials in split order -- its own from
  // registers -- onto beta * Out: the arithmetic and order of gemm_splitk_reduce, so the
  // result is bitwise that of the two-launch form, without the separate memory pass
  __shared__ unsigned int last;
  __threadfence();  // this split's partial visible device-wide before it counts
  __syncthreads();
  if (t == 0) {
    const unsigned int prev = atomicAdd(tile_ctr + id, 1u);
    last = prev == (unsigned)S - 1;
    if (last) tile_ctr[id] = 0;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  const int me = blockIdx.y;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wc * 64 + j * 16 + (lane & 15);
    if (n >= N) continue;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * 128 + i * 16 + 4 * (lane >> 4) + r;
        if (m >= M) continue;
        const int64_t o = (int64_t)m * N + n;
        float a = beta != 0.f ? Out[o] : 0.f;
        if (beta != 0.f && beta != 1.f) a *= beta;
        for (int q = 0; q < S; ++q)
          a += q == me ? acc[i][j][r]
                       : __hip_atomic_load(P + (int64_t)q * M * N + o, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
        Out[o] = a;
      }
  }
}

// out[i] = beta * out[i] + sum over the S partials (fixed order: deterministic)
__global__ void __launch_bounds__(256)
gemm_splitk_reduce_kernel(const float4* __restrict__ P, int S, int64_t n4, float4* __restrict__ out,
                          float beta) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    float4 a = beta != 0.f ? out[i] : float4{0.f, 0.f, 0.f, 0.f};
    if (beta != 0.f && beta != 1.f) a = float4{a.x * beta, a.y * beta, a.z * beta, a.w * beta};
    for (int s = 0; s < S; ++s) {
      const float4 v = P[(int64_t)s * n4 + i];
      a.x += v.x;
      a.y += v.y;
      a.z += v.z;
      a.w += v.w;
    }
    out[i] = a;
  }
}

// phase: 0 = GEMM + split-K reduce, 1 = the GEMM into `part` only, 2 = the reduce only
// (a caller can hold the reduce back so that a later GEMM is not queued behind it)
void gemm_tn256(const __bf16* A, int64_t lda, const __bf16* B, int64_t ldb, int M, int N, int K,
                int splits, float* part, float* out, float beta, int phase, unsigned int* tile_ctr,
                hipStream_t st) {
  if (M <= 0 || N <= 0) return;
  if (splits < 1 || K % g256::BK != 0 || K / g256::BK < splits || M % 8 || N % 8 || lda % 8 ||
      ldb % 8)
    throw std::runtime_error("gemm_tn256: K % 64, K / 64 >= splits, M / N / ld % 8");
  const int tiles_m = (M + g256::BM - 1) / g256::BM, tiles_n = (N + g256::BN - 1) / g256::BN;
  dim3 grid(tiles_m * tiles_n, splits);
  // phase 3: the reduce inside the GEMM's last split per tile (tile_ctr: tiles_m x tiles_n
  // zeroed counters, left zeroed)
  if (phase == 3 && splits == 1) phase = 0;
  if (phase != 2) {
    gemm_tn256_kernel<<<grid, g256::TH, 0, st>>>(A, lda, B, ldb, M, N, K, part, tiles_n,
                                                 phase == 3 ? out : nullptr, beta,
                                                 phase == 3 ? tile_ctr : nullptr);
    PSAMD_HIP_CHECK(hipGetLastError());
  }
  if (phase == 1 || phase == 3) return;
  const int64_t n4 = (int64_t)M * N / 4;
  gemm_splitk_reduce_kernel<<<grid_for(n4, 256, 4096), 256, 0, st>>>(
      reinterpret_cast<const float4*>(part), splits, n4, reinterpret_cast<float4*>(out), beta);
  PSAMD_HIP_CHECK(hipGetLastError());
}

// out [C, R] = in [R, C]^T, bf16, R and C multiples of 64: a 64 x 64 tile through LDS
// (rows padded by 8 elements), 16-B loads and stores. The weight copy W^T that lets the
// input gradient dZ W run on the K-major 256 x 256 kernel (torch's strided copy took
// ~50 us for 1024 x 4992).
__global__ void __launch_bounds__(256)
transpose_bf16_kernel(const uint16_t* __restrict__ in, int R, int C, uint16_t* __restrict__ out) {
  __shared__ uint16_t tile[64][72];
  const int t = threadIdx.x;
  const int tc = blockIdx.x % (C / 64), tr = blockIdx.x / (C / 64);
  const int r0 = tr * 64, c0 = tc * 64;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int idx = q * 256 + t, r = idx >> 3, ch = idx & 7;
    const uint4 v = *reinterpret_cast<const uint4*>(in + (int64_t)(r0 + r) * C + c0 + ch * 8);
    *reinterpret_cast<uint4*>(&tile[r][ch * 8]) = v;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int idx = q * 256 + t, j = idx >> 3, ch = idx & 7;  // output row j = input col
    uint16_t h[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) h[e] = tile[ch * 8 + e][j];
    uint4 v;
    v.x = h[0] | ((uint32_t)h[1] << 16);
    v.y = h[2] | ((uint32_t)h[3] << 16);
    v.z = h[4] | ((uint32_t)h[5] << 16);
    v.w = h[6] | ((uint32_t)h[7] << 16);
    *reinterpret_cast<uint4*>(out + (int64_t)(c0 + j) * R + r0 + ch * 8) = v;
  }
}

void transpose_bf16(const void* in, int R, int C, void* out, hipStream_t st) {
  if (R <= 0 || C <= 0) return;
  if (R % 64 || C % 64) throw std::runtime_error("transpose_bf16: R, C multiples of 64");
  transpose_bf16_kernel<<<(unsigned)((R / 64) * (C / 64)), 256, 0, st>>>(
      (const uint16_t*)in, R, C, (uint16_t*)out);
  PSAMD_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// Ring variant (variant 4): K-steps of 32 through a 4-slot LDS ring (4 x 32 KiB: A | B
// of 256 rows x 64 B), the DMA of K-step p+3 issued while K-step p is read, so a
// K-step has ~4-5 barrier intervals (2-3 MFMA segments of 512 cycles) between its
// DMA and its first read. Per K-step a wave has a READ interval (its 8 A + 4 B
// fragments, its 4 LDS-DMA instructions of K-step p+3, lgkmcnt(0)) and an MFMA
// interval (the 32 MFMAs of its 128 x 64 output), each closed by a raw s_barrier; the
// second wave row (waves 4-7, one beside each first-row wave on its SIMD) runs one
// barrier behind, so every SIMD alternates the two waves' 512-cycle MFMA runs while
// the other wave reads (twice the MFMA run of the 16-MFMA quadrant phases of
// variants 1-2: half the barriers per FLOP). Ordering, by global barrier index
// (row 0's K-step p: read interval 2p, MFMA interval 2p+1; row 1's one later):
// * RAW: every wave waits for its share of K-step p+1 (vmcnt counting the younger
//   DMAs of K-steps p+2, p+3) before barrier 2p+1, the barrier before its first read;
// * WAR: slot (p+3) % 4 held K-step p-1, whose reads each row retired (lgkmcnt(0))
//   before the barrier closing its read interval (2p-2, 2p-1); its DMA is issued after
//   barrier 2p-1 (row 0 in interval 2p, row 1 in 2p+1).
// LDS row image: 64-B rows, 16-B chunk c of row r at c ^ ((r >> 2) & 3) (a
// ds_read_b128 lane group, rows r..r+15 of one chunk, covers all 64 banks); the
// swizzle goes on the DMA's per-lane global source (the LDS-DMA writes lane-linear).
namespace g256r {
constexpr int BK = 32, NSLOT = 4;
constexpr int OP_BYTES = 256 * BK * 2;   // 16 KiB per operand per K-step
constexpr int SLOT_BYTES = 2 * OP_BYTES; // A | B
}  // namespace g256r

__device__ __forceinline__ int g256r_swz(int r, int c) { return c ^ ((r >> 2) & 3); }

// this wave's 4 DMA instructions of a K-step: wi = q*8 + wave, 0-15 A rows 16 wi.., 16-31 B
__device__ __forceinline__ void g256r_stage(const __bf16* __restrict__ A, int64_t lda, int M,
                                            const __bf16* __restrict__ B, int64_t ldb, int N,
                                            int m0, int n0, int k0, char* slot, int wave,
                                            int lane) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int wi = q * 8 + wave;
    const bool isb = wi >= 16;  // (q >= 2: wave-uniform)
    const int rowb = (wi & 15) * 16;
    const int row = rowb + (lane >> 2);
    const int c = g256r_swz(row, lane & 3);
    const __bf16* p = isb ? B : A;
    const int64_t ld = isb ? ldb : lda;
    const int lim = isb ? N : M;
    int gr = (isb ? n0 : m0) + row;
    gr = gr < lim ? gr : lim - 1;
    __builtin_amdgcn_global_load_lds(
        (const void*)(p + (int64_t)gr * ld + k0 + c * 8),
        (__attribute__((address_space(3))) void*)(slot + (isb ? g256r::OP_BYTES : 0) + rowb * 64),
        16, 0, 0);
  }
}

#define G256R_VMCNT(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
// wait for this wave's DMA of K-step p+1 (younger: those of K-steps p+2 .. min(p+3, nk-1))
#define G256R_WAIT_NEXT(p, nk)                    \
  do {                                            \
    const int y_ = min((p) + 3, (nk) - 1) - ((p) + 1); \
    if (y_ >= 2) G256R_VMCNT(8);                  \
    else if (y_ == 1) G256R_VMCNT(4);             \
    else G256R_VMCNT(0);                          \
  } while (0)

__global__ void __launch_bounds__(g256::TH)
gemm_nt256r_kernel(const __bf16* __restrict__ A, int64_t lda, const __bf16* __restrict__ B,
                   int64_t ldb, int M, int N, int K, const float* __restrict__ bias, int relu,
                   __bf16* __restrict__ C, int64_t ldc, float* __restrict__ Cf, int64_t ldcf,
                   int tiles_n) {
  using namespace g256;
  __shared__ __attribute__((aligned(16))) char smem[g256r::NSLOT * g256r::SLOT_BYTES];  // 128 KiB
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int id = g256_xcd(blockIdx.x, gridDim.x);
  const int tm = id / tiles_n, tn = id - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = K / g256r::BK;
  // prologue: K-steps 0..2 in flight, K-step 0 landed everywhere before barrier -1
  for (int p = 0; p < 3 && p < nk; ++p)
    g256r_stage(A, lda, M, B, ldb, N, m0, n0, p * g256r::BK, smem + p * g256r::SLOT_BYTES, wave,
                lane);
  if (nk >= 3) G256R_VMCNT(8);
  else if (nk == 2) G256R_VMCNT(4);
  else G256R_VMCNT(0);
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // the second wave row runs one barrier behind
  const int c = lane >> 4;
  for (int p = 0; p < nk; ++p) {
    const char* cur = smem + (p & 3) * g256r::SLOT_BYTES;
    // ---- READ interval
    bf16x8 a[8], b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = wc * 64 + j * 16 + (lane & 15);
      b[j] = *reinterpret_cast<const bf16x8*>(cur + g256r::OP_BYTES + r * 64 + g256r_swz(r, c) * 16);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = wr * 128 + i * 16 + (lane & 15);
      a[i] = *reinterpret_cast<const bf16x8*>(cur + r * 64 + g256r_swz(r, c) * 16);
    }
    if (p + 3 < nk)
      g256r_stage(A, lda, M, B, ldb, N, m0, n0, (p + 3) * g256r::BK,
                  smem + ((p + 3) & 3) * g256r::SLOT_BYTES, wave, lane);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (wr == 1) G256R_WAIT_NEXT(p, nk);
    __builtin_amdgcn_s_barrier();
    // ---- MFMA interval
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    if (wr == 0) G256R_WAIT_NEXT(p, nk);
    __builtin_amdgcn_s_barrier();
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // match the second row's extra barrier
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  // epilogue (as gemm_nt256_kernel): m = m0 + wr*128 + i*16 + 4*(lane>>4) + r,
  // n = n0 + wc*64 + j*16 + (lane&15)
  if (C && !Cf && (ldc & 7) == 0 && m0 + BM <= M && n0 + BN <= N) {
    __bf16* st = reinterpret_cast<__bf16*>(smem);  // [256][256] bf16 = 128 KiB
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int nl = wc * 64 + j * 16 + (lane & 15);
      const float bv = bias ? bias[n0 + nl] : 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ml = wr * 128 + i * 16 + 4 * (lane >> 4) + r;
          float v = acc[i][j][r] + bv;
          if (relu) v = v > 0.f ? v : 0.f;
          st[ml * BN + nl] = (__bf16)v;
        }
    }
    __syncthreads();
#pragma unroll 4
    for (int q = 0; q < BM * BN / 8 / TH; ++q) {
      const int ch = q * TH + t;
      const int ml = ch >> 5, nc = (ch & 31) * 8;
      *reinterpret_cast<uint4*>(C + (int64_t)(m0 + ml) * ldc + n0 + nc) =
          *reinterpret_cast<const uint4*>(st + ml * BN + nc);
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wc * 64 + j * 16 + (lane & 15);
    if (n >= N) continue;
    const float bv = bias ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * 128 + i * 16 + 4 * (lane >> 4) + r;
        if (m >= M) continue;
        float v = acc[i][j][r] + bv;
        if (relu) v = v > 0.f ? v : 0.f;
        if (C) C[(int64_t)m * ldc + n] = (__bf16)v;
        if (Cf) Cf[(int64_t)m * ldcf + n] = v;
      }
    }
  }
}
// ---------------------------------------------------------------------------
// 32x32x16 ring variant (variant 6): variant 4's LDS ring, barriers and wave layout, the
// 128 x 64 wave tile as 4 x 2 v_mfma_f32_32x32x16_bf16 tiles (lane l: A[row l&31][k 8(l>>5)
// ..+7] of a 16-k sub-step, B likewise; C col l&31, rows (r&3) + 8(r>>2) + 4(l>>5)):
// 16 MFMAs of 32 cycles per K-step instead of 32 of 16. The LDS traffic per K-step is
// unchanged (the wave tile fixes it: 8 A + 4 B ds_read_b128), so the variant trades
// issue slots only; the guide's bare-loop measurement puts 32x32x16 at ~0.87x the
// FLOP/s of 16x16x32 (MI355X_MICROARCH.md, "bare bf16 MFMA loops").
// Measured (profiles/r5_gemm_32x32.log): correct, slower than variant 4 on every W&D
// shape (1199 vs 1306 TFLOP/s on 16384 x 1024 x 4992, 782 vs 819 on the dX product).
// Kept for A/B.
__global__ void __launch_bounds__(g256::TH)
gemm_nt256r32_kernel(const __bf16* __restrict__ A, int64_t lda, const __bf16* __restrict__ B,
                   int64_t ldb, int M, int N, int K, const float* __restrict__ bias, int relu,
                   __bf16* __restrict__ C, int64_t ldc, float* __restrict__ Cf, int64_t ldcf,
                   int tiles_n) {
  using namespace g256;
  __shared__ __attribute__((aligned(16))) char smem[g256r::NSLOT * g256r::SLOT_BYTES];  // 128 KiB
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int id = g256_xcd(blockIdx.x, gridDim.x);
  const int tm = id / tiles_n, tn = id - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int nk = K / g256r::BK;
  // prologue: K-steps 0..2 in flight, K-step 0 landed everywhere before barrier -1
  for (int p = 0; p < 3 && p < nk; ++p)
    g256r_stage(A, lda, M, B, ldb, N, m0, n0, p * g256r::BK, smem + p * g256r::SLOT_BYTES, wave,
                lane);
  if (nk >= 3) G256R_VMCNT(8);
  else if (nk == 2) G256R_VMCNT(4);
  else G256R_VMCNT(0);
  __builtin_amdgcn_s_barrier();
  if (wr == 1) __builtin_amdgcn_s_barrier();  // the second wave row runs one barrier behind
  const int h = lane >> 5;  // k half of a 16-k sub-step
  for (int p = 0; p < nk; ++p) {
    const char* cur = smem + (p & 3) * g256r::SLOT_BYTES;
    // ---- READ interval: per 16-k sub-step ks, chunk 2 ks + h of rows (lane & 31)
    bf16x8 a[4][2], b[2][2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = 2 * ks + h;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = wc * 64 + j * 32 + (lane & 31);
        b[j][ks] = *reinterpret_cast<const bf16x8*>(cur + g256r::OP_BYTES + r * 64 +
                                                    g256r_swz(r, c) * 16);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = wr * 128 + i * 32 + (lane & 31);
        a[i][ks] = *reinterpret_cast<const bf16x8*>(cur + r * 64 + g256r_swz(r, c) * 16);
      }
    }
    if (p + 3 < nk)
      g256r_stage(A, lda, M, B, ldb, N, m0, n0, (p + 3) * g256r::BK,
                  smem + ((p + 3) & 3) * g256r::SLOT_BYTES, wave, lane);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (wr == 1) G256R_WAIT_NEXT(p, nk);
    __builtin_amdgcn_s_barrier();
    // ---- MFMA interval
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i][ks], b[j][ks], acc[i][j], 0, 0,
                                                              0);
    __builtin_amdgcn_s_setprio(0);
    if (wr == 0) G256R_WAIT_NEXT(p, nk);
    __builtin_amdgcn_s_barrier();
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // match the second row's extra barrier
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  // epilogue: m = m0 + wr*128 + i*32 + (r&3) + 8*(r>>2) + 4*(lane>>5),
  // n = n0 + wc*64 + j*32 + (lane&31)
  if (C && !Cf && (ldc & 7) == 0 && m0 + BM <= M && n0 + BN <= N) {
    __bf16* st = reinterpret_cast<__bf16*>(smem);  // [256][256] bf16 = 128 KiB
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int nl = wc * 64 + j * 32 + (lane & 31);
      const float bv = bias ? bias[n0 + nl] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ml = wr * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          float v = acc[i][j][r] + bv;
          if (relu) v = v > 0.f ? v : 0.f;
          st[ml * BN + nl] = (__bf16)v;
        }
    }
    __syncthreads();
#pragma unroll 4
    for (int q = 0; q < BM * BN / 8 / TH; ++q) {
      const int ch = q * TH + t;
      const int ml = ch >> 5, nc = (ch & 31) * 8;
      *reinterpret_cast<uint4*>(C + (int64_t)(m0 + ml) * ldc + n0 + nc) =
          *reinterpret_cast<const uint4*>(st + ml * BN + nc);
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wc * 64 + j * 32 + (lane & 31);
    if (n >= N) continue;
    const float bv = bias ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wr * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= M) continue;
        float v = acc[i][j][r] + bv;
        if (relu) v = v > 0.f ? v : 0.f;
        if (C) C[(int64_t)m * ldc + n] = (__bf16)v;
        if (Cf) Cf[(int64_t)m * ldcf + n] = v;
      }
    }
  }
}
#undef G256R_WAIT_NEXT
#undef G256R_VMCNT

// ---------------------------------------------------------------------------
// Four-wave variant (variant 5): 256 threads = 4 waves as 2 (M) x 2 (N), ONE wave per
// SIMD, each owning a 128 x 128 output = 8 x 8 v_mfma_f32_16x16x32_bf16 tiles (256
// accumulator registers per lane: the unified VGPR/AGPR file of a 1-wave-per-SIMD
// kernel). Per K-step of 64 a wave reads 8 A + 8 B fragments per sub-step of 32 (32
// ds_read_b128 for 128 MFMAs: a third fewer LDS bytes per FLOP than the 8-wave 128 x 64
// layout, 128 KiB of fragment reads + 64 KiB of DMA per CU per K-step against 2048
// MFMA cycles per SIMD). Same LDS image / DMA / swizzle as gemm_nt256_kernel (two 64 KiB
// buffers). A single wave per SIMD hides its own latency by software pipelining:
//   K-step kt: DMA of kt+1 (into the buffer K-step kt-1 used: every wave retired its
//   reads of it before barrier kt-1); sub-step 1 fragments of kt in flight during the
//   64 MFMAs of sub-step 0; the first 32 MFMAs of sub-step 1; then vmcnt(0) (this wave's
//   DMA of kt+1 landed) + barrier kt, and sub-step 0 fragments of kt+1 in flight during
//   the last 32 MFMAs of kt.
// Measured (profiles/r5_gemm_w4.log): correct but the slowest variant, 1000 vs 1306
// (variant 4) vs 1438 (hipBLASLt) TFLOP/s on 16384 x 1024 x 4992: as compiled, the
// 256 VGPRs hold the fragments plus every hoisted DMA / LDS address and the loop moves
// 72 registers between the AGPR and VGPR halves per K-step. Kept for A/B.
namespace g256w {
constexpr int TH = 256, NW = 4;
}

// LDS-DMA of one 256 x 64 operand tile by 4 waves: wave-instruction wi = q*4 + wave
// fills rows wi*8 .. wi*8+7 (bytes [wi*1024, +1024)), q = 0..7
__device__ __forceinline__ void g256w_stage(const __bf16* __restrict__ p, int64_t ld, int rows,
                                            int r0, int k0, char* dst, int wave, int lane) {
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int wi = q * g256w::NW + wave;
    const int row = wi * 8 + (lane >> 3);
    const int c = g256_swz(row, lane & 7);
    int gr = r0 + row;
    gr = gr < rows ? gr : rows - 1;
    const __bf16* src = p + (int64_t)gr * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)src,
                                     (__attribute__((address_space(3))) void*)(dst + wi * 1024),
                                     16, 0, 0);
  }
}

__global__ void __launch_bounds__(g256w::TH, 1)
gemm_nt256w4_kernel(const __bf16* __restrict__ A, int64_t lda, const __bf16* __restrict__ B,
                    int64_t ldb, int M, int N, int K, const float* __restrict__ bias, int relu,
                    __bf16* __restrict__ C, int64_t ldc, float* __restrict__ Cf, int64_t ldcf,
                    int tiles_n) {
  using namespace g256;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF_BYTES];  // 128 KiB
  const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const int id = g256_xcd(blockIdx.x, gridDim.x);
  const int tm = id / tiles_n, tn = id - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nk = K / BK;
  auto rd_a = [&](const char* buf, int ks, int i) {
    const int c = ks * 4 + (lane >> 4), r = wr * 128 + i * 16 + (lane & 15);
    return *reinterpret_cast<const bf16x8*>(buf + r * 128 + g256_swz(r, c) * 16);
  };
  auto rd_b = [&](const char* buf, int ks, int j) {
    const int c = ks * 4 + (lane >> 4), r = wc * 128 + j * 16 + (lane & 15);
    return *reinterpret_cast<const bf16x8*>(buf + TILE_BYTES + r * 128 + g256_swz(r, c) * 16);
  };
  g256w_stage(A, lda, M, m0, 0, smem, wave, lane);
  g256w_stage(B, ldb, N, n0, 0, smem + TILE_BYTES, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  bf16x8 a0[8], b0[8], a1[8], b1[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) a0[i] = rd_a(smem, 0, i);
#pragma unroll
  for (int j = 0; j < 8; ++j) b0[j] = rd_b(smem, 0, j);
  for (int kt = 0; kt < nk; ++kt) {
    const char* cur = smem + (kt & 1) * BUF_BYTES;
    char* nxt = smem + ((kt + 1) & 1) * BUF_BYTES;
    const bool more = kt + 1 < nk;
    if (more) {
      g256w_stage(A, lda, M, m0, (kt + 1) * BK, nxt, wave, lane);
      g256w_stage(B, ldb, N, n0, (kt + 1) * BK, nxt + TILE_BYTES, wave, lane);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) a1[i] = rd_a(cur, 1, i);
#pragma unroll
    for (int j = 0; j < 8; ++j) b1[j] = rd_b(cur, 1, j);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i], b0[j], acc[i][j], 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i], b1[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    if (more) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of kt+1 landed
      __builtin_amdgcn_s_barrier();                     // ... every wave's
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 8; ++i) a0[i] = rd_a(nxt, 0, i);
#pragma unroll
      for (int j = 0; j < 8; ++j) b0[j] = rd_b(nxt, 0, j);
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 4; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i], b1[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  // epilogue: C[m][n], m = m0 + wr*128 + i*16 + 4*(lane>>4) + r, n = n0 + wc*128 + j*16 + (lane&15)
  if (C && !Cf && (ldc & 7) == 0 && m0 + BM <= M && n0 + BN <= N) {
    __bf16* st = reinterpret_cast<__bf16*>(smem);  // [256][256] bf16 = 128 KiB
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int nl = wc * 128 + j * 16 + (lane & 15);
      const float bv = bias ? bias[n0 + nl] : 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ml = wr * 128 + i * 16 + 4 * (lane >> 4) + r;
          float v = acc[i][j][r] + bv;
          if (relu) v = v > 0.f ? v : 0.f;
          st[ml * BN + nl] = (__bf16)v;
        }
    }
    __syncthreads();
#pragma unroll 4
    for (int q = 0; q < BM * BN / 8 / g256w::TH; ++q) {  // 32 chunks of 8 bf16 per thread
      const int ch = q * g256w::TH + t;
      const int ml = ch >> 5, nc = (ch & 31) * 8;
      *reinterpret_cast<uint4*>(C + (int64_t)(m0 + ml) * ldc + n0 + nc) =
          *reinterpret_cast<const uint4*>(st + ml * BN + nc);
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int n = n0 + wc * 128 + j * 16 + (lane & 15);
    if (n >= N) continue;
    const float bv = bias ? bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wr * 128 + i * 16 + 4 * (lane >> 4) + r;
        if (m >= M) continue;
        float v = acc[i][j][r] + bv;
        if (relu) v = v > 0.f ? v : 0.f;
        if (C) C[(int64_t)m * ldc + n] = (__bf16)v;
        if (Cf) Cf[(int64_t)m * ldcf + n] = v;
      }
    }
  }
}

void gemm_nt256(const __bf16* A, int64_t lda, const __bf16* B, int64_t ldb, int M, int N, int K,
                const float* bias, bool relu, __bf16* C, int64_t ldc, float* Cf, int64_t ldcf,
                int variant, hipStream_t st) {
  if (M <= 0 || N <= 0) return;
  if (K % g256::BK != 0 || lda % 8 || ldb % 8) throw std::runtime_error("gemm_nt256: K % 64, ld % 8");
  const int tiles_m = (M + g256::BM - 1) / g256::BM, tiles_n = (N + g256::BN - 1) / g256::BN;
  if (variant == 6)
    gemm_nt256r32_kernel<<<tiles_m * tiles_n, g256::TH, 0, st>>>(A, lda, B, ldb, M, N, K, bias,
                                                                 relu ? 1 : 0, C, ldc, Cf, ldcf,
                                                                 tiles_n);
  else if (variant == 5)
    gemm_nt256w4_kernel<<<tiles_m * tiles_n, g256w::TH, 0, st>>>(A, lda, B, ldb, M, N, K, bias,
                                                                 relu ? 1 : 0, C, ldc, Cf, ldcf,
                                                                 tiles_n);
  else if (variant == 4)
    gemm_nt256r_kernel<<<tiles_m * tiles_n, g256::TH, 0, st>>>(A, lda, B, ldb, M, N, K, bias,
                                                               relu ? 1 : 0, C, ldc, Cf, ldcf,
                                                               tiles_n);
  else if (variant == 2)
    gemm_nt256p8_kernel<<<tiles_m * tiles_n, g256::TH, 0, st>>>(A, lda, B, ldb, M, N, K, bias,
                                                                relu ? 1 : 0, C, ldc, Cf, ldcf,
                                                                tiles_n);
  else if (variant == 1)
    gemm_nt256pp_kernel<<<tiles_m * tiles_n, g256::TH, 0, st>>>(A, lda, B, ldb, M, N, K, bias,
                                                                relu ? 1 : 0, C, ldc, Cf, ldcf,
                                                                tiles_n);
  else if (variant == 3)
    gemm_nt256_kernel<true><<<tiles_m * tiles_n, g256::TH, 0, st>>>(A, lda, B, ldb, M, N, K, bias,
                                                                    relu ? 1 : 0, C, ldc, Cf, ldcf,
                                                                    tiles_n);
  else
    gemm_nt256_kernel<false><<<tiles_m * tiles_n, g256::TH, 0, st>>>(A, lda, B, ldb, M, N, K, bias,
                                                                     relu ? 1 : 0, C, ldc, Cf,
                                                                     ldcf, tiles_n);
  PSAMD_HIP_CHECK(hipGetLastError());
}

}  // namespace psamd
