// Fixed-capacity multi-GPU exchange: pack / unpack kernels.
//
// The reference moves a pull or push as one ZeroMQ message per server, sized
// by its sliced key list (src/system/message.h:120-159 sliceKeyOrderedMsg,
// src/system/van.cc:117-170). Over RCCL a variable-size all-to-all needs the
// per-peer sizes on the HOST, i.e. one device->host sync per step. Here every
// peer gets a fixed row of H int32 words instead, with the live counts in the
// row header, so the whole step (pack -> all-to-all -> owner update/resolve ->
// all-to-all -> unpack) runs without a host round trip and replays from HIP
// graphs between the collectives.
//
// Row p of the send buffer (H words, H >= 4 + C * kw + gradient words):
//   [0] nkeys   keys of this step owned by rank p (<= C)
//   [1] ngrads  gradients of the previous step's keys for rank p (<= C)
//   [2..3]      FixingFloat min / max of the row's gradients, else padding (keeps
//               the key region 16-B aligned)
//   [4, 4 + C*kw)  keys: u32 (kw = 1, mixed key space <= 32 bits) or u64
//   [4 + C*kw, ..) gradients: C f32 bit patterns, or C nb-byte FixingFloat codes
// The unique keys of a step are owner-ordered (sorted mixed keys, or the owner
// bucketing of a hash localisation with `perm` = owner-order -> unique id), and
// off[G+1] (device) are the owner run offsets. Keys past C in a run are dropped
// and counted in *ovf (the trainer raises on it; the capacity carries a large
// statistical margin over the per-peer count of hashed keys).
#include "common.cuh"
#include "kv_slot.cuh"
#include "loss.cuh"

namespace psamd {

constexpr int kMaxPeers = 64;

// Largest p with off[p] <= j (off non-decreasing, off[0] = 0).
__device__ __forceinline__ int owner_of_pos(const int64_t* soff, int G, int64_t j) {
  int lo = 0, hi = G - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (soff[mid] <= j) lo = mid; else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ void load_offsets(const int64_t* __restrict__ off, int G,
                                             int64_t* soff) {
  for (int t = threadIdx.x; t <= G; t += blockDim.x) soff[t] = off[t];
  __syncthreads();
}

// homes != null (the merged exchange): also the partition bounds of each row at word b0
// (see tpf_pack_keys_kernel, tploc.hip)
__global__ void xchg_pack_keys_kernel(const uint64_t* __restrict__ ukeys,
                                      const int32_t* __restrict__ n_uniq, int64_t n_host,
                                      const int64_t* __restrict__ off, int G, int64_t C, int kw,
                                      int64_t H, int32_t* __restrict__ send,
                                      int32_t* __restrict__ ovf, const uint64_t* __restrict__ homes,
                                      int64_t b0, int lgP) {
  __shared__ int64_t soff[kMaxPeers + 1];
  load_offsets(off, G, soff);
  const int P = 1 << lgP;
  if (blockIdx.x == 0 && threadIdx.x < G) {
    const int p = threadIdx.x;
    const int64_t cnt = soff[p + 1] - soff[p];
    send[(int64_t)p * H] = (int32_t)(cnt < C ? cnt : C);
    if (cnt > C && ovf) atomicAdd(ovf, (int32_t)(cnt - C));
    if (homes && cnt == 0)
      for (int j = 0; j <= P; ++j) send[(int64_t)p * H + b0 + j] = 0;
  }
  const int64_t n = dev_len(n_uniq, n_host);
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int p = owner_of_pos(soff, G, j);
    const int64_t i = j - soff[p];
    if (i >= C) continue;
    int32_t* row = send + (int64_t)p * H + 4;
    const uint64_t k = ukeys[j];
    if (kw == 1) row[i] = (int32_t)(uint32_t)k;
    else reinterpret_cast<uint64_t*>(row)[i] = k;
    if (homes) {
      const uint64_t hb = homes[2 * p], hm = homes[2 * p + 1];
      int32_t* rb = send + (int64_t)p * H + b0;
      const int q = key_part(k, hb, hm, lgP);
      const int q0 = i > 0 ? key_part(ukeys[j - 1], hb, hm, lgP) + 1 : 0;
      for (int jj = q0; jj <= q; ++jj) rb[jj] = (int32_t)i;
      const int64_t nr = soff[p + 1] - soff[p];
      if (i == (nr < C ? nr : C) - 1)  // the row's last key: the tail bounds
        for (int jj = q + 1; jj <= P; ++jj) rb[jj] = (int32_t)(i + 1);
    }
  }
}

__global__ void xchg_pack_grads_kernel(const float* __restrict__ grad,
                                       const int32_t* __restrict__ perm,
                                       const int32_t* __restrict__ n_uniq, int64_t n_host,
                                       const int64_t* __restrict__ off, int G, int64_t C, int kw,
                                       int64_t H, int32_t* __restrict__ send,
                                       uint32_t* __restrict__ hist, int hist_stripes,
                                       double* __restrict__ metrics,
                                       int64_t* __restrict__ step_counter,
                                       const int32_t* __restrict__ ovf,
                                       int32_t* __restrict__ ovf_host) {
  __shared__ int64_t soff[kMaxPeers + 1];
  // the overflow counter (final for this step: its key pack ran earlier in stream
  // order) goes to the host-mapped flag here instead of in a 1-thread launch of its
  // own (4 us of launch + system-scope release per step at 8 peers)
  if (ovf_host && blockIdx.x == 0 && threadIdx.x == 0) ovf_host[0] = ovf[0];
  // block 0 also turns the step's AUC histogram into metrics (the forward is done):
  // the single-block AUC launch leaves the worker half of the step
  if (hist && blockIdx.x == 0) auc_hist_block(hist, 2048, hist_stripes, metrics, step_counter);
  load_offsets(off, G, soff);
  if (blockIdx.x == 0 && threadIdx.x < G) {
    const int p = threadIdx.x;
    const int64_t cnt = soff[p + 1] - soff[p];
    send[(int64_t)p * H + 1] = (int32_t)(cnt < C ? cnt : C);
  }
  const int64_t n = dev_len(n_uniq, n_host);
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int p = owner_of_pos(soff, G, j);
    const int64_t i = j - soff[p];
    if (i >= C) continue;
    const int64_t u = perm ? (int64_t)perm[j] : j;
    const float g = in_range(u, n_host) ? grad[u] : 0.f;
    reinterpret_cast<float*>(send + (int64_t)p * H + 4 + C * kw)[i] = g;
  }
}

// Clears the gradient counts of every row (a flush / first step sends no grads).
__global__ void xchg_clear_grads_kernel(int32_t* __restrict__ send, int G, int64_t H) {
  if (threadIdx.x < G) send[(int64_t)threadIdx.x * H + 1] = 0;
}

__global__ void xchg_clear_keys_kernel(int32_t* __restrict__ send, int G, int64_t H) {
  if (threadIdx.x < G) send[(int64_t)threadIdx.x * H] = 0;
}

// w_local[unique id] <- the owner's reply (recv_w row p = weights of the keys this
// rank sent to p, in send order); dropped (overflow) keys read 0.
__global__ void xchg_unpack_w_kernel(const float* __restrict__ recv_w,
                                     const int32_t* __restrict__ perm,
                                     const int32_t* __restrict__ n_uniq, int64_t n_host,
                                     const int64_t* __restrict__ off, int G, int64_t C,
                                     int64_t wstride, float* __restrict__ w_local) {
  __shared__ int64_t soff[kMaxPeers + 1];
  load_offsets(off, G, soff);
  const int64_t n = dev_len(n_uniq, n_host);
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * blockDim.x) {
    const int p = owner_of_pos(soff, G, j);
    const int64_t i = j - soff[p];
    const float v = i < C ? recv_w[(int64_t)p * wstride + i] : 0.f;
    const int64_t u = perm ? (int64_t)perm[j] : j;
    if (in_range(u, n_host)) w_local[u] = v;
  }
}

// Copies the device overflow counter into host-mapped (pinned) memory so the
// host can poll it every step without a stream synchronisation: the trainer
// raises at the first step whose published count is non-zero.
__global__ void xchg_publish_kernel(const int32_t* __restrict__ src, int32_t* __restrict__ dst) {
  if (threadIdx.x == 0) dst[0] = src[0];
}

void xchg_publish(const int32_t* src, int32_t* host_mapped_dst, hipStream_t st) {
  xchg_publish_kernel<<<1, 64, 0, st>>>(src, host_mapped_dst);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void xchg_pack_keys(const uint64_t* ukeys, const int32_t* n_uniq, int64_t n_host,
                    const int64_t* off, int G, int64_t C, int kw, int64_t H, int32_t* send,
                    int32_t* ovf, const uint64_t* homes, int64_t b0, int lgP, hipStream_t st) {
  xchg_pack_keys_kernel<<<grid_for(n_host, 256), 256, 0, st>>>(ukeys, n_uniq, n_host, off, G, C,
                                                                kw, H, send, ovf, homes, b0, lgP);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void xchg_pack_grads(const float* grad, const int32_t* perm, const int32_t* n_uniq,
                     int64_t n_host, const int64_t* off, int G, int64_t C, int kw, int64_t H,
                     int32_t* send, uint32_t* hist, int hist_stripes, double* metrics,
                     int64_t* step_counter, const int32_t* ovf, int32_t* ovf_host,
                     hipStream_t st) {
  xchg_pack_grads_kernel<<<grid_for(n_host, 256), 256, 0, st>>>(grad, perm, n_uniq, n_host, off,
                                                                 G, C, kw, H, send, hist, hist_stripes,
                                                                 metrics, step_counter, ovf,
                                                                 ovf_host);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void xchg_clear_counts(int32_t* send, int G, int64_t H, bool keys, bool grads, hipStream_t st) {
  if (grads) xchg_clear_grads_kernel<<<1, 64, 0, st>>>(send, G, H);
  if (keys) xchg_clear_keys_kernel<<<1, 64, 0, st>>>(send, G, H);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void xchg_unpack_w(const float* recv_w, const int32_t* perm, const int32_t* n_uniq,
                   int64_t n_host, const int64_t* off, int G, int64_t C, int64_t wstride,
                   float* w_local, hipStream_t st) {
  xchg_unpack_w_kernel<<<grid_for(n_host, 256), 256, 0, st>>>(
      recv_w, perm, n_uniq, n_host, off, G, C, wstride > 0 ? wstride : C, w_local);
  PSAMD_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// FixingFloat on the padded exchange (reference src/filter/fixing_float.h:44-95,
// enabled per push by async_sgd.h:273-277): the gradient region of row p carries
// ceil(C * nb / 4) words of nb-byte fixed-point codes; header words [2], [3] hold
// the row's min / max as order-preserving ints (max gets +1e-6 when decoded, as
// the reference does). Stochastic rounding draws from a counter RNG keyed by
// (seed, device step clock, row, index), so graph replays draw fresh bits.
__device__ __forceinline__ int ff_ord(float f) {
  const int b = __float_as_int(f);
  return b >= 0 ? b : b ^ 0x7fffffff;
}
__device__ __forceinline__ float ff_unord(int b) {
  return __int_as_float(b >= 0 ? b : b ^ 0x7fffffff);
}

__global__ void xchg_ff_init_kernel(int32_t* __restrict__ send, int G, int64_t H) {
  if (threadIdx.x < G) {
    send[(int64_t)threadIdx.x * H + 2] = ff_ord(3.4e38f);
    send[(int64_t)threadIdx.x * H + 3] = ff_ord(-3.4e38f);
  }
}

// Stage grad(t) in owner order into gstage[p*C + i] and reduce each row's min/max.
__global__ void xchg_ff_stage_kernel(const float* __restrict__ grad,
                                     const int32_t* __restrict__ perm,
                                     const int32_t* __restrict__ n_uniq, int64_t n_host,
                                     const int64_t* __restrict__ off, int G, int64_t C, int64_t H,
                                     int32_t* __restrict__ send, float* __restrict__ gstage) {
  __shared__ int64_t soff[kMaxPeers + 1];
  load_offsets(off, G, soff);
  if (blockIdx.x == 0 && threadIdx.x < G) {
    const int p = threadIdx.x;
    const int64_t cnt = soff[p + 1] - soff[p];
    send[(int64_t)p * H + 1] = (int32_t)(cnt < C ? cnt : C);
  }
  const int64_t n = dev_len(n_uniq, n_host);
  const int lane = threadIdx.x & 63;
  for (int64_t j0 = blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~63); j0 < n;
       j0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = j0 + lane;
    int p = -1;
    float lo = 3.4e38f, hi = -3.4e38f;
    if (j < n) {
      p = owner_of_pos(soff, G, j);
      const int64_t i = j - soff[p];
      if (i < C) {
        const int64_t u = perm ? (int64_t)perm[j] : j;
        const float g = in_range(u, n_host) ? grad[u] : 0.f;
        gstage[(int64_t)p * C + i] = g;
        if (g == g) { lo = g; hi = g; }
      } else {
        p = -1;
      }
    }
    const int p0 = __shfl(p, 0, 64);
    const bool uniform = __ballot(p != p0) == 0ull;
    if (uniform) {  // the common case: the whole wave is in one owner's run
      lo = wave_min(lo);
      hi = wave_max(hi);
      if (lane == 0 && p0 >= 0) {
        atomicMin(&send[(int64_t)p0 * H + 2], ff_ord(lo));
        atomicMax(&send[(int64_t)p0 * H + 3], ff_ord(hi));
      }
    } else if (p >= 0) {
      atomicMin(&send[(int64_t)p * H + 2], ff_ord(lo));
      atomicMax(&send[(int64_t)p * H + 3], ff_ord(hi));
    }
  }
}

// per > 0 (the flat layout's tpf_pack_grads): the row's min / max from its producer
// workgroups' partials at gstage[G * C + 2 w] (w in [p per, (p + 1) per)), reduced by every
// block of the row (a few hundred floats from L2), the header written by block 0; per = 0:
// the header words as reduced by the producer's atomics (xchg_ff_stage_kernel).
__global__ void xchg_ff_encode_kernel(const float* __restrict__ gstage, int64_t C, int kw,
                                      int64_t H, int nb, uint64_t seed,
                                      const int64_t* __restrict__ step,
                                      int32_t* __restrict__ send, int per) {
  const int p = blockIdx.y;
  int32_t* row = send + (int64_t)p * H;
  const int64_t n = dev_len(row + 1, C);
  float lo, hi;
  if (per > 0) {
    __shared__ float sl[4], sh[4];
    const float* part = gstage + (int64_t)gridDim.y * C + 2 * (int64_t)p * per;
    float a = 3.4e38f, z = -3.4e38f;
    for (int w = threadIdx.x; w < per; w += blockDim.x) {
      a = fminf(a, part[2 * w]);
      z = fmaxf(z, part[2 * w + 1]);
    }
    a = wave_min(a);
    z = wave_max(z);
    if ((threadIdx.x & 63) == 0) {
      sl[threadIdx.x >> 6] = a;
      sh[threadIdx.x >> 6] = z;
    }
    __syncthreads();
    a = fminf(fminf(sl[0], sl[1]), fminf(sl[2], sl[3]));
    z = fmaxf(fmaxf(sh[0], sh[1]), fmaxf(sh[2], sh[3]));
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      row[2] = ff_ord(a);
      row[3] = ff_ord(z);
    }
    lo = ff_unord(ff_ord(a));
    hi = ff_unord(ff_ord(z)) + 1e-6f;
  } else {
    lo = ff_unord(row[2]);
    hi = ff_unord(row[3]) + 1e-6f;
  }
  const double bin = (double)hi - (double)lo;
  const double ratio = (double)((1ull << (8 * nb)) - 2ull);
  const uint64_t sd = fmix64(seed ^ fmix64((step ? (uint64_t)*step : 0ull) * 0x9e3779b97f4a7c15ull +
                                           (uint64_t)p));
  uint8_t* code = reinterpret_cast<uint8_t*>(row + 4 + C * kw);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v = gstage[(int64_t)p * C + i];
    v = v > hi ? hi : (v < lo ? lo : v);
    const double t = bin > 0 ? ((double)v - lo) / bin * ratio : 0.0;
    const double f = floor(t);
    const double u = (double)u01(rng64(sd, (uint64_t)i)) - 1e-12;
    uint64_t r = (uint64_t)f + ((t - f) > u ? 1ull : 0ull);
    for (int b = 0; b < nb; ++b) { code[i * nb + b] = (uint8_t)(r & 0xff); r >>= 8; }
  }
}

// Owner: codes of every source row -> gin[s*C + i] (f32), in front of the updates.
__global__ void xchg_ff_decode_kernel(const int32_t* __restrict__ recv, int64_t C, int kw,
                                      int64_t H, int nb, float* __restrict__ gin) {
  const int s = blockIdx.y;
  const int32_t* row = recv + (int64_t)s * H;
  const int64_t n = dev_len(row + 1, C);
  const float lo = ff_unord(row[2]), hi = ff_unord(row[3]) + 1e-6f;
  const double bin = (double)hi - (double)lo;
  const double ratio = (double)((1ull << (8 * nb)) - 2ull);
  const uint8_t* code = reinterpret_cast<const uint8_t*>(row + 4 + C * kw);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t r = 0;
    for (int b = 0; b < nb; ++b) r |= (uint64_t)code[i * nb + b] << (8 * b);
    gin[(int64_t)s * C + i] = (float)((double)r / ratio * bin + lo);
  }
}

void xchg_ff_pack_grads(const float* grad, const int32_t* perm, const int32_t* n_uniq,
                        int64_t n_host, const int64_t* off, int G, int64_t C, int kw, int64_t H,
                        int nb, uint64_t seed, const int64_t* step, int32_t* send, float* gstage,
                        hipStream_t st) {
  xchg_ff_init_kernel<<<1, 64, 0, st>>>(send, G, H);
  PSAMD_HIP_CHECK(hipGetLastError());
  xchg_ff_stage_kernel<<<grid_for(n_host, 256), 256, 0, st>>>(grad, perm, n_uniq, n_host, off, G,
                                                               C, H, send, gstage);
  PSAMD_HIP_CHECK(hipGetLastError());
  dim3 grid(grid_for(C, 256, 512), G);
  xchg_ff_encode_kernel<<<grid, 256, 0, st>>>(gstage, C, kw, H, nb, seed, step, send, 0);
  PSAMD_HIP_CHECK(hipGetLastError());
}

// the two halves of xchg_ff_pack_grads around a producer that stages the rows itself (the
// flat layout's tpf_pack_grads writes gstage and the rows' min / max)
void xchg_ff_init(int32_t* send, int G, int64_t H, hipStream_t st) {
  xchg_ff_init_kernel<<<1, 64, 0, st>>>(send, G, H);
  PSAMD_HIP_CHECK(hipGetLastError());
}
void xchg_ff_encode(const float* gstage, int G, int64_t C, int kw, int64_t H, int nb, uint64_t seed,
                    const int64_t* step, int32_t* send, int per, hipStream_t st) {
  dim3 grid(grid_for(C, 256, 512), G);
  xchg_ff_encode_kernel<<<grid, 256, 0, st>>>(gstage, C, kw, H, nb, seed, step, send, per);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void xchg_ff_decode(const int32_t* recv, int G, int64_t C, int kw, int64_t H, int nb, float* gin,
                    hipStream_t st) {
  dim3 grid(grid_for(C, 256, 512), G);
  xchg_ff_decode_kernel<<<grid, 256, 0, st>>>(recv, C, kw, H, nb, gin);
  PSAMD_HIP_CHECK(hipGetLastError());
}

}  // namespace psamd
