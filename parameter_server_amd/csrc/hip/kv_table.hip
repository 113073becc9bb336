// HBM-resident sharded key/value store for scalar linear models.
//
// Replaces the reference's per-server CPU hash map `KVStore<K,V,E,S>`
// (src/parameter/kv_store.h:28-80) whose entries implement the optimizer
// (FTRLEntry / SGDEntry / AdaGradEntry, src/app/linear_method/async_sgd.h:71-124).
//
// Layout: open addressing, linear probing, one 32-byte slot per key
//   { u64 key(mixed) | f32 w | f32 z | f32 n | f32 acc | u32 cnt | u32 flags }
// so a lookup that hits on its first probe touches exactly one 32-B sector and
// the optimizer read-modify-write touches the same sector again. Probe index =
// fmix64(key) & mask. 10^9 keys at load 0.5 = 64 GB: fits one MI355X's 288 GB.
//
// Concurrency: a key transitions EMPTY -> key exactly once via 64-bit CAS, so
// a stale plain load can only return EMPTY (then the CAS is authoritative) or
// the final key. Payload updates to distinct slots are race free (callers
// dedupe keys per launch); cross-source duplicates are applied by sequential
// launches (reference semantics: every push message is one optimizer step)
// or by the accumulate/apply pair (synchronous / BSP aggregation).
#include "kv_slot.cuh"
#include "loss.cuh"
#include <stdexcept>
#include <string>

namespace psamd {

__global__ void kv_init_kernel(Slot* __restrict__ slots, int64_t cap) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < cap;
       i += (int64_t)gridDim.x * blockDim.x) {
    Slot s;
    s.key = kEmptyKey;
    s.w = s.z = s.n = s.acc = 0.f;
    s.cnt = s.flags = 0;
    slots[i] = s;
  }
}

// Lookup (optionally insert) every key; write its slot index (-1 if absent or
// table full) and optionally its weight. The fused weight is exact for any init: a
// lane that finds a key another lane of this launch has just claimed reads the weight
// only once the inserter published it (kv_slot.cuh published_w), else the init value.
__global__ void kv_resolve_kernel(Slot* __restrict__ slots, uint64_t mask, uint64_t home_base,
                                  uint64_t home_m, int home_shr,
                                  const uint64_t* __restrict__ keys, int64_t n_host,
                                  const int32_t* __restrict__ n_dev,
                                  int64_t* __restrict__ out_slot, float* __restrict__ out_w,
                                  int insert, int init_type, float init_v, float init_s,
                                  uint64_t seed, int32_t* __restrict__ err,
                                  int32_t* __restrict__ inserted) {
  const int64_t n = dev_len(n_dev, n_host);
  int local_ins = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float w;
    const int64_t found = resolve_key(slots, mask, home_base, home_m, home_shr, keys[i], insert,
                                      init_type, init_v, init_s, seed, &w, &local_ins);
    if (found < 0 && insert && err) atomicOr(err, 1);  // table full
    out_slot[i] = found;
    if (out_w) out_w[i] = w;
  }
  if (inserted) {
    int tot = wave_sum(local_ins);
    if ((threadIdx.x & 63) == 0 && tot) atomicAdd(inserted, tot);
  }
}

// Owner side of the fixed-capacity exchange (exchange.hip): the received buffer
// holds one row of H int32 words per source rank, [nkeys, ngrads, -, -, keys (C x kw
// words), grads (C)]. blockIdx.y = source; resolves that row's nkeys keys into
// out_slot[s*C + i] and out_w[s*C + i] (the weights that travel back).
__global__ void kv_resolve_rows_kernel(Slot* __restrict__ slots, uint64_t mask,
                                       uint64_t home_base, uint64_t home_m, int home_shr,
                                       const int32_t* __restrict__ recv, int64_t H, int64_t C,
                                       int kw, int64_t* __restrict__ out_slot,
                                       float* __restrict__ out_w, int64_t wstride,
                                       int insert, int init_type,
                                       float init_v, float init_s, uint64_t seed,
                                       int32_t* __restrict__ err, int32_t* __restrict__ inserted,
                                       uint64_t* __restrict__ out_key, int32_t* __restrict__ bnd,
                                       int lgP) {
  const int s = blockIdx.y;
  const int32_t* row = recv + (int64_t)s * H;
  const int64_t n = dev_len(row, C);
  const int P = 1 << lgP;
  int32_t* rb = bnd ? bnd + (int64_t)s * (P + 1) : nullptr;
  if (rb && n == 0 && blockIdx.x == 0)
    for (int q = threadIdx.x; q <= P; q += blockDim.x) rb[q] = 0;
  int local_ins = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t h = kw == 1 ? (uint64_t)(uint32_t)row[4 + i]
                               : reinterpret_cast<const uint64_t*>(row + 4)[i];
    float w;
    const int64_t found = resolve_key(slots, mask, home_base, home_m, home_shr, h, insert,
                                      init_type, init_v, init_s, seed, &w, &local_ins);
    if (found < 0 && insert && err) atomicOr(err, 1);
    out_slot[(int64_t)s * C + i] = found;
    out_w[(int64_t)s * wstride + i] = w;
    if (out_key) out_key[(int64_t)s * C + i] = h;
    if (rb) {  // partition bounds of this (sorted) row: rb[q] = #keys of partition < q
      const int q = key_part(h, home_base, home_m, lgP);
      int q0 = 0;
      if (i > 0) {
        const uint64_t hp = kw == 1 ? (uint64_t)(uint32_t)row[4 + i - 1]
                                    : reinterpret_cast<const uint64_t*>(row + 4)[i - 1];
        q0 = key_part(hp, home_base, home_m, lgP) + 1;
      }
      for (int j = q0; j <= q; ++j) rb[j] = (int32_t)i;
      if (i == n - 1)
        for (int j = q + 1; j <= P; ++j) rb[j] = (int32_t)n;
    }
  }
  if (inserted) {
    int tot = wave_sum(local_ins);
    if ((threadIdx.x & 63) == 0 && tot) atomicAdd(inserted, tot);
  }
}

// out[i] = slot.w (0 for missing), gathered by cached slot index.
__global__ void kv_gather_kernel(const Slot* __restrict__ slots, int64_t cap,
                                 const int64_t* __restrict__ slot_idx, int64_t n_host,
                                 const int32_t* __restrict__ n_dev, float* __restrict__ out,
                                 int field) {
  const int64_t n = dev_len(n_dev, n_host);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = slot_idx[i];
    float v = 0.f;
    if (in_range(s, cap)) {
      const float* f = &slots[s].w;
      v = f[field];
    }
    out[i] = v;
  }
}

// Set fields (checkpoint restore / explicit assignment).
__global__ void kv_set_kernel(Slot* __restrict__ slots, int64_t cap,
                              const int64_t* __restrict__ slot_idx,
                              int64_t n, const float* __restrict__ w,
                              const float* __restrict__ z, const float* __restrict__ nn) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = slot_idx[i];
    if (!in_range(s, cap)) continue;
    if (w) publish_init(&slots[s], w[i]);  // (an explicit weight counts as published)
    if (z) slots[s].z = z[i];
    if (nn) slots[s].n = nn[i];
  }
}

// Apply one pushed gradient per (unique within this launch) slot.
// stats: [0] nnz delta (as double), [1] sum w_new^2, [2] sum (w_new-w_old)^2.
__global__ void kv_update_kernel(Slot* __restrict__ slots, int64_t cap,
                                 const int64_t* __restrict__ slot_idx,
                                 const float* __restrict__ grad, int64_t n_host,
                                 const int32_t* __restrict__ n_dev, UpdateParams p,
                                 double* __restrict__ stats, int acc_stripes,
                                 uint32_t* __restrict__ hist, int nbins, int hist_stripes,
                                 double* __restrict__ metrics, int64_t* __restrict__ step_counter) {
  // block 0 also turns the step's AUC histogram into metrics (the forward finished
  // before this launch): the separate single-block AUC launch leaves the critical path
  if (hist && blockIdx.x == 0) auc_hist_block(hist, nbins, hist_stripes, metrics, step_counter);
  const int64_t n = dev_len(n_dev, n_host);
  double dnnz = 0, wsum = 0, dsum = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t si = slot_idx[i];
    if (!in_range(si, cap)) continue;
    const float g = grad[i] * p.grad_scale;
    if (g != g) continue;  // NaN mark = filtered entry (reference SparseFilter)
    Slot s = slots[si];
    const float w_old = apply_update(s, g, p);
    slots[si] = s;
    dnnz += (double)((s.w != 0.f) - (w_old != 0.f));
    wsum += (double)s.w * s.w;
    const double d = (double)s.w - w_old;
    dsum += d * d;
  }
  if (stats) {  // per-wave DPP sums, lane 63 adds to the striped accumulators (no barriers)
    const double a = wave_sum_dpp(dnnz), b = wave_sum_dpp(wsum), c = wave_sum_dpp(dsum);
    if ((threadIdx.x & 63) == 63) {
      double* st = acc_stripe(stats, acc_stripes);
      if (a != 0) atomicAdd(&st[0], a);
      if (b != 0) atomicAdd(&st[1], b);
      if (c != 0) atomicAdd(&st[2], c);
    }
  }
}

// Synchronous aggregation: acc += g; the first toucher of a slot appends it to the
// touched list (one list atomic per wavefront, not per lane).
__device__ __forceinline__ void accumulate_one(Slot* __restrict__ slots, int64_t cap, int64_t si,
                                               float g, bool valid, int64_t* __restrict__ touched,
                                               int32_t* __restrict__ n_touched,
                                               int64_t touched_cap) {
  bool first = false;
  if (valid && in_range(si, cap) && g == g) {  // NaN mark = filtered entry
    atomicAdd(&slots[si].acc, g);
    first = atomicOr(&slots[si].flags, 1u) == 0u;
  }
  const uint64_t m = __ballot(first);
  if (!m) return;
  const int lane = threadIdx.x & 63;
  const int leader = __ffsll((long long)m) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(n_touched, (int)__popcll(m));
  base = __shfl(base, leader, 64);
  if (first) {
    const int pos = base + (int)__popcll(m & ((1ull << lane) - 1ull));
    if (pos < touched_cap) touched[pos] = si;
  }
}

__global__ void kv_accumulate_kernel(Slot* __restrict__ slots, int64_t cap,
                                     const int64_t* __restrict__ slot_idx,
                                     const float* __restrict__ grad, int64_t n_host,
                                     const int32_t* __restrict__ n_dev,
                                     int64_t* __restrict__ touched, int32_t* __restrict__ n_touched,
                                     int64_t touched_cap) {
  const int64_t n = dev_len(n_dev, n_host);
  // whole wavefronts iterate together (the list append uses a ballot)
  for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~63); i0 < n;
       i0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = i0 + (threadIdx.x & 63);
    const bool valid = i < n;
    accumulate_one(slots, cap, valid ? slot_idx[i] : -1, valid ? grad[i] : 0.f, valid, touched,
                   n_touched, touched_cap);
  }
}

// The owner's pushes of one step, all source rows in ONE launch (blockIdx.y = source):
// row s has ngrads = recv[s*H + 1] gradients at grad[s*gstride + i] for the slots
// slot_idx[s*C + i] resolved by that source's pull.
__global__ void kv_accumulate_rows_kernel(Slot* __restrict__ slots, int64_t cap,
                                          const int64_t* __restrict__ slot_idx,
                                          const float* __restrict__ grad, int64_t gstride,
                                          const int32_t* __restrict__ recv, int64_t H, int64_t C,
                                          int64_t* __restrict__ touched,
                                          int32_t* __restrict__ n_touched, int64_t touched_cap) {
  const int s = blockIdx.y;
  const int64_t n = dev_len(recv + (int64_t)s * H + 1, C);
  for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~63); i0 < n;
       i0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = i0 + (threadIdx.x & 63);
    const bool valid = i < n;
    accumulate_one(slots, cap, valid ? slot_idx[(int64_t)s * C + i] : -1,
                   valid ? grad[(int64_t)s * gstride + i] : 0.f, valid, touched, n_touched,
                   touched_cap);
  }
}

__global__ void kv_apply_accumulated_kernel(Slot* __restrict__ slots, int64_t cap,
                                            const int64_t* __restrict__ touched,
                                            const int32_t* __restrict__ n_touched, int64_t max_n,
                                            UpdateParams p, double* __restrict__ stats,
                                            int acc_stripes) {
  const int64_t n = dev_len(n_touched, max_n);
  double dnnz = 0, wsum = 0, dsum = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t si = touched[i];
    if (!in_range(si, cap)) continue;
    Slot s = slots[si];
    const float g = s.acc * p.grad_scale;
    s.acc = 0.f;
    s.flags &= ~1u;  // (bit 1, the published-init mark, stays)
    const float w_old = apply_update(s, g, p);
    slots[si] = s;
    dnnz += (double)((s.w != 0.f) - (w_old != 0.f));
    wsum += (double)s.w * s.w;
    const double d = (double)s.w - w_old;
    dsum += d * d;
  }
  if (stats) {  // per-wave DPP sums, lane 63 adds to the striped accumulators (no barriers)
    const double a = wave_sum_dpp(dnnz), b = wave_sum_dpp(wsum), c = wave_sum_dpp(dsum);
    if ((threadIdx.x & 63) == 63) {
      double* st = acc_stripe(stats, acc_stripes);
      if (a != 0) atomicAdd(&st[0], a);
      if (b != 0) atomicAdd(&st[1], b);
      if (c != 0) atomicAdd(&st[2], c);
    }
  }
}

// ---------------------------------------------------------------------------
// The owner's pushes of one exchange, ALL G source rows, with per-push semantics
// (reference KVStore::setValue applies every push message as its own optimizer
// step, src/parameter/kv_store.h:47-57): a slot pushed by several sources gets
// their gradients one after the other in source-rank order. Instead of G
// launches (one per source row, the rows run in order), two launches for any G:
//   link:  each entry e = s*C + i (slot k) swaps itself into a per-exchange scratch
//          hash keyed by k (64-bit word = k << 32 | head entry) and keeps the
//          entry it replaced in nxt[e] -> one chain per slot, <= G entries long
//          (a source row holds distinct keys, so distinct slots);
//   apply: the entry that is the final head of its chain walks it, applies the
//          gradients in increasing entry order (= source order) to a register copy
//          of the slot and stores it once.
// Bitwise the same weights as the per-row launch sequence. Scratch: link[HS] u64
// (HS = power of two >= 2 * G * C), reset to ~0 by the launcher, nxt[G * C] i32.
constexpr int kMaxChain = 64;  // source rows per exchange (exchange.hip kMaxPeers)
__device__ __forceinline__ uint64_t link_probe_start(int64_t k, uint64_t hmask) {
  return fmix64((uint64_t)k) & hmask;
}

__global__ void kv_link_rows_kernel(const int64_t* __restrict__ slot_idx, int64_t cap,
                                    const float* __restrict__ grad, int64_t gstride,
                                    const int32_t* __restrict__ recv, int64_t H, int64_t C,
                                    unsigned long long* __restrict__ link, uint64_t hmask,
                                    int32_t* __restrict__ nxt) {
  const int s = blockIdx.y;
  const int64_t n = dev_len(recv + (int64_t)s * H + 1, C);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = (int64_t)s * C + i;
    const int64_t k = slot_idx[e];
    const float g = grad[(int64_t)s * gstride + i];
    if (!in_range(k, cap) || g != g) continue;  // NaN mark = filtered entry
    uint64_t h = link_probe_start(k, hmask);
    for (uint64_t probe = 0; probe <= hmask; ++probe) {
      unsigned long long cur = link[h];
      bool done = false;
      while (true) {
        if (cur == ~0ull) {  // empty: claim it for k
          const unsigned long long mine = ((unsigned long long)k << 32) | (uint32_t)e;
          const unsigned long long prev = atomicCAS(&link[h], cur, mine);
          if (prev == cur) { nxt[e] = -1; done = true; break; }
          cur = prev;
          continue;
        }
        if ((int64_t)(cur >> 32) != k) break;  // another slot: next probe
        const unsigned long long mine = (cur & 0xffffffff00000000ull) | (uint32_t)e;
        const unsigned long long prev = atomicCAS(&link[h], cur, mine);
        if (prev == cur) { nxt[e] = (int32_t)(uint32_t)(cur & 0xffffffffull); done = true; break; }
        cur = prev;
      }
      if (done) break;
      h = (h + 1) & hmask;
    }
  }
}

__global__ void kv_apply_rows_kernel(Slot* __restrict__ slots, int64_t cap,
                                     const int64_t* __restrict__ slot_idx,
                                     const float* __restrict__ grad, int64_t gstride,
                                     const int32_t* __restrict__ recv, int64_t H, int64_t C,
                                     const unsigned long long* __restrict__ link, uint64_t hmask,
                                     const int32_t* __restrict__ nxt, int64_t n_ent,
                                     UpdateParams p, double* __restrict__ stats, int acc_stripes) {
  const int s = blockIdx.y;
  const int64_t n = dev_len(recv + (int64_t)s * H + 1, C);
  double dnnz = 0, wsum = 0, dsum = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = (int64_t)s * C + i;
    const int64_t k = slot_idx[e];
    const float g0 = grad[(int64_t)s * gstride + i];
    if (!in_range(k, cap) || g0 != g0) continue;
    uint64_t h = link_probe_start(k, hmask);
    unsigned long long cur = ~0ull;
    for (uint64_t probe = 0; probe <= hmask; ++probe) {
      cur = link[h];
      if (cur == ~0ull || (int64_t)(cur >> 32) == k) break;
      h = (h + 1) & hmask;
    }
    if (cur == ~0ull || (int64_t)(uint32_t)(cur & 0xffffffffull) != e) continue;  // not the head
    // chain length (<= number of source rows) and apply in increasing entry order
    int len = 0;
    for (int32_t c = (int32_t)e; c >= 0 && len < kMaxChain; c = nxt[c]) {
      if (!in_range((int64_t)c, n_ent)) break;
      ++len;
    }
    Slot sl = slots[k];
    int64_t last = -1;
    for (int it = 0; it < len; ++it) {
      int64_t best = INT64_MAX;
      int walked = 0;
      for (int32_t c = (int32_t)e; c >= 0 && walked < len; c = nxt[c], ++walked)
        if ((int64_t)c > last && (int64_t)c < best) best = c;
      if (best == INT64_MAX) break;
      const int64_t bs = best / C, bi = best - bs * C;
      const float g = grad[bs * gstride + bi] * p.grad_scale;
      const float w_old = apply_update(sl, g, p);
      dnnz += (double)((sl.w != 0.f) - (w_old != 0.f));
      wsum += (double)sl.w * sl.w;
      const double d = (double)sl.w - w_old;
      dsum += d * d;
      last = best;
    }
    slots[k] = sl;
  }
  if (stats) {  // per-wave DPP sums, lane 63 adds to the striped accumulators (no barriers)
    const double a = wave_sum_dpp(dnnz), b = wave_sum_dpp(wsum), c = wave_sum_dpp(dsum);
    if ((threadIdx.x & 63) == 63) {
      double* st = acc_stripe(stats, acc_stripes);
      if (a != 0) atomicAdd(&st[0], a);
      if (b != 0) atomicAdd(&st[1], b);
      if (c != 0) atomicAdd(&st[2], c);
    }
  }
}

// The same per-push semantics in ONE launch without global atomics or scratch
// resets, for shards with an ordered home whose source rows are sorted by key
// (the localisers' unique lists are): the resolve of the pull recorded each row's
// keys and the bounds of P = 2^lgP key-range partitions (kv_resolve_rows), so
// every partition is a run of consecutive entries in each row and no key spans
// two partitions. One workgroup per partition gathers its runs into LDS in
// windows of <= kApWin entries (a window ends at the smallest "last loaded key"
// of the rows that did not fit, so every key's entries share a window), chains
// entries of equal slot through an LDS hash, and the head of each chain applies
// its gradients in increasing entry order (= source-rank order) to a register
// copy of the slot: bitwise the weights of kv_apply_rows.
// (exchange.hip ff_unord: the order-preserving int of a FixingFloat row header -> float)
__device__ __forceinline__ float ff_unord_kv(int b) {
  return __int_as_float(b >= 0 ? b : b ^ 0x7fffffff);
}
constexpr int kApWin = 1024;   // entries per window
constexpr int kApRun = 16;     // a chain up to this long is ordered in LDS
constexpr int kApHash = 2048;  // LDS hash slots (power of two, >= 2 * kApWin)

// The body of kv_apply_part_kernel for partition blockIdx.x (also the apply half of
// kv_owner_part_kernel below).
__device__ __forceinline__ void apply_part_block(
    Slot* __restrict__ slots, int64_t cap, const int64_t* __restrict__ slot_idx,
    const uint64_t* __restrict__ keys, const float* __restrict__ grad, int64_t gstride,
    const int32_t* __restrict__ recv, int64_t H, int64_t C, int G,
    const int32_t* __restrict__ bnd, int lgP, UpdateParams p, double* __restrict__ stats,
    int acc_stripes, int ffnb = 0, int kw = 1) {
  __shared__ uint32_t hk[kApHash];
  __shared__ int32_t hh[kApHash];
  __shared__ int32_t went[kApWin], wnx[kApWin], whs[kApWin];
  __shared__ float wg[kApWin];
  __shared__ int32_t wrun[256 * kApRun];  // per-thread chain runs (blockDim 256)
  __shared__ int32_t ra[kMaxChain], re[kMaxChain], roff[kMaxChain + 1], rcnt[kMaxChain];
  __shared__ uint64_t thk[kMaxChain];
  __shared__ uint64_t thr;
  const int tid = threadIdx.x, P = 1 << lgP, part = blockIdx.x;
  const int CH = max(1, kApWin / G);
  // ffnb > 0: the pushes are FixingFloat codes in the received rows, decoded here (the
  // math of xchg_ff_decode_kernel, bit for bit) instead of by a separate launch
  __shared__ double flo[kMaxChain], fbin[kMaxChain];
  const double fratio = ffnb ? (double)((1ull << (8 * ffnb)) - 2ull) : 1.0;
  if (ffnb && tid < G) {
    const int32_t* row = recv + (int64_t)tid * H;
    const float lo = ff_unord_kv(row[2]), hi = ff_unord_kv(row[3]) + 1e-6f;
    flo[tid] = lo;
    fbin[tid] = (double)hi - (double)lo;
  }
  if (tid < G) {
    const int32_t n = (int32_t)dev_len(recv + (int64_t)tid * H + 1, C);
    const int32_t* rb = bnd + (int64_t)tid * (P + 1);
    const int32_t a = min(rb[part], n), b = min(rb[part + 1], n);
    ra[tid] = a;
    re[tid] = max(a, b);
  }
  for (int h = tid; h < kApHash; h += blockDim.x) {
    hk[h] = 0xffffffffu;
    hh[h] = -1;
  }
  double dnnz = 0, wsum = 0, dsum = 0;
  for (;;) {
    __syncthreads();
    // the window's end keys of the rows that do not fit: one load per row, all rows in
    // parallel (a serial loop over the rows was a chain of up to G dependent global loads)
    if (tid < G) {
      const int rem = re[tid] - ra[tid];
      thk[tid] = rem > CH ? keys[(int64_t)tid * C + ra[tid] + CH - 1] : ~0ull;
      rcnt[tid] = 0;
    }
    __syncthreads();
    if (tid == 0) {
      int off = 0;
      uint64_t t = ~0ull;
      for (int s = 0; s < G; ++s) {
        roff[s] = off;
        off += min(re[s] - ra[s], CH);
        t = min(t, thk[s]);
      }
      roff[G] = off;
      thr = t;
    }
    __syncthreads();
    const int tot = roff[G];
    if (tot == 0) break;
    const uint64_t th = thr;
    for (int w = tid; w < tot; w += blockDim.x) {
      int lo = 0, hi = G - 1;  // row of window entry w: last s with roff[s] <= w
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (roff[mid] <= w) lo = mid; else hi = mid - 1;
      }
      const int s = lo;
      const int64_t i = ra[s] + (w - roff[s]);
      const int64_t e = (int64_t)s * C + i;
      int32_t ent = -1;
      const uint64_t key = keys[e];  // three independent loads in flight together
      const int64_t k = slot_idx[e];
      float g;
      if (ffnb) {
        const uint8_t* code =
            reinterpret_cast<const uint8_t*>(recv + (int64_t)s * H + 4 + C * kw) + i * ffnb;
        uint64_t r = 0;
        for (int b = 0; b < ffnb; ++b) r |= (uint64_t)code[b] << (8 * b);
        g = (float)((double)r / fratio * fbin[s] + flo[s]);
      } else {
        g = grad[(int64_t)s * gstride + i];
      }
      if (key <= th) {
        atomicAdd(&rcnt[s], 1);
        if (in_range(k, cap) && g == g) {  // NaN mark = filtered entry
          const uint32_t ks = (uint32_t)k;
          uint32_t hp = (ks * 0x9E3779B1u) >> (32 - 11);  // log2(kApHash) = 11
          for (int probe = 0; probe < kApHash; ++probe) {
            const uint32_t prev = atomicCAS(&hk[hp], 0xffffffffu, ks);
            if (prev == 0xffffffffu || prev == ks) break;
            hp = (hp + 1) & (kApHash - 1);
          }
          ent = (int32_t)e;
          wg[w] = g;
          whs[w] = (int32_t)hp;
          wnx[w] = atomicExch(&hh[hp], w);
        }
      }
      went[w] = ent;
    }
    __syncthreads();
    for (int w = tid; w < tot; w += blockDim.x) {
      if (went[w] < 0 || hh[whs[w]] != w) continue;  // not the head of its chain
      const int64_t k = (int64_t)hk[whs[w]];
      Slot sl = slots[k];  // (the slot's load in flight while the chain is ordered)
      // the chain (keys shared by several source rows: hot features) into this thread's
      // LDS run, insertion-sorted by entry (= source-rank) order: one pointer chase and
      // ~len^2 / 4 compares, instead of a full chain walk per applied entry (len^2
      // dependent LDS reads: 64 for a key in all 8 rows of an 8-peer exchange)
      int32_t* run = wrun + tid * kApRun;
      int len = 0;
      int c = w;
      for (; c >= 0 && len < kApRun; c = wnx[c]) {
        const int32_t e = went[c];
        int q = len++;
        for (; q > 0 && went[run[q - 1]] > e; --q) run[q] = run[q - 1];
        run[q] = c;
      }
      if (c < 0) {
        for (int it = 0; it < len; ++it) {
          const int bw = run[it];
          const float w_old = apply_update(sl, wg[bw] * p.grad_scale, p);
          dnnz += (double)((sl.w != 0.f) - (w_old != 0.f));
          wsum += (double)sl.w * sl.w;
          const double d = (double)sl.w - w_old;
          dsum += d * d;
        }
      } else {  // (a longer chain: the selection walk)
        len = 0;
        for (int cc = w; cc >= 0 && len < kMaxChain; cc = wnx[cc]) ++len;
        int32_t last = -1;
        for (int it = 0; it < len; ++it) {  // next entry in increasing (source) order
          int32_t best = INT32_MAX, bw = -1, walked = 0;
          for (int cc = w; cc >= 0 && walked < len; cc = wnx[cc], ++walked)
            if (went[cc] > last && went[cc] < best) { best = went[cc]; bw = cc; }
          if (bw < 0) break;
          const float w_old = apply_update(sl, wg[bw] * p.grad_scale, p);
          dnnz += (double)((sl.w != 0.f) - (w_old != 0.f));
          wsum += (double)sl.w * sl.w;
          const double d = (double)sl.w - w_old;
          dsum += d * d;
          last = best;
        }
      }
      slots[k] = sl;
    }
    __syncthreads();
    if (tid < G) ra[tid] += rcnt[tid];
    for (int h = tid; h < kApHash; h += blockDim.x) {
      hk[h] = 0xffffffffu;
      hh[h] = -1;
    }
  }
  if (stats) {  // per-wave DPP sums, lane 63 adds to the striped accumulators (no barriers)
    const double a = wave_sum_dpp(dnnz), b = wave_sum_dpp(wsum), c = wave_sum_dpp(dsum);
    if ((threadIdx.x & 63) == 63) {
      double* st = acc_stripe(stats, acc_stripes);
      if (a != 0) atomicAdd(&st[0], a);
      if (b != 0) atomicAdd(&st[1], b);
      if (c != 0) atomicAdd(&st[2], c);
    }
  }
}

__global__ __launch_bounds__(256) void kv_apply_part_kernel(
    Slot* __restrict__ slots, int64_t cap, const int64_t* __restrict__ slot_idx,
    const uint64_t* __restrict__ keys, const float* __restrict__ grad, int64_t gstride,
    const int32_t* __restrict__ recv, int64_t H, int64_t C, int G,
    const int32_t* __restrict__ bnd, int lgP, UpdateParams p, double* __restrict__ stats,
    int acc_stripes, int ffnb, int kw) {
  apply_part_block(slots, cap, slot_idx, keys, grad, gstride, recv, H, C, G, bnd, lgP, p, stats,
                   acc_stripes, ffnb, kw);
}

// The owner's half of one merged exchange (models/sparse_lr.py mx_exchange) in ONE
// launch, one workgroup per key-range partition q of the owner's ordered home:
//   resolve  lookup-or-insert of the pulled keys of partition q from every source row
//            (row word b0.. holds the row's partition bounds, written by the sender's
//            key pack), their slots / keys / bounds for the later apply, and their
//            weights into the next exchange's send rows (row stride H)
//   apply    the pushes of partition q (kv_apply_part semantics: one optimizer step per
//            source row, rank order) at the slots an earlier resolve recorded
// post = resolve first (the pulls miss this exchange's pushes), else apply first. A
// key's resolve and apply run in the same workgroup, ordered by a barrier (workgroup
// scope: write-through L1), so no key is read and written by two workgroups.
__global__ __launch_bounds__(256) void kv_owner_part_kernel(
    Slot* __restrict__ slots, int64_t cap, uint64_t mask, uint64_t home_base, uint64_t home_m,
    int home_shr, const int32_t* __restrict__ recv, int64_t H, int64_t C, int kw, int G,
    int64_t b0, int lgP, int64_t* __restrict__ slot_out, uint64_t* __restrict__ key_out,
    int32_t* __restrict__ bnd_out, float* __restrict__ wout, int init_type, float init_v,
    float init_s, uint64_t seed, int32_t* __restrict__ err, int32_t* __restrict__ inserted,
    const int64_t* __restrict__ slot_idx, const uint64_t* __restrict__ keys,
    const float* __restrict__ grad, int64_t gstride, const int32_t* __restrict__ bnd_in,
    int do_apply, int post, UpdateParams p, double* __restrict__ stats, int acc_stripes) {
  __shared__ int32_t sa[kMaxChain], roff[kMaxChain + 1];
  const int tid = threadIdx.x, P = 1 << lgP, q = blockIdx.x;
  for (int phase = 0; phase < 2; ++phase) {
    const bool resolve = (phase == 0) == (post != 0);
    if (!resolve) {
      if (do_apply)
        apply_part_block(slots, cap, slot_idx, keys, grad, gstride, recv, H, C, G, bnd_in, lgP,
                         p, stats, acc_stripes);
      __syncthreads();
      continue;
    }
    if (tid < G) {
      const int32_t* row = recv + (int64_t)tid * H;
      const int32_t n = (int32_t)dev_len(row, C);
      const int32_t* rb = row + b0;
      const int32_t a = min(max(rb[q], 0), n), b = min(max(rb[q + 1], a), n);
      sa[tid] = a;
      roff[tid + 1] = b - a;
      int32_t* ob = bnd_out + (int64_t)tid * (P + 1);
      ob[q] = a;
      if (q == P - 1) ob[P] = n;
    }
    __syncthreads();
    if (tid == 0) {
      roff[0] = 0;
      for (int s = 0; s < G; ++s) roff[s + 1] += roff[s];
    }
    __syncthreads();
    const int tot = roff[G];
    int local_ins = 0;
    for (int w = tid; w < tot; w += blockDim.x) {
      int lo = 0, hi = G - 1;  // row of entry w: last s with roff[s] <= w
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (roff[mid] <= w) lo = mid; else hi = mid - 1;
      }
      const int s = lo;
      const int64_t i = sa[s] + (w - roff[s]);
      const int32_t* row = recv + (int64_t)s * H;
      const uint64_t h = kw == 1 ? (uint64_t)(uint32_t)row[4 + i]
                                 : reinterpret_cast<const uint64_t*>(row + 4)[i];
      float wv;
      const int64_t found = resolve_key(slots, mask, home_base, home_m, home_shr, h, 1,
                                        init_type, init_v, init_s, seed, &wv, &local_ins);
      if (found < 0 && err) atomicOr(err, 1);
      slot_out[(int64_t)s * C + i] = found;
      key_out[(int64_t)s * C + i] = h;
      wout[(int64_t)s * H + i] = wv;
    }
    if (inserted) {
      const int t = wave_sum(local_ins);
      if ((threadIdx.x & 63) == 0 && t) atomicAdd(inserted, t);
    }
    __syncthreads();
  }
}

// Occupancy / sparsity census: out[0] = occupied slots, out[1] = nonzero w.
__global__ void kv_census_kernel(const Slot* __restrict__ slots, int64_t cap,
                                 unsigned long long* __restrict__ out) {
  unsigned long long occ = 0, nz = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < cap;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = slots[i].key;
    if (k != kEmptyKey) {
      ++occ;
      nz += slots[i].w != 0.f;
    }
  }
  occ = wave_sum(occ);
  nz = wave_sum(nz);
  if ((threadIdx.x & 63) == 0) {
    if (occ) atomicAdd(&out[0], occ);
    if (nz) atomicAdd(&out[1], nz);
  }
}

// ---------------------------------------------------------------------------
// Host launchers
void kv_init(void* slots, int64_t cap, hipStream_t st) {
  kv_init_kernel<<<grid_for(cap, 256, 8192), 256, 0, st>>>((Slot*)slots, cap);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void kv_resolve(void* slots, int64_t cap, const uint64_t* keys, int64_t n, const int32_t* n_dev,
                int64_t* out_slot, float* out_w, bool insert, int init_type, float init_v,
                float init_s, uint64_t seed, int32_t* err, int32_t* inserted, uint64_t home_base,
                uint64_t home_m, hipStream_t st) {
  int lg = 0;
  while ((1ll << lg) < cap) ++lg;
  kv_resolve_kernel<<<grid_for(n, 256), 256, 0, st>>>(
      (Slot*)slots, (uint64_t)(cap - 1), home_base, home_m, 64 - lg, keys, n, n_dev, out_slot,
      out_w, insert ? 1 : 0, init_type, init_v, init_s, seed, err, inserted);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void kv_resolve_rows(void* slots, int64_t cap, const int32_t* recv, int G, int64_t H, int64_t C,
                     int kw, int64_t* out_slot, float* out_w, int64_t wstride, bool insert,
                     int init_type, float init_v, float init_s, uint64_t seed, int32_t* err,
                     int32_t* inserted, uint64_t home_base, uint64_t home_m, uint64_t* out_key,
                     int32_t* bnd, int lgP, hipStream_t st) {
  int lg = 0;
  while ((1ll << lg) < cap) ++lg;
  dim3 grid(grid_for(C, 256, 1024), G);
  if (bnd && !home_m) throw std::runtime_error("kv_resolve_rows: partition bounds need an ordered home");
  kv_resolve_rows_kernel<<<grid, 256, 0, st>>>(
      (Slot*)slots, (uint64_t)(cap - 1), home_base, home_m, 64 - lg, recv, H, C, kw, out_slot,
      out_w, wstride > 0 ? wstride : C, insert ? 1 : 0, init_type, init_v, init_s, seed, err,
      inserted, out_key, bnd, lgP);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void kv_gather(const void* slots, int64_t cap, const int64_t* slot_idx, int64_t n,
               const int32_t* n_dev, float* out, int field, hipStream_t st) {
  kv_gather_kernel<<<grid_for(n, 256), 256, 0, st>>>((const Slot*)slots, cap, slot_idx, n, n_dev,
                                                     out, field);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void kv_set(void* slots, int64_t cap, const int64_t* slot_idx, int64_t n, const float* w,
            const float* z, const float* nn, hipStream_t st) {
  kv_set_kernel<<<grid_for(n, 256), 256, 0, st>>>((Slot*)slots, cap, slot_idx, n, w, z, nn);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void kv_update(void* slots, int64_t cap, const int64_t* slot_idx, const float* grad, int64_t n,
               const int32_t* n_dev, int algo, int lr_type, float alpha, float beta, float l1,
               float l2, float grad_scale, float max_delta, double* stats, int acc_stripes,
               uint32_t* hist, int nbins, int hist_stripes, double* metrics,
               int64_t* step_counter, hipStream_t st) {
  UpdateParams p{algo, lr_type, alpha, beta, l1, l2, grad_scale, max_delta};
  if (hist && nbins != 2048) throw std::runtime_error("kv_update: the fused AUC needs 2048 bins");
  kv_update_kernel<<<grid_for(n, 256), 256, 0, st>>>((Slot*)slots, cap, slot_idx, grad, n, n_dev,
                                                     p, stats, acc_stripes, hist, nbins,
                                                     hist_stripes, metrics, step_counter);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void kv_accumulate(void* slots, int64_t cap, const int64_t* slot_idx, const float* grad,
                   int64_t n, const int32_t* n_dev, int64_t* touched, int32_t* n_touched,
                   int64_t touched_cap, hipStream_t st) {
  kv_accumulate_kernel<<<grid_for(n, 256), 256, 0, st>>>((Slot*)slots, cap, slot_idx, grad, n,
                                                         n_dev, touched, n_touched, touched_cap);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void kv_accumulate_rows(void* slots, int64_t cap, const int64_t* slot_idx, const float* grad,
                        int64_t gstride, const int32_t* recv, int G, int64_t H, int64_t C,
                        int64_t* touched, int32_t* n_touched, int64_t touched_cap,
                        hipStream_t st) {
  dim3 grid(grid_for(C, 256, 1024), G);
  kv_accumulate_rows_kernel<<<grid, 256, 0, st>>>((Slot*)slots, cap, slot_idx, grad, gstride, recv,
                                                  H, C, touched, n_touched, touched_cap);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void kv_apply_accumulated(void* slots, int64_t cap, const int64_t* touched, const int32_t* n_touched,
                          int64_t max_n, int algo, int lr_type, float alpha, float beta, float l1,
                          float l2, float grad_scale, float max_delta, double* stats, int acc_stripes,
                          hipStream_t st) {
  UpdateParams p{algo, lr_type, alpha, beta, l1, l2, grad_scale, max_delta};
  kv_apply_accumulated_kernel<<<grid_for(max_n, 256), 256, 0, st>>>((Slot*)slots, cap, touched,
                                                                    n_touched, max_n, p, stats,
                                                                    acc_stripes);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void kv_update_rows(void* slots, int64_t cap, const int64_t* slot_idx, const float* grad,
                    int64_t gstride, const int32_t* recv, int G, int64_t H, int64_t C,
                    unsigned long long* link, int64_t link_size, int32_t* nxt, int algo,
                    int lr_type, float alpha, float beta, float l1, float l2, float grad_scale,
                    float max_delta, double* stats, int acc_stripes, hipStream_t st) {
  if (cap > (int64_t(1) << 32)) throw std::runtime_error("kv_update_rows: capacity > 2^32");
  if (link_size < 2 * (int64_t)G * C || (link_size & (link_size - 1)))
    throw std::runtime_error("kv_update_rows: link scratch must be a power of two >= 2*G*C");
  if (G < 1 || G > kMaxChain) throw std::runtime_error("kv_update_rows: 1..64 source rows");
  UpdateParams p{algo, lr_type, alpha, beta, l1, l2, grad_scale, max_delta};
  fill_async<unsigned long long>(link, link_size, ~0ull, st);
  dim3 grid(grid_for(C, 256, 1024), G);
  kv_link_rows_kernel<<<grid, 256, 0, st>>>(slot_idx, cap, grad, gstride, recv, H, C, link,
                                            (uint64_t)(link_size - 1), nxt);
  PSAMD_HIP_CHECK(hipGetLastError());
  kv_apply_rows_kernel<<<grid, 256, 0, st>>>((Slot*)slots, cap, slot_idx, grad, gstride, recv, H,
                                             C, link, (uint64_t)(link_size - 1), nxt,
                                             (int64_t)G * C, p, stats, acc_stripes);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void kv_apply_part(void* slots, int64_t cap, const int64_t* slot_idx, const uint64_t* keys,
                   const float* grad, int64_t gstride, const int32_t* recv, int G, int64_t H,
                   int64_t C, const int32_t* bnd, int lgP, int algo, int lr_type, float alpha,
                   float beta, float l1, float l2, float grad_scale, float max_delta,
                   double* stats, int acc_stripes, int ffnb, int kw, hipStream_t st) {
  if (cap > (int64_t(1) << 32) - 1) throw std::runtime_error("kv_apply_part: capacity >= 2^32");
  if ((int64_t)G * C >= (int64_t(1) << 31)) throw std::runtime_error("kv_apply_part: G*C >= 2^31");
  if (G < 1 || G > kMaxChain) throw std::runtime_error("kv_apply_part: 1..64 source rows");
  if (lgP < 0 || lgP > 20) throw std::runtime_error("kv_apply_part: lgP in 0..20");
  UpdateParams p{algo, lr_type, alpha, beta, l1, l2, grad_scale, max_delta};
  kv_apply_part_kernel<<<1 << lgP, 256, 0, st>>>((Slot*)slots, cap, slot_idx, keys, grad, gstride,
                                                 recv, H, C, G, bnd, lgP, p, stats, acc_stripes,
                                                 ffnb, kw);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void kv_owner_part(void* slots, int64_t cap, uint64_t home_base, uint64_t home_m,
                   const int32_t* recv, int G, int64_t H, int64_t C, int kw, int64_t b0, int lgP,
                   int64_t* slot_out, uint64_t* key_out, int32_t* bnd_out, float* wout,
                   int init_type, float init_v, float init_s, uint64_t seed, int32_t* err,
                   int32_t* inserted, const int64_t* slot_idx, const uint64_t* keys,
                   const float* grad, int64_t gstride, const int32_t* bnd_in, bool do_apply,
                   bool post, int algo, int lr_type, float alpha, float beta, float l1, float l2,
                   float grad_scale, float max_delta, double* stats, int acc_stripes,
                   hipStream_t st) {
  if (cap > (int64_t(1) << 32) - 1) throw std::runtime_error("kv_owner_part: capacity >= 2^32");
  if ((int64_t)G * C >= (int64_t(1) << 31)) throw std::runtime_error("kv_owner_part: G*C >= 2^31");
  if (G < 1 || G > kMaxChain) throw std::runtime_error("kv_owner_part: 1..64 source rows");
  if (lgP < 0 || lgP > 20) throw std::runtime_error("kv_owner_part: lgP in 0..20");
  if (!home_m) throw std::runtime_error("kv_owner_part: needs an ordered home");
  int lg = 0;
  while ((1ll << lg) < cap) ++lg;
  UpdateParams p{algo, lr_type, alpha, beta, l1, l2, grad_scale, max_delta};
  kv_owner_part_kernel<<<1 << lgP, 256, 0, st>>>(
      (Slot*)slots, cap, (uint64_t)(cap - 1), home_base, home_m, 64 - lg, recv, H, C, kw, G, b0,
      lgP, slot_out, key_out, bnd_out, wout, init_type, init_v, init_s, seed, err, inserted,
      slot_idx, keys, grad, gstride, bnd_in, do_apply ? 1 : 0, post ? 1 : 0, p, stats,
      acc_stripes);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void kv_census(const void* slots, int64_t cap, unsigned long long* out, hipStream_t st) {
  kv_census_kernel<<<grid_for(cap, 256, 4096), 256, 0, st>>>((const Slot*)slots, cap, out);
  PSAMD_HIP_CHECK(hipGetLastError());
}

}  // namespace psamd
