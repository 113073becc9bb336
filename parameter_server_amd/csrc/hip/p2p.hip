// One-sided peer-HBM data plane ("p2p" exchange, asynchronous SGD without collectives).
//
// Reference: the async-SGD worker issues every minibatch's pull without a barrier and
// never waits for another worker (src/app/linear_method/async_sgd.h:219-238); the
// server applies each push as it arrives (src/parameter/kv_store.h:47-57). Over RCCL
// every push / pull is a collective, so one slow rank stalls all of them. Here each
// rank maps its peers' shards and inboxes into its own address space (IPC handles,
// exchanged once at setup) and moves data with plain loads / stores over xGMI:
//
//   pull   p2p_lookup_rows: the keys of row p (owned by peer p) are probed straight in
//          peer p's open-addressing table (read only; a key the owner has not inserted
//          yet reads as its init value); the local row resolves with insert into the
//          own shard. No message, no owner involvement.
//   push   p2p_post: row p (keys + gradients of this step for owner p, in the padded
//          exchange's row layout [nkeys, ngrads, min, max | keys | f32 gradients or
//          FixingFloat nb-byte codes]) is written into peer p's inbox ring entry
//          [self][seq % Q]; a release fence at system scope, then the entry's sequence
//          word in the inbox's sequence area (after the G x Q entries). The ring has Q
//          entries per source: a pusher waits (bounded spin on the owner's applied
//          counter) only when it is Q steps ahead of what that owner has applied, the
//          staleness bound of this mode.
//   apply  p2p_gather: the owner snapshots, per source, whether the next entry's
//          sequence word has arrived (system-scope acquire) and copies the ready
//          entries into one G-row staging buffer; kv_resolve_rows + kv_update_rows
//          (kv_table.hip) then apply them with per-push semantics (rank order per key);
//          p2p_commit publishes the applied counters the pushers read.
//
// The inbox and the applied counters are written by one GPU and read by another inside
// running kernels (a pusher spins on an owner's counter), so they live in FINE-GRAINED
// device memory (hipExtMallocWithFlags(hipDeviceMallocFinegrained), exported through
// the same IPC handles): coarse-grained memory is only coherent across devices at kernel
// boundaries.
//
// Every kernel here is bounded: a wait gives up after `spin` microseconds (s_memrealtime)
// and reports through err (bit 8) instead of hanging; the post's last kernel publishes
// err into pinned host memory, so the trainer fails at the first push that gave up
// (its sequence number is consumed: the owner would wait for it forever).
#include "kv_slot.cuh"

#include <hip/hip_runtime.h>

#include <cstring>
#include <stdexcept>

namespace psamd {

constexpr int kP2pMaxPeers = 64;

struct PeerTab {  // a peer's (or the own) shard geometry, mirrored as 5 int64 per peer
  Slot* slots;
  uint64_t mask;
  uint64_t home_base;
  uint64_t home_m;
  int64_t shr;
};
static_assert(sizeof(PeerTab) == 40, "PeerTab is 5 x 8 bytes");

__device__ __forceinline__ int32_t p2p_load_acquire(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void p2p_store_release(int32_t* p, int32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// pull: grid (blocks, G); row p of `send` holds send[p*H] keys at send + p*H + 4.
__global__ void __launch_bounds__(256)
p2p_lookup_rows_kernel(const PeerTab* __restrict__ tabs, int self, const int32_t* __restrict__ send,
                       int64_t H, int64_t C, int kw, float* __restrict__ wout,
                       int64_t* __restrict__ slot_out, int init_type, float init_v, float init_s,
                       uint64_t seed, int32_t* __restrict__ err, int32_t* __restrict__ inserted) {
  const int p = blockIdx.y;
  const int32_t* row = send + (int64_t)p * H;
  const int64_t n = dev_len(row, C);
  const PeerTab tb = tabs[p];
  const bool own = p == self;
  int local_ins = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t h = kw == 1 ? (uint64_t)(uint32_t)row[4 + i]
                               : reinterpret_cast<const uint64_t*>(row + 4)[i];
    float w;
    const int64_t found = resolve_key(tb.slots, tb.mask, tb.home_base, tb.home_m, (int)tb.shr, h,
                                      own ? 1 : 0, init_type, init_v, init_s, seed, &w,
                                      &local_ins);
    if (own) {
      if (found < 0 && err) atomicOr(err, 1);
      slot_out[(int64_t)p * C + i] = found;
    } else if (found < 0) {
      w = init_value(h, init_type, init_v, init_s, seed);  // what the owner will insert
    }
    wout[(int64_t)p * C + i] = w;
  }
  if (inserted) {
    const int tot = wave_sum(local_ins);
    if ((threadIdx.x & 63) == 0 && tot) atomicAdd(inserted, tot);
  }
}

// push, step 1 (one block): ring space of every peer. ok[p] = 1 once peer p has applied
// through seq - Q from this source (its applied counter lives in its memory).
__global__ void p2p_space_kernel(int32_t* const* __restrict__ applied, int G, int self,
                                 int32_t seq, int Q, int64_t spin, int32_t* __restrict__ ok,
                                 int32_t* __restrict__ err) {
  const int p = threadIdx.x;
  if (p >= G) return;
  if (p == self) {
    ok[p] = 0;
    return;
  }
  const int32_t* a = applied[p] + self;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz constant clock
  while (p2p_load_acquire(a) < seq - Q) {
    if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > spin * 100) {  // spin: microseconds
      atomicOr(err, 8);
      ok[p] = 0;
      return;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  ok[p] = 1;
}

// gradient words of a row with ng gradients: f32, or nb-byte FixingFloat codes
__device__ __forceinline__ int64_t p2p_grad_words(int64_t ng, int nb) {
  return nb ? (ng * nb + 3) / 4 : ng;
}

// push, step 2: grid (blocks, G). Copies the live words of row p (the 4 header words,
// nkeys keys, the gradient words) into peer p's ring entry; the entry's sequence word
// is written by p2p_flag_kernel after this launch completed.
__global__ void __launch_bounds__(256)
p2p_copy_kernel(const int32_t* __restrict__ send, int64_t H, int64_t C, int kw, int nb,
                int32_t* const* __restrict__ rings, int self, int32_t seq, int Q,
                const int32_t* __restrict__ ok) {
  const int p = blockIdx.y;
  if (!ok[p]) return;
  const int32_t* row = send + (int64_t)p * H;
  int32_t* dst = rings[p] + ((int64_t)self * Q + (seq - 1) % Q) * H;
  const int64_t nk = dev_len(row, C), ng = dev_len(row + 1, C);
  const int64_t g0 = 4 + C * kw;
  const int64_t tot = 4 + nk * kw + p2p_grad_words(ng, nb);
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < tot;
       e += (int64_t)gridDim.x * blockDim.x) {
    int64_t o;
    if (e < 4) o = e;
    else if (e < 4 + nk * kw) o = e;
    else o = g0 + (e - 4 - nk * kw);
    dst[o] = row[o];
  }
  __threadfence_system();
}

// the sequence word of ring entry [src][q] sits after the G x Q entries of H words
__device__ __forceinline__ int64_t p2p_seq_word(int G, int Q, int64_t H, int src, int q) {
  return (int64_t)G * Q * H + (int64_t)src * Q + q;
}

__global__ void p2p_flag_kernel(int32_t* const* __restrict__ rings, int64_t H, int G, int self,
                                int32_t seq, int Q, const int32_t* __restrict__ ok,
                                const int32_t* __restrict__ err, int32_t* __restrict__ err_host) {
  const int p = threadIdx.x;
  if (p == 0 && err_host)  // (the space kernel's give-up, for the host to raise on)
    __hip_atomic_store(err_host, *err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (p >= G || !ok[p]) return;
  __threadfence_system();
  p2p_store_release(rings[p] + p2p_seq_word(G, Q, H, self, (seq - 1) % Q), seq);
}

// apply, step 1 (one block): which source has its next entry ready; stage row headers.
__global__ void p2p_ready_kernel(const int32_t* __restrict__ inbox, const int32_t* __restrict__ applied,
                                 int G, int self, int Q, int64_t H, int32_t* __restrict__ stage,
                                 int32_t* __restrict__ ready) {
  const int s = threadIdx.x;
  if (s >= G) return;
  int32_t r = 0, hd[4] = {0, 0, 0, 0};
  if (s != self) {
    const int32_t next = applied[s] + 1;
    const int32_t* e = inbox + ((int64_t)s * Q + (next - 1) % Q) * H;
    if (p2p_load_acquire(inbox + p2p_seq_word(G, Q, H, s, (next - 1) % Q)) == next) {
      r = 1;
      for (int k = 0; k < 4; ++k) hd[k] = e[k];
    }
  }
  ready[s] = r;
  for (int k = 0; k < 4; ++k) stage[(int64_t)s * H + k] = hd[k];
}

// apply, step 2: grid (blocks, G): the ready entries' keys and gradients -> staging rows.
__global__ void __launch_bounds__(256)
p2p_stage_kernel(const int32_t* __restrict__ inbox, const int32_t* __restrict__ applied, int Q,
                 int64_t H, int64_t C, int kw, int nb, const int32_t* __restrict__ ready,
                 int32_t* __restrict__ stage) {
  const int s = blockIdx.y;
  if (!ready[s]) return;
  const int32_t next = applied[s] + 1;
  const int32_t* e = inbox + ((int64_t)s * Q + (next - 1) % Q) * H;
  int32_t* d = stage + (int64_t)s * H;
  const int64_t nk = dev_len(d, C), ng = dev_len(d + 1, C);
  const int64_t g0 = 4 + C * kw, gw = p2p_grad_words(ng, nb);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nk * kw + gw;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t o = i < nk * kw ? 4 + i : g0 + (i - nk * kw);
    d[o] = e[o];
  }
}

// apply, step 3: publish the applied counters (read remotely by the pushers).
__global__ void p2p_commit_kernel(int32_t* __restrict__ applied, const int32_t* __restrict__ ready,
                                  int G, int64_t* __restrict__ total) {
  const int s = threadIdx.x;
  if (s >= G || !ready[s]) return;
  p2p_store_release(applied + s, applied[s] + 1);
  if (total) atomicAdd(reinterpret_cast<unsigned long long*>(total), 1ull);
}

// ---------------------------------------------------------------------------- host
static void p2p_check_g(int G, int self) {
  if (G < 1 || G > kP2pMaxPeers || self < 0 || self >= G)
    throw std::runtime_error("p2p: 1..64 ranks, 0 <= self < G");
}

void p2p_lookup_rows(const void* tabs, int G, int self, const int32_t* send, int64_t H,
                     int64_t C, int kw, float* wout, int64_t* slot_out, int init_type,
                     float init_v, float init_s, uint64_t seed, int32_t* err, int32_t* inserted,
                     hipStream_t st) {
  p2p_check_g(G, self);
  dim3 grid(grid_for(C, 256, 1024), G);
  p2p_lookup_rows_kernel<<<grid, 256, 0, st>>>((const PeerTab*)tabs, self, send, H, C, kw, wout,
                                               slot_out, init_type, init_v, init_s, seed, err,
                                               inserted);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void p2p_post(const int32_t* send, int64_t H, int64_t C, int kw, int nb, int G, int self,
              int32_t seq, int Q, void* const* rings, void* const* applied, int32_t* ok,
              int32_t* err, int32_t* err_host, int64_t spin, hipStream_t st) {
  p2p_check_g(G, self);
  if (seq < 1 || Q < 1) throw std::runtime_error("p2p_post: seq >= 1, Q >= 1");
  if (nb < 0 || nb > 7) throw std::runtime_error("p2p_post: FixingFloat 0..7 bytes");
  p2p_space_kernel<<<1, 64, 0, st>>>((int32_t* const*)applied, G, self, seq, Q, spin, ok, err);
  PSAMD_HIP_CHECK(hipGetLastError());
  dim3 grid(grid_for(2 * C, 256, 256), G);
  p2p_copy_kernel<<<grid, 256, 0, st>>>(send, H, C, kw, nb, (int32_t* const*)rings, self, seq, Q,
                                        ok);
  PSAMD_HIP_CHECK(hipGetLastError());
  p2p_flag_kernel<<<1, 64, 0, st>>>((int32_t* const*)rings, H, G, self, seq, Q, ok, err,
                                    err_host);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void p2p_gather(const int32_t* inbox, const int32_t* applied, int G, int self, int Q, int64_t H,
                int64_t C, int kw, int nb, int32_t* stage, int32_t* ready, hipStream_t st) {
  p2p_check_g(G, self);
  p2p_ready_kernel<<<1, 64, 0, st>>>(inbox, applied, G, self, Q, H, stage, ready);
  PSAMD_HIP_CHECK(hipGetLastError());
  dim3 grid(grid_for(2 * C, 256, 256), G);
  p2p_stage_kernel<<<grid, 256, 0, st>>>(inbox, applied, Q, H, C, kw, nb, ready, stage);
  PSAMD_HIP_CHECK(hipGetLastError());
}

// Fine-grained device memory (coherent across devices while kernels run), zeroed.
void* p2p_fine_alloc(size_t bytes) {
  void* p = nullptr;
  PSAMD_HIP_CHECK(hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained));
  PSAMD_HIP_CHECK(hipMemset(p, 0, bytes));
  return p;
}
void p2p_fine_free(void* p) { (void)hipFree(p); }

void p2p_commit(int32_t* applied, const int32_t* ready, int G, int64_t* total, hipStream_t st) {
  p2p_commit_kernel<<<1, 64, 0, st>>>(applied, ready, G, total);
  PSAMD_HIP_CHECK(hipGetLastError());
}

// IPC: export a device buffer (any pointer inside a hipMalloc allocation) as
// [hipIpcMemHandle_t | offset], import it as a device pointer in this process.
static_assert(sizeof(hipIpcMemHandle_t) <= 64, "IPC handle size");

void ipc_export(const void* ptr, uint8_t* out72) {
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  PSAMD_HIP_CHECK(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)ptr));
  hipIpcMemHandle_t h;
  PSAMD_HIP_CHECK(hipIpcGetMemHandle(&h, (void*)base));
  std::memset(out72, 0, 72);
  std::memcpy(out72, &h, sizeof(h));
  const int64_t off = (const char*)ptr - (const char*)base;
  std::memcpy(out72 + 64, &off, 8);
}

void* ipc_import(const uint8_t* in72) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, in72, sizeof(h));
  int64_t off = 0;
  std::memcpy(&off, in72 + 64, 8);
  void* base = nullptr;
  PSAMD_HIP_CHECK(hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess));
  return (char*)base + off;
}

void ipc_close(void* ptr, int64_t off) {
  PSAMD_HIP_CHECK(hipIpcCloseMemHandle((char*)ptr - off));
}

}  // namespace psamd
