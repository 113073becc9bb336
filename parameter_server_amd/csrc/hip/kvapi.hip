// Generic k-value push / pull of the GPU KVWorker / KVServer API
// (parameter/sharded_kv.py) on the fixed-row exchange of exchange.hip.
//
// Reference: KVVector<K, V> carries k values per key (src/parameter/kv_vector.h:13-100),
// a push / pull is one message per server sliced by key range
// (src/system/message.h:120-159) and the server merges values with a PLUS / ASSIGN
// op (kv_vector.h:70-75). Here a call's keys are localised on the device (sorted
// unique mixed keys + CSC order), every peer gets a fixed row
//   [hdr 4 | keys C*kw | values C*k f32]
// (header word 0 = live key count), rows go through ONE equal-split all-to-all, and
// the owner resolves, serves or merges all G source rows in one launch each. No
// per-call sizes reach the host, so push / pull never synchronise the stream.
// Registered key sets (KVWorker.register_keys, the reference's KeyCachingFilter,
// src/filter/key_caching.h:6-76) push key-less rows [hdr 4 | values C*k] (kw = 0)
// against the owner's cached slots, and their pulls need no request rows at all: the
// owner serves its cached slots straight into the one value all-to-all.
#include "common.cuh"

namespace psamd {

constexpr int kApiMaxPeers = 64;

__device__ __forceinline__ int api_owner_of_pos(const int64_t* soff, int G, int64_t j) {
  int lo = 0, hi = G - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (soff[mid] <= j) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// Duplicate keys of a push are summed per unique key in CSC order (positions of a
// key's run are ascending: the localiser's sort is stable), so the reduction order
// is deterministic. Thread = (unique key u, value column j): consecutive lanes read
// consecutive columns of one position row.
__global__ void kvv_pack_vals_kernel(const float* __restrict__ vals, int k,
                                     const int32_t* __restrict__ pos_s,
                                     const int32_t* __restrict__ seg_start,
                                     const int32_t* __restrict__ n_uniq, int64_t u_cap,
                                     int64_t nnz, const int64_t* __restrict__ off, int G,
                                     int64_t C, int kw, int64_t H, int32_t* __restrict__ send) {
  __shared__ int64_t soff[kApiMaxPeers + 1];
  for (int t = threadIdx.x; t <= G; t += blockDim.x) soff[t] = off[t];
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x < G) {  // header word 1: value count (= key count)
    const int64_t cnt = soff[threadIdx.x + 1] - soff[threadIdx.x];
    send[(int64_t)threadIdx.x * H + 1] = (int32_t)(cnt < C ? cnt : C);
    if (kw == 0) send[(int64_t)threadIdx.x * H] = (int32_t)(cnt < C ? cnt : C);  // key-less row
  }
  const int64_t n = dev_len(n_uniq, u_cap);
  const int64_t total = n * k;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t u = e / k;
    const int j = (int)(e - u * k);
    const int p = api_owner_of_pos(soff, G, u);
    const int64_t i = u - soff[p];
    if (i >= C) continue;
    int64_t r0 = seg_start[u], r1 = seg_start[u + 1];
    r0 = r0 < 0 ? 0 : (r0 > nnz ? nnz : r0);
    r1 = r1 < r0 ? r0 : (r1 > nnz ? nnz : r1);
    float s = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
      const int64_t pos = pos_s[r];
      if (in_range(pos, nnz)) s += vals[pos * k + j];
    }
    reinterpret_cast<float*>(send + (int64_t)p * H + 4 + C * kw)[i * k + j] = s;
  }
}

// Owner: the value rows of every resolved entry of every source row -> rec[s*C*k ..].
// grid.y = source row; table row sl starts at table_vals + sl * stride (stride = k for a
// [cap, k] value block, 8 floats for the w field of the 32-B KV slots).
__global__ void kvv_serve_kernel(const int32_t* __restrict__ recv, int64_t H, int64_t C,
                                 const int64_t* __restrict__ slot,
                                 const float* __restrict__ table_vals, int64_t cap, int k,
                                 int64_t stride, float* __restrict__ rec) {
  const int s = blockIdx.y;
  const int64_t n = dev_len(recv + (int64_t)s * H, C);
  const int64_t total = n * k;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / k;
    const int j = (int)(e - i * k);
    const int64_t sl = slot[(int64_t)s * C + i];
    rec[(int64_t)s * C * k + e] = in_range(sl, cap) ? table_vals[sl * stride + j] : 0.f;
  }
}

// Owner merge of pushed values, all source rows in one launch (grid.y = source row):
// op 0 = PLUS (float atomics: the sum over sources commutes), op 1 = ASSIGN (called
// once per source row in rank order, s_begin .. s_begin + gridDim.y).
__global__ void kvv_apply_kernel(const int32_t* __restrict__ recv, int64_t H, int64_t C, int kw,
                                 int s_begin, const int64_t* __restrict__ slot,
                                 float* __restrict__ table_vals, int64_t cap, int k, int op) {
  const int s = s_begin + blockIdx.y;
  const int32_t* row = recv + (int64_t)s * H;
  const int64_t n = dev_len(row, C);
  const float* v = reinterpret_cast<const float*>(row + 4 + C * kw);
  const int64_t total = n * k;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / k;
    const int j = (int)(e - i * k);
    const int64_t sl = slot[(int64_t)s * C + i];
    if (!in_range(sl, cap)) continue;
    const float x = v[e];
    if (x != x) continue;  // SparseFilter NaN mark: no value for this key
    if (op == 0) atomicAdd(&table_vals[sl * k + j], x);
    else table_vals[sl * k + j] = x;
  }
}

// Pulled records -> values in request order: out[i, :] = record of key i's unique id.
__global__ void kvv_unpack_kernel(const float* __restrict__ rec, int64_t C, int k,
                                  const int64_t* __restrict__ off, int G,
                                  const int32_t* __restrict__ local_col, int64_t nnz,
                                  float* __restrict__ out) {
  __shared__ int64_t soff[kApiMaxPeers + 1];
  for (int t = threadIdx.x; t <= G; t += blockDim.x) soff[t] = off[t];
  __syncthreads();
  const int64_t total = nnz * k;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / k;
    const int j = (int)(e - i * k);
    const int64_t u = local_col[i];
    const int p = api_owner_of_pos(soff, G, u);
    const int64_t idx = u - soff[p];
    out[e] = (u >= 0 && u < soff[G] && idx < C) ? rec[((int64_t)p * C + idx) * k + j] : 0.f;
  }
}

// off[G+1] of a single shard from the device unique count (no host read): [0, n].
__global__ void kvv_single_off_kernel(const int32_t* __restrict__ n_uniq, int64_t* __restrict__ off) {
  if (threadIdx.x == 0) {
    off[0] = 0;
    off[1] = n_uniq[0];
  }
}

void kvv_pack_vals(const float* vals, int k, const int32_t* pos_s, const int32_t* seg_start,
                   const int32_t* n_uniq, int64_t u_cap, int64_t nnz, const int64_t* off, int G,
                   int64_t C, int kw, int64_t H, int32_t* send, hipStream_t st) {
  kvv_pack_vals_kernel<<<grid_for(u_cap * k, 256, 4096), 256, 0, st>>>(
      vals, k, pos_s, seg_start, n_uniq, u_cap, nnz, off, G, C, kw, H, send);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void kvv_serve(const int32_t* recv, int G, int64_t H, int64_t C, const int64_t* slot,
               const float* table_vals, int64_t cap, int k, int64_t stride, float* rec,
               hipStream_t st) {
  dim3 grid(grid_for(C * k, 256, 1024), G);
  kvv_serve_kernel<<<grid, 256, 0, st>>>(recv, H, C, slot, table_vals, cap, k, stride, rec);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void kvv_apply(const int32_t* recv, int G, int64_t H, int64_t C, int kw, const int64_t* slot,
               float* table_vals, int64_t cap, int k, int op, hipStream_t st) {
  if (op == 0) {
    dim3 grid(grid_for(C * k, 256, 1024), G);
    kvv_apply_kernel<<<grid, 256, 0, st>>>(recv, H, C, kw, 0, slot, table_vals, cap, k, 0);
    PSAMD_HIP_CHECK(hipGetLastError());
    return;
  }
  for (int s = 0; s < G; ++s) {  // ASSIGN: later source ranks win, as in rank order
    dim3 grid(grid_for(C * k, 256, 1024), 1);
    kvv_apply_kernel<<<grid, 256, 0, st>>>(recv, H, C, kw, s, slot, table_vals, cap, k, 1);
    PSAMD_HIP_CHECK(hipGetLastError());
  }
}

void kvv_unpack(const float* rec, int64_t C, int k, const int64_t* off, int G,
                const int32_t* local_col, int64_t nnz, float* out, hipStream_t st) {
  kvv_unpack_kernel<<<grid_for(nnz * k, 256, 4096), 256, 0, st>>>(rec, C, k, off, G, local_col,
                                                                   nnz, out);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void kvv_single_off(const int32_t* n_uniq, int64_t* off, hipStream_t st) {
  kvv_single_off_kernel<<<1, 64, 0, st>>>(n_uniq, off);
  PSAMD_HIP_CHECK(hipGetLastError());
}

}  // namespace psamd
