// LDS atomic throughput probe: 1024-thread workgroups, 8192-entry LDS array, each lane
// issues ITERS atomics to pseudo-random (or strided) addresses. Prints ns per
// workgroup-round and cycles per wave-instruction estimate (clock64 deltas).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE>  // 0 ds_add_f32, 1 ds_add_u32, 2 ds_add_u64, 3 ds_write_b32 (no atomic), 4 ds_add_rtn_u32,
                     // 5 ds_cmpst_rtn_b32 (atomicCAS), 6 ds_max_u32, 7 ds_add_rtn_f32
__global__ void __launch_bounds__(1024) k(const uint16_t* idx, float* out, long long* cyc, int iters) {
  __shared__ uint64_t a64[8192];
  float* af = reinterpret_cast<float*>(a64);
  uint32_t* au = reinterpret_cast<uint32_t*>(a64);
  for (int i = threadIdx.x; i < 8192; i += 1024) a64[i] = 0;
  __syncthreads();
  const long long t0 = clock64();
  uint32_t acc = 0;
  for (int it = 0; it < iters; ++it) {
    const int e = idx[(blockIdx.x * 1024 + threadIdx.x) * 8 + (it & 7)] & 8191;
    if (MODE == 0) atomicAdd(&af[e], 1.0f);
    else if (MODE == 1) atomicAdd(&au[e], 1u);
    else if (MODE == 2) atomicAdd((unsigned long long*)&a64[e], 1ull);
    else if (MODE == 3) au[e] = it;
    else if (MODE == 4) acc += atomicAdd(&au[e], 1u);
    else if (MODE == 5) acc += atomicCAS(&au[e], (uint32_t)it, (uint32_t)it + 1);
    else if (MODE == 6) atomicMax(&au[e], (uint32_t)it);
    else acc += (uint32_t)atomicAdd(&af[e], 1.0f);
  }
  __syncthreads();
  const long long t1 = clock64();
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
  out[blockIdx.x * 1024 + threadIdx.x] = af[threadIdx.x] + acc;
}

// global atomics into a per-workgroup 8192-entry slice (no cross-CU sharing)
template <int MODE>  // 0 f32 add, 1 u32 add, 2 u64 add, 3 u32 CAS, 4 f64 add
__global__ void __launch_bounds__(1024) kg(const uint16_t* idx, void* arr, int iters) {
  float* af = reinterpret_cast<float*>(arr) + (size_t)blockIdx.x * 8192 * 2;
  uint32_t* au = reinterpret_cast<uint32_t*>(arr) + (size_t)blockIdx.x * 8192 * 2;
  unsigned long long* a64 = reinterpret_cast<unsigned long long*>(arr) + (size_t)blockIdx.x * 8192;
  double* ad = reinterpret_cast<double*>(arr) + (size_t)blockIdx.x * 8192;
  for (int it = 0; it < iters; ++it) {
    const int e = idx[(blockIdx.x * 1024 + threadIdx.x) * 8 + (it & 7)] & 8191;
    if (MODE == 0) atomicAdd(&af[e], 1.0f);
    else if (MODE == 1) atomicAdd(&au[e], 1u);
    else if (MODE == 2) atomicAdd(&a64[e], 1ull);
    else if (MODE == 3) atomicCAS(&au[e], (uint32_t)it, (uint32_t)it + 1);
    else atomicAdd(&ad[e], 1.0);
  }
}

int main() {
  const int WG = 256 * 2, N = WG * 1024 * 8, IT = 10;
  uint16_t* h = (uint16_t*)malloc(N * 2);
  for (int dist = 0; dist < 3; ++dist) {
    uint32_t s = 12345;
    for (int i = 0; i < N; ++i) {
      s = s * 1664525u + 1013904223u;
      // 0: uniform random over 8192; 1: zipf-ish hot (1/8 of lanes on 16 hot entries); 2: lane-linear
      h[i] = dist == 0 ? (s >> 16) & 8191 : dist == 1 ? (((s >> 8) & 7) == 0 ? (s >> 20) & 15 : (s >> 16) & 8191) : (i / 8) & 8191;
    }
    uint16_t* d; float* o; long long* c;
    hipMalloc(&d, N * 2); hipMalloc(&o, WG * 1024 * 4); hipMalloc(&c, WG * 8);
    hipMemcpy(d, h, N * 2, hipMemcpyHostToDevice);
    const char* names[] = {"ds_add_f32", "ds_add_u32", "ds_add_u64", "ds_write_b32", "ds_add_rtn_u32",
                           "ds_cmpst_rtn_b32", "ds_max_u32", "ds_add_rtn_f32"};
    for (int m = 0; m < 8; ++m) {
      hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(a);
        if (m == 0) k<0><<<WG, 1024>>>(d, o, c, IT);
        if (m == 1) k<1><<<WG, 1024>>>(d, o, c, IT);
        if (m == 2) k<2><<<WG, 1024>>>(d, o, c, IT);
        if (m == 3) k<3><<<WG, 1024>>>(d, o, c, IT);
        if (m == 4) k<4><<<WG, 1024>>>(d, o, c, IT);
        if (m == 5) k<5><<<WG, 1024>>>(d, o, c, IT);
        if (m == 6) k<6><<<WG, 1024>>>(d, o, c, IT);
        if (m == 7) k<7><<<WG, 1024>>>(d, o, c, IT);
        hipEventRecord(b); hipEventSynchronize(b);
      }
      float ms; hipEventElapsedTime(&ms, a, b);
      long long hc[WG]; hipMemcpy(hc, c, WG * 8, hipMemcpyDeviceToHost);
      double mc = 0; for (int i = 0; i < WG; ++i) mc += hc[i]; mc /= WG;
      printf("dist %d %-15s kernel %.1f us, cycles per WG loop %.0f, per wave-instr (16 waves x %d) %.1f\n",
             dist, names[m], ms * 1e3, mc, IT, mc / (16.0 * IT));
    }
    void* g; (void)hipMalloc(&g, (size_t)WG * 8192 * 8); (void)hipMemset(g, 0, (size_t)WG * 8192 * 8);
    const char* gn[] = {"global f32 add", "global u32 add", "global u64 add", "global u32 CAS", "global f64 add"};
    for (int m = 0; m < 5; ++m) {
      hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
      for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(a);
        if (m == 0) kg<0><<<WG, 1024>>>(d, g, IT);
        if (m == 1) kg<1><<<WG, 1024>>>(d, g, IT);
        if (m == 2) kg<2><<<WG, 1024>>>(d, g, IT);
        if (m == 3) kg<3><<<WG, 1024>>>(d, g, IT);
        if (m == 4) kg<4><<<WG, 1024>>>(d, g, IT);
        (void)hipEventRecord(b); (void)hipEventSynchronize(b);
      }
      float ms; (void)hipEventElapsedTime(&ms, a, b);
      printf("dist %d %-15s kernel %.1f us for %d atomics (%.1f G/s)\n", dist, gn[m], ms * 1e3,
             WG * 1024 * IT, WG * 1024.0 * IT / (ms * 1e-3) / 1e9);
    }
    (void)hipFree(g);
    hipFree(d); hipFree(o); hipFree(c);
  }
  return 0;
}
