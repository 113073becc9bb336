// Python bindings (torch tensors in, kernels on the current HIP stream).
// Every op validates device / dtype / contiguity and sizes on the host BEFORE
// launching, so a malformed call raises instead of faulting the GPU.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "common.cuh"
#include "countmin.cuh"

namespace psamd {
// kv_table.hip
void kv_init(void*, int64_t, hipStream_t);
void kv_resolve(void*, int64_t, const uint64_t*, int64_t, const int32_t*, int64_t*, float*, bool,
                int, float, float, uint64_t, int32_t*, int32_t*, uint64_t, uint64_t, hipStream_t);
void kv_accumulate_rows(void*, int64_t, const int64_t*, const float*, int64_t, const int32_t*, int,
                        int64_t, int64_t, int64_t*, int32_t*, int64_t, hipStream_t);
void kv_update_rows(void*, int64_t, const int64_t*, const float*, int64_t, const int32_t*, int,
                    int64_t, int64_t, unsigned long long*, int64_t, int32_t*, int, int, float, float,
                    float, float, float, float, double*, int, hipStream_t);
void kv_resolve_rows(void*, int64_t, const int32_t*, int, int64_t, int64_t, int, int64_t*, float*,
                     int64_t, bool, int, float, float, uint64_t, int32_t*, int32_t*, uint64_t,
                     uint64_t, uint64_t*, int32_t*, int, hipStream_t);
void kv_apply_part(void*, int64_t, const int64_t*, const uint64_t*, const float*, int64_t,
                   const int32_t*, int, int64_t, int64_t, const int32_t*, int, int, int, float, float,
                   float, float, float, float, double*, int, int, int, hipStream_t);
// p2p.hip
void p2p_lookup_rows(const void*, int, int, const int32_t*, int64_t, int64_t, int, float*, int64_t*,
                     int, float, float, uint64_t, int32_t*, int32_t*, hipStream_t);
void p2p_post(const int32_t*, int64_t, int64_t, int, int, int, int, int32_t, int, void* const*,
              void* const*, int32_t*, int32_t*, int32_t*, int64_t, hipStream_t);
void p2p_gather(const int32_t*, const int32_t*, int, int, int, int64_t, int64_t, int, int,
                int32_t*, int32_t*, hipStream_t);
void* p2p_fine_alloc(size_t);
void p2p_fine_free(void*);
void p2p_commit(int32_t*, const int32_t*, int, int64_t*, hipStream_t);
void ipc_export(const void*, uint8_t*);
void* ipc_import(const uint8_t*);
void ipc_close(void*, int64_t);
// tploc.hip
void tp_gather(const uint16_t*, const int32_t*, int64_t, int32_t*, hipStream_t);
bool tp_fwd_bwd_supported(int);
void tp_fb_set_prof(uint64_t*);
void tp_tile_set_prof(uint64_t*);
void tp_fwd_bwd(const uint16_t*, const int32_t*, const int32_t*, int64_t, int, const float*,
                const float*, int64_t, const float*, int64_t, int, float*, double*, uint32_t*, int,
                int, int, float*, const int32_t*, const int32_t*, const int32_t*, float*, int64_t,
                bool, hipStream_t);
void tp_fwd_bwd_csr(const uint16_t*, const int32_t*, const int32_t*, int64_t, const int64_t*,
                    const int32_t*, const float*, const float*, int64_t, const float*, int64_t, int,
                    float*, double*, uint32_t*, int, int, int, float*, const int32_t*,
                    const int32_t*, const int32_t*, float*, int64_t, bool, hipStream_t);
void tp_seg_update(const int32_t*, const int32_t*, int64_t, const int32_t*, const float*,
                   const int32_t*, const int32_t*, unsigned long long*, int64_t, const int64_t*, void*,
                   int64_t, int, int, float, float, float, float, float, float, double*, int,
                   uint32_t*, int, int, double*, int64_t*, hipStream_t);
int tpf_groups(int64_t, int);
int tpf_key_region();
int tpf_entry_region();
size_t tpf_temp_bytes(int64_t, int);
void localize_tpf(const uint64_t*, int64_t, KeyMix, void*, size_t, int32_t*, uint16_t*, uint64_t*,
                  int32_t*, uint16_t*, int32_t*, int32_t*, bool, hipStream_t, const CmArgs*,
                  uint8_t*, float*, int64_t, int32_t*, int);
bool tpf_exchange_ok(int64_t, int, int);
void tpf_pack_keys(int64_t, int, int, const int32_t*, const uint64_t*, int64_t, int, int64_t,
                   int32_t*, int32_t*, const uint64_t*, int64_t, int, hipStream_t);
void tpf_unpack_w(int64_t, int, int, const int32_t*, const int32_t*, const uint16_t*, int64_t,
                  const float*, int64_t, float*, int64_t, hipStream_t);
void tpf_pack_grads(int64_t, int, int, const int32_t*, const int32_t*, const uint16_t*, int64_t, int,
                    int64_t, const float*, int64_t, int32_t*, bool, float*, uint32_t*, int, double*,
                    int64_t*, const int32_t*, int32_t*, hipStream_t);
void tpf_step(int64_t, int, const int32_t*, const int32_t*, const uint16_t*, const uint32_t*,
              const float*, int64_t, const int32_t*, const uint64_t*, const int32_t*,
              const uint16_t*, uint32_t*, float*, int64_t, void*, int64_t, uint64_t, uint64_t, int,
              float, float, uint64_t, int32_t*, int32_t*, int, int, float, float, float, float,
              float, float, double*, int, uint32_t*, int, int, double*, int64_t*, hipStream_t);
int64_t tploc_stride(int64_t);
int64_t tpf_stride(int64_t);
int64_t tpf_stride_max(int64_t);
int tpf_tile_log2(int64_t);
int tploc_buckets(int64_t, int);
int tploc_tile();
bool tploc_supported(int64_t, int);
size_t tploc_temp_bytes(int64_t, int);
void localize_tp(const uint64_t*, int64_t, KeyMix, void*, size_t, int32_t*, uint16_t*, int32_t*,
                 int32_t*, uint64_t*, int32_t*, int32_t*, int32_t*, int32_t*, int32_t*, float*,
                 unsigned long long*, int32_t*, int64_t, uint64_t*, hipStream_t);
void tp_backward(const uint16_t*, const int32_t*, int64_t, const int32_t*, int, const float*,
                 const float*, int64_t, float*, const int32_t*, const int32_t*, const int32_t*,
                 float*, int64_t, hipStream_t);
// gemm256.hip
void gemm_tn256(const __bf16*, int64_t, const __bf16*, int64_t, int, int, int, int, float*, float*,
                float, int, unsigned int*, hipStream_t);
void transpose_bf16(const void*, int, int, void*, hipStream_t);
void gemm_nt256(const __bf16*, int64_t, const __bf16*, int64_t, int, int, int, const float*, bool,
                __bf16*, int64_t, float*, int64_t, int, hipStream_t);
// kvapi.hip
void kvv_pack_vals(const float*, int, const int32_t*, const int32_t*, const int32_t*, int64_t,
                   int64_t, const int64_t*, int, int64_t, int, int64_t, int32_t*, hipStream_t);
void kvv_serve(const int32_t*, int, int64_t, int64_t, const int64_t*, const float*, int64_t, int,
               int64_t, float*, hipStream_t);
void kvv_apply(const int32_t*, int, int64_t, int64_t, int, const int64_t*, float*, int64_t, int, int,
               hipStream_t);
void kvv_unpack(const float*, int64_t, int, const int64_t*, int, const int32_t*, int64_t, float*,
                hipStream_t);
void kvv_single_off(const int32_t*, int64_t*, hipStream_t);
// fm.hip
void fm_fwd_bwd(const void*, const void*, const int64_t*, int64_t, int64_t, const float*, int64_t,
                int, int, const int32_t*, const float*, int64_t, const float*, float*, void*,
                double*, uint32_t*, int, int, hipStream_t);
void fm_l2(float*, const void*, const int64_t*, int64_t, const int32_t*, int64_t, int, float,
           hipStream_t);
// exchange.hip
void xchg_pack_keys(const uint64_t*, const int32_t*, int64_t, const int64_t*, int, int64_t, int,
                    int64_t, int32_t*, int32_t*, const uint64_t*, int64_t, int, hipStream_t);
void kv_owner_part(void*, int64_t, uint64_t, uint64_t, const int32_t*, int, int64_t, int64_t, int,
                   int64_t, int, int64_t*, uint64_t*, int32_t*, float*, int, float, float, uint64_t,
                   int32_t*, int32_t*, const int64_t*, const uint64_t*, const float*, int64_t,
                   const int32_t*, bool, bool, int, int, float, float, float, float, float, float,
                   double*, int, hipStream_t);
void xchg_pack_grads(const float*, const int32_t*, const int32_t*, int64_t, const int64_t*, int,
                     int64_t, int, int64_t, int32_t*, uint32_t*, int, double*, int64_t*, const int32_t*, int32_t*, hipStream_t);
void xchg_clear_counts(int32_t*, int, int64_t, bool, bool, hipStream_t);
void xchg_publish(const int32_t*, int32_t*, hipStream_t);
void xchg_unpack_w(const float*, const int32_t*, const int32_t*, int64_t, const int64_t*, int,
                   int64_t, int64_t, float*, hipStream_t);
void xchg_ff_pack_grads(const float*, const int32_t*, const int32_t*, int64_t, const int64_t*, int,
                        int64_t, int, int64_t, int, uint64_t, const int64_t*, int32_t*, float*,
                        hipStream_t);
void xchg_ff_decode(const int32_t*, int, int64_t, int, int64_t, int, float*, hipStream_t);
void xchg_ff_init(int32_t*, int, int64_t, hipStream_t);
void xchg_ff_encode(const float*, int, int64_t, int, int64_t, int, uint64_t, const int64_t*,
                    int32_t*, int, hipStream_t);
void kv_gather(const void*, int64_t, const int64_t*, int64_t, const int32_t*, float*, int,
               hipStream_t);
void kv_set(void*, int64_t, const int64_t*, int64_t, const float*, const float*, const float*,
            hipStream_t);
void kv_update(void*, int64_t, const int64_t*, const float*, int64_t, const int32_t*, int, int,
               float, float, float, float, float, float, double*, int, uint32_t*, int, int, double*, int64_t*, hipStream_t);
void kv_accumulate(void*, int64_t, const int64_t*, const float*, int64_t, const int32_t*, int64_t*,
                   int32_t*, int64_t, hipStream_t);
void kv_apply_accumulated(void*, int64_t, const int64_t*, const int32_t*, int64_t, int, int, float,
                          float, float, float, float, float, double*, int, hipStream_t);
void kv_census(const void*, int64_t, unsigned long long*, hipStream_t);
// localize.hip
void mix_iota(const uint64_t*, int64_t, KeyMix, uint64_t*, int32_t*, hipStream_t);
void mix_keys(const uint64_t*, int64_t, KeyMix, uint64_t*, bool, hipStream_t);
size_t rocprim_sort_temp_bytes(int64_t, int);
void rocprim_sort_pairs(void*, size_t, const uint64_t*, uint64_t*, const int32_t*, int32_t*,
                        int64_t, int, hipStream_t);
size_t radix_sort_temp_bytes(int64_t);
void radix_sort_pairs(void*, size_t, const uint64_t*, uint64_t*, const int32_t*, int32_t*, int64_t,
                      int, hipStream_t);
size_t scan_temp_bytes(int64_t);
void inclusive_scan_i32(void*, size_t, const int32_t*, int32_t*, int64_t, hipStream_t);
void rle(const uint64_t*, const int32_t*, int64_t, int32_t*, int32_t*, void*, size_t, uint64_t*,
         int32_t*, int32_t*, int32_t*, float*, float*, hipStream_t);
void seg_counts(const int32_t*, const int32_t*, int64_t, uint8_t*, int, hipStream_t);
void owner_split(const uint64_t*, const int32_t*, int64_t, const uint64_t*, int, int64_t*,
                 hipStream_t);
void owner_of(const uint64_t*, int64_t, const uint64_t*, int, int32_t*, hipStream_t);
// sort32.hip
size_t localize32_temp_bytes(int64_t);
size_t partloc_temp_bytes(int64_t, int);
bool partloc_supported(int64_t, int);
void localize_part(const uint64_t*, int64_t, KeyMix, void*, size_t, int32_t*, int32_t*, uint64_t*,
                   int32_t*, int32_t*, int32_t*, float*, float*, int32_t*, int64_t, hipStream_t);
size_t sort40_temp_bytes(int64_t);
void sort40(const uint64_t*, int64_t, KeyMix, void*, size_t, uint64_t*, int32_t*, hipStream_t);
void localize32(const uint64_t*, int64_t, KeyMix, void*, size_t, uint32_t*, int32_t*, int32_t*,
                uint64_t*, int32_t*, int32_t*, int32_t*, float*, float*, int, hipStream_t);
// linear.hip
void linear_fwd(const int64_t*, int64_t, int, const int32_t*, const float*, const float*, int64_t,
                const float*, int, float*, float*, float*, double*, uint32_t*, int, int, int,
                hipStream_t);
void linear_bwd(const int32_t*, const int32_t*, int64_t, const int32_t*, int, const float*,
                const float*, int64_t, const float*, float*, float*, int64_t, hipStream_t);
void auc_from_hist(uint32_t*, int, int, double*, int64_t*, hipStream_t);
void csr_rows(const int64_t*, int64_t, int32_t*, hipStream_t);
void criteo_set_tables(const uint32_t*, const float*);
void criteo_gen(uint64_t, int64_t, const int64_t*, int64_t, int64_t, uint64_t, float, uint64_t*,
                float*, int64_t*, hipStream_t);
void add_i64(int64_t*, int64_t, hipStream_t);
// filters.hip
void cm_insert(uint32_t*, uint64_t, int, int, uint32_t, const uint64_t*, const uint8_t*, int64_t,
               const int32_t*, hipStream_t);
void cm_query(const uint32_t*, uint64_t, int, int, uint32_t, const uint64_t*, int64_t,
              const int32_t*, int, int32_t*, uint8_t*, hipStream_t);
void compact_kept(const int32_t*, const int32_t*, int64_t, const int32_t*, int32_t*, int32_t*,
                  int32_t*, const uint64_t*, uint64_t*, hipStream_t);
void cm_insert_seg(uint32_t*, uint64_t, int, int, uint32_t, const uint64_t*, const int32_t*,
                   int64_t, const int32_t*, hipStream_t);
void ff_minmax(const float*, int64_t, float*, hipStream_t);
void ff_encode(const float*, int64_t, const float*, int, uint64_t, uint8_t*, hipStream_t);
void ff_decode(const uint8_t*, int64_t, const float*, int, float*, hipStream_t);
void key_signature(const uint64_t*, int64_t, unsigned long long*, hipStream_t);
// bcd.hip
void bcd_grad(const int32_t*, const int32_t*, const float*, int64_t, int64_t, int64_t, int64_t,
              const double*, const float*, int64_t, const double*, const uint8_t*, double*,
              double*, hipStream_t);
void bcd_grad_chunked(const int32_t*, const int32_t*, const float*, const int64_t*, int64_t,
                      int64_t, int64_t, const double*, const float*, int64_t, const double*,
                      const uint8_t*, double*, double*, double*, bool, bool, const int32_t*,
                      int64_t, hipStream_t);
void bcd_rowpass(int64_t, double*, const float*, const int32_t*, const float*, const double*,
                 int64_t, const int32_t*, const float*, int64_t, int64_t, const double*,
                 const uint8_t*, int, int, long long*, double*, double*, double*, const int32_t*,
                 int64_t, long long*, bool, hipStream_t);
void bcd_update(int64_t, int64_t, double*, double*, double*, double*, uint8_t*, double*, double,
                double, double, double, unsigned long long*, bool, bool, const long long*, int,
                hipStream_t);
void bcd_replica(int64_t, int64_t, int64_t, int64_t, double*, double*, double*, uint8_t*, double,
                 hipStream_t);
void bcd_dual(const int32_t*, const int32_t*, const float*, int64_t, int64_t, int64_t, int64_t,
              const double*, const float*, double*, int64_t, bool, hipStream_t);
void bcd_objective(const double*, int64_t, double*, hipStream_t);
int bcd_rows_max_cols();
int bcd_part_segments();
void bcd_grad_rows(const int32_t*, const int32_t*, const float*, int64_t, int64_t, int64_t, int64_t,
                   const double*, const float*, int64_t, double*, uint8_t*, int, int,
                   long long*, double*, double*, double*, double*, unsigned long long*,
                   unsigned int*, double, double, double, double, hipStream_t);
void bcd_server_stats(const double*, const uint8_t*, int64_t, int64_t, double*, hipStream_t);
// embedding.hip
void emb_init_rows(const int64_t*, const uint64_t*, int64_t, const int32_t*, int64_t, void*,
                   uint8_t*, int, uint64_t, float, hipStream_t);
void emb_gather_rows(const int64_t*, int64_t, const int32_t*, int64_t, const void*, int, void*,
                     hipStream_t);
void emb_expand(const int32_t*, int64_t, const int64_t*, int64_t, const void*, int64_t, int, void*,
                hipStream_t);
int64_t emb_grad_part_floats(int64_t, int);
void emb_padded_serve(const int32_t*, int64_t, int64_t, int, int, const int64_t*, const float*,
                      int64_t, void*, uint8_t*, int, uint64_t, float, int32_t*, hipStream_t);
void emb_unpack_records(const int32_t*, int64_t, int, const int64_t*, const int32_t*, int64_t,
                        int, void*, float*, hipStream_t);
void emb_pack_grads(const float*, const float*, const int64_t*, const int32_t*, int64_t, int64_t,
                    int, int, int32_t*, hipStream_t);
void emb_grad_reduce(const int32_t*, const int32_t*, const int32_t*, const int32_t*, int64_t,
                     int64_t, const void*, int, float*, float*, const float*, int, float*,
                     hipStream_t);
bool emb_grad_wide_ok(int);
void emb_update(const int64_t*, int64_t, const int32_t*, int64_t, const float*, const void*, void*,
                float*, int, float, float, void*, const float*, const int*, const float*, double*,
                int, hipStream_t);
void wd_head(const void*, int64_t, int, const float*, const float*, const float*, int64_t,
             const int32_t*, int, const float*, float*, void*, float*, float*, float*, double*,
             uint32_t*, int, int, hipStream_t);
void colred_bf16(const void*, int64_t, int, const float*, float*, const float*, float*,
                 hipStream_t);
void adam_update(float*, float*, float*, float*, int64_t, float, float, float, float, float,
                 float, float, void*, const int64_t*, bool, hipStream_t);
// spmv.hip
void spmv(bool, const int64_t*, const void*, int, const void*, int, int64_t, int64_t, const void*,
          int64_t, double, double, void*, int64_t, hipStream_t);
// gemm.hip
void gemm_bf16(bool, bool, const void*, int, const void*, int, int, int, int, int, const float*,
               const void*, int, void*, int, float*, int, float, int, float*, hipStream_t);
}  // namespace psamd

using at::Tensor;
using c10::optional;
namespace py = pybind11;

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check(bool ok, const std::string& msg) {
  if (!ok) throw std::invalid_argument(msg);
}

void chk(const Tensor& t, at::ScalarType dt, const char* name) {
  check(t.is_cuda(), std::string(name) + ": must be a GPU tensor");
  check(t.is_contiguous(), std::string(name) + ": must be contiguous");
  check(t.scalar_type() == dt, std::string(name) + ": wrong dtype " +
                                   std::string(c10::toString(t.scalar_type())));
}

template <typename T>
T* ptr(const Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }

template <typename T>
T* optr(const optional<Tensor>& t, at::ScalarType dt, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  chk(*t, dt, name);
  return reinterpret_cast<T*>(t->data_ptr());
}

uint64_t inv_mod64(uint64_t a) {  // a odd; Newton iteration for a^-1 mod 2^64
  uint64_t x = a;
  for (int i = 0; i < 6; ++i) x *= 2 - a * x;
  return x;
}

psamd::KeyMix make_keymix(int bits) {
  check(bits >= 2 && bits <= 64, "key bits must be in [2, 64]");
  psamd::KeyMix m;
  m.bits = bits;
  m.mask = bits == 64 ? ~0ull : ((1ull << bits) - 1);
  m.a = 0xbf58476d1ce4e5b9ull & m.mask;
  m.b = 0x94d049bb133111ebull & m.mask;
  m.a |= 1;
  m.b |= 1;
  m.ai = inv_mod64(m.a) & m.mask;
  m.bi = inv_mod64(m.b) & m.mask;
  m.s = (bits + 1) / 2;
  return m;
}

// Stripe count of a contended-accumulator buffer (common.cuh acc_stripe).
int acc_stripes_of(const Tensor& t) {
  return t.numel() >= psamd::kAccStripes * psamd::kAccStride ? psamd::kAccStripes : 1;
}
int acc_stripes_of(const optional<Tensor>& t) {
  return t.has_value() && t->defined() ? acc_stripes_of(*t) : 1;
}

int64_t slot_capacity(const Tensor& slots) {
  chk(slots, at::kLong, "slots");
  check(slots.dim() == 2 && slots.size(1) == 4, "slots must be [capacity, 4] int64 (32-B slots)");
  const int64_t cap = slots.size(0);
  check(cap > 0 && (cap & (cap - 1)) == 0, "slot capacity must be a power of two");
  return cap;
}

// ---- validate-once launchers (the single ops and LaunchList share them) ----
using Launch = std::function<void(hipStream_t)>;
// A launch list op gets the list's current stream by reference: kernel ops launch on
// it, control ops switch it or order it against events (a multi-stream iteration of the
// data pipeline as ONE host call, bench.py).
using Op = std::function<void(hipStream_t&)>;
struct LaunchList {
  std::vector<Op> ops;
  std::vector<const char*> names;  // per op (a failing op is named in the error)
  std::vector<py::object> keep;    // the torch streams / events the control ops use
  void push(Launch l, const char* name) {
    ops.push_back([l](hipStream_t& s) { l(s); });
    names.push_back(name);
  }
  void push_op(Op o, const char* name) {
    ops.push_back(std::move(o));
    names.push_back(name);
  }
};

// A linear HIP graph composed natively: child graphs (torch CUDAGraphs captured with
// keep_graph=True, cloned in) and event wait / record nodes, chained in order. One launch
// replays a stream's whole iteration with its cross-stream event edges in the graph
// (bench.py's merged pipeline, PSAMD_MX_G2; benchmarks/probe_graph_events.py).
struct GraphChain {
  hipGraph_t g = nullptr;
  hipGraphExec_t ex = nullptr;
  hipGraphNode_t last = nullptr;
  std::vector<py::object> keep;
  GraphChain() { PSAMD_HIP_CHECK(hipGraphCreate(&g, 0)); }
  ~GraphChain() {
    if (ex) (void)hipGraphExecDestroy(ex);
    if (g) (void)hipGraphDestroy(g);
  }
  GraphChain(const GraphChain&) = delete;
  GraphChain& operator=(const GraphChain&) = delete;
  void chain(hipGraphNode_t n) { last = n; }
  const hipGraphNode_t* deps() const { return last ? &last : nullptr; }
  size_t ndeps() const { return last ? 1 : 0; }
};

Launch make_kv_resolve(Tensor slots, Tensor keys, optional<Tensor> n_dev, Tensor out_slot,
                       optional<Tensor> out_w, bool insert, int init_type, double init_v,
                       double init_s, uint64_t seed, optional<Tensor> err,
                       optional<Tensor> inserted, uint64_t home_base, uint64_t home_m) {
  const int64_t cap = slot_capacity(slots);
  chk(keys, at::kLong, "keys");
  chk(out_slot, at::kLong, "out_slot");
  const int64_t n = keys.numel();
  check(out_slot.numel() >= n, "out_slot too small");
  float* w = optr<float>(out_w, at::kFloat, "out_w");
  if (w) check(out_w->numel() >= n, "out_w too small");
  int32_t* nd = optr<int32_t>(n_dev, at::kInt, "n_dev");
  int32_t* ep = optr<int32_t>(err, at::kInt, "err");
  int32_t* ip = optr<int32_t>(inserted, at::kInt, "inserted");
  // (the lambda's tensor copies keep the buffers alive as long as the launcher)
  return [=, keep = std::vector<optional<Tensor>>{slots, keys, n_dev, out_slot, out_w, err,
                                                  inserted}](hipStream_t st) {
    psamd::kv_resolve(slots.data_ptr(), cap, ptr<uint64_t>(keys), n, nd, ptr<int64_t>(out_slot), w,
                      insert, init_type, (float)init_v, (float)init_s, seed, ep, ip, home_base,
                      home_m, st);
  };
}

Launch make_tp_seg_update(Tensor pos_s, Tensor segid, int64_t n, Tensor n_ent, Tensor psum,
                          Tensor seg_start, Tensor n_uniq, Tensor pieces, Tensor slot_idx,
                          Tensor slots, int algo, int lr_type, double alpha, double beta,
                          double l1, double l2, double grad_scale, double max_delta,
                          optional<Tensor> stats, optional<Tensor> hist, optional<Tensor> metrics,
                          optional<Tensor> step_counter) {
  chk(pos_s, at::kInt, "pos_s");
  chk(segid, at::kInt, "segid");
  chk(n_ent, at::kInt, "n_ent");
  chk(psum, at::kFloat, "psum");
  chk(seg_start, at::kInt, "seg_start");
  chk(n_uniq, at::kInt, "n_uniq");
  chk(pieces, at::kLong, "pieces");
  chk(slot_idx, at::kLong, "slot_idx");
  const int64_t cap = slot_capacity(slots);
  check(n > 0, "tp_seg_update: n > 0");
  check(alpha > 0, "learning rate alpha must be > 0");
  const int64_t N = psamd::tploc_stride(n);
  check(pos_s.numel() >= N && segid.numel() >= N && psum.numel() >= N &&
            seg_start.numel() >= N + 1, "tp_seg_update: entry buffers < stride");
  const int64_t ucap = std::min(pieces.numel(), slot_idx.numel());
  uint32_t* hp = optr<uint32_t>(hist, at::kInt, "hist");
  double* mp = optr<double>(metrics, at::kDouble, "metrics");
  constexpr int kBins = 2048;
  if (hp) check(mp && hist->numel() % (2 * kBins) == 0 && hist->numel() / (2 * kBins) <= 8,
                "tp_seg_update: hist = stripes x 2 x 2048 (<= 8 stripes) with metrics");
  double* sp = optr<double>(stats, at::kDouble, "stats");
  const int sstripes = acc_stripes_of(stats);
  const int hstripes = hp ? (int)(hist->numel() / (2 * kBins)) : 1;
  int64_t* cp = optr<int64_t>(step_counter, at::kLong, "step_counter");
  return [=, keep = std::vector<optional<Tensor>>{pos_s, segid, n_ent, psum, seg_start, n_uniq,
                                                  pieces, slot_idx, slots, stats, hist, metrics,
                                                  step_counter}](hipStream_t st) {
    psamd::tp_seg_update(ptr<int32_t>(pos_s), ptr<int32_t>(segid), n, ptr<int32_t>(n_ent),
                         ptr<float>(psum), ptr<int32_t>(seg_start), ptr<int32_t>(n_uniq),
                         reinterpret_cast<unsigned long long*>(pieces.data_ptr()), ucap,
                         ptr<int64_t>(slot_idx), slots.data_ptr(), cap, algo, lr_type, (float)alpha,
                         (float)beta, (float)l1, (float)l2, (float)grad_scale, (float)max_delta,
                         sp, sstripes, hp, kBins, hstripes, mp, cp, st);
  };
}

// ent_uid = None: the flat layout (w_local = w_ent in tile-entry order, no entry CSC;
// pos_s / segid / n_ent / grad unused and reduce must be false)
Launch make_tp_fwd_bwd(Tensor rep, Tensor dcnt, optional<Tensor> ent_uid, int64_t n, int width,
                       optional<Tensor> vals, Tensor w_local, Tensor labels, int64_t B,
                       int loss_type, Tensor coef, optional<Tensor> metrics,
                       optional<Tensor> hist, int nbins, Tensor psum, optional<Tensor> pos_s,
                       optional<Tensor> segid, optional<Tensor> n_ent, optional<Tensor> grad,
                       bool reduce) {
  chk(rep, at::kShort, "rep");
  chk(dcnt, at::kInt, "dcnt");
  const int32_t* eu = optr<int32_t>(ent_uid, at::kInt, "ent_uid");
  chk(w_local, at::kFloat, "w_local");
  chk(labels, at::kFloat, "labels");
  chk(coef, at::kFloat, "coef");
  chk(psum, at::kFloat, "psum");
  int32_t* ps = optr<int32_t>(pos_s, at::kInt, "pos_s");
  int32_t* sg = optr<int32_t>(segid, at::kInt, "segid");
  int32_t* ne = optr<int32_t>(n_ent, at::kInt, "n_ent");
  float* gr = optr<float>(grad, at::kFloat, "grad");
  check(psamd::tp_fwd_bwd_supported(width) && n == B * (int64_t)width && n > 0,
        "tp_fwd_bwd: fixed width 9..64 (tp_fwd_bwd_supported) and n == B * width");
  const int64_t N = eu ? psamd::tploc_stride(n) : psamd::tpf_stride(n);
  check(rep.numel() >= n && dcnt.numel() >= N / psamd::tploc_tile(), "tp_fwd_bwd: rep / dcnt");
  check(psum.numel() >= N, "tp_fwd_bwd: psum < stride");
  if (eu) {
    check(ent_uid->numel() >= N, "tp_fwd_bwd: ent_uid < stride");
    check(ps && sg && ne && gr && pos_s->numel() >= N && segid->numel() >= N,
          "tp_fwd_bwd: entry CSC buffers");
  } else {
    check(w_local.numel() >= N && !reduce, "tp_fwd_bwd flat: w_ent >= stride, no reduce");
  }
  check(labels.numel() >= B && coef.numel() >= B, "labels/coef too small");
  const float* v = optr<float>(vals, at::kFloat, "vals");
  if (v) check(vals->numel() >= n, "vals too small");
  uint32_t* hp = optr<uint32_t>(hist, at::kInt, "hist");
  if (hp) check(nbins > 0 && nbins <= 8192 && hist->numel() >= 2 * nbins, "hist size");
  double* mp = optr<double>(metrics, at::kDouble, "metrics");
  if (mp) check(metrics->numel() >= 5, "metrics needs >= 5 slots");
  const int mstripes = acc_stripes_of(metrics);
  const int hstripes = hp ? (int)std::max<int64_t>(1, hist->numel() / (2 * nbins)) : 1;
  const int64_t gcap = gr ? grad->numel() : 0;
  return [=, keep = std::vector<optional<Tensor>>{rep, dcnt, ent_uid, vals, w_local, labels, coef,
                                                  metrics, hist, psum, pos_s, segid, n_ent,
                                                  grad}](hipStream_t st) {
    psamd::tp_fwd_bwd(ptr<uint16_t>(rep), ptr<int32_t>(dcnt), eu, n, width, v,
                      ptr<float>(w_local), w_local.numel(), ptr<float>(labels), B, loss_type,
                      ptr<float>(coef), mp, hp, nbins, mstripes, hstripes, ptr<float>(psum),
                      ps, sg, ne, gr, gcap, reduce, st);
  };
}

// Variable-width / valued rows (CSR): row_ptr [B+1] int64, rows [n] int32 (row of every
// occurrence, csr_rows), vals [n] or None. Same buffers / flat rule as make_tp_fwd_bwd.
Launch make_tp_fwd_bwd_csr(Tensor rep, Tensor dcnt, optional<Tensor> ent_uid, int64_t n,
                           Tensor row_ptr, Tensor rows, optional<Tensor> vals, Tensor w_local,
                           Tensor labels, int64_t B, int loss_type, Tensor coef,
                           optional<Tensor> metrics, optional<Tensor> hist, int nbins,
                           Tensor psum, optional<Tensor> pos_s, optional<Tensor> segid,
                           optional<Tensor> n_ent, optional<Tensor> grad, bool reduce) {
  chk(rep, at::kShort, "rep");
  chk(dcnt, at::kInt, "dcnt");
  chk(row_ptr, at::kLong, "row_ptr");
  chk(rows, at::kInt, "rows");
  const int32_t* eu = optr<int32_t>(ent_uid, at::kInt, "ent_uid");
  chk(w_local, at::kFloat, "w_local");
  chk(labels, at::kFloat, "labels");
  chk(coef, at::kFloat, "coef");
  chk(psum, at::kFloat, "psum");
  int32_t* ps = optr<int32_t>(pos_s, at::kInt, "pos_s");
  int32_t* sg = optr<int32_t>(segid, at::kInt, "segid");
  int32_t* ne = optr<int32_t>(n_ent, at::kInt, "n_ent");
  float* gr = optr<float>(grad, at::kFloat, "grad");
  check(n > 0 && B > 0 && row_ptr.numel() >= B + 1 && rows.numel() >= n,
        "tp_fwd_bwd_csr: row_ptr [B+1], rows [n]");
  check(psamd::tploc_stride(n) / psamd::tploc_tile() <= 640, "tp_fwd_bwd_csr: <= 5.2 M keys");
  const int64_t N = eu ? psamd::tploc_stride(n) : psamd::tpf_stride(n);
  check(rep.numel() >= n && dcnt.numel() >= N / psamd::tploc_tile(), "tp_fwd_bwd_csr: rep / dcnt");
  check(psum.numel() >= N, "tp_fwd_bwd_csr: psum < stride");
  if (eu) {
    check(ent_uid->numel() >= N, "tp_fwd_bwd_csr: ent_uid < stride");
    check(!reduce || (ps && sg && ne && gr && pos_s->numel() >= N && segid->numel() >= N),
          "tp_fwd_bwd_csr: entry CSC buffers");
  } else {
    check(w_local.numel() >= N && !reduce, "tp_fwd_bwd_csr flat: w_ent >= stride, no reduce");
  }
  check(labels.numel() >= B && coef.numel() >= B, "labels/coef too small");
  const float* v = optr<float>(vals, at::kFloat, "vals");
  if (v) check(vals->numel() >= n, "vals too small");
  uint32_t* hp = optr<uint32_t>(hist, at::kInt, "hist");
  if (hp) check(nbins > 0 && nbins <= 8192 && hist->numel() >= 2 * nbins, "hist size");
  double* mp = optr<double>(metrics, at::kDouble, "metrics");
  if (mp) check(metrics->numel() >= 5, "metrics needs >= 5 slots");
  const int mstripes = acc_stripes_of(metrics);
  const int hstripes = hp ? (int)std::max<int64_t>(1, hist->numel() / (2 * nbins)) : 1;
  const int64_t gcap = gr ? grad->numel() : 0;
  return [=, keep = std::vector<optional<Tensor>>{rep, dcnt, ent_uid, row_ptr, rows, vals,
                                                  w_local, labels, coef, metrics, hist, psum,
                                                  pos_s, segid, n_ent, grad}](hipStream_t st) {
    psamd::tp_fwd_bwd_csr(ptr<uint16_t>(rep), ptr<int32_t>(dcnt), eu, n, ptr<int64_t>(row_ptr),
                          ptr<int32_t>(rows), v, ptr<float>(w_local), w_local.numel(),
                          ptr<float>(labels), B, loss_type, ptr<float>(coef), mp, hp, nbins,
                          mstripes, hstripes, ptr<float>(psum), ps, sg, ne, gr, gcap, reduce, st);
  };
}

// Owner homes of the merged exchange's partition bounds: [G, 2] int64 (base, m) per owner;
// the bounds (P + 1 words) go at word b0 of each H-word row, past the key words.
const uint64_t* check_homes(const optional<Tensor>& homes, int G, int64_t H, int64_t b0, int lgP,
                            int64_t key_end) {
  if (!homes) return nullptr;
  chk(*homes, at::kLong, "homes");
  check(homes->numel() >= 2 * G, "homes: [G, 2] (base, m) per owner");
  check(lgP >= 0 && lgP <= 20 && b0 >= key_end && b0 + (1 << lgP) + 1 <= H,
        "partition bounds: b0 past the keys, P + 1 words inside the row");
  return reinterpret_cast<const uint64_t*>(homes->data_ptr<int64_t>());
}

// Flat-layout buffers of one localisation (Localizer mode "tpf"): checked against the
// geometry of an n-key minibatch.
struct TpfBufs {
  Tensor cnt, uniqf, ent_pos, ent_j, slot_u;
};
// (partial = true: empty tensors are buffers the caller does not use)
void check_tpf(const TpfBufs& f, int64_t n, int bits, const char* what, bool partial = false) {
  check(psamd::tploc_supported(n, bits), std::string(what) + ": tp geometry (2..34 key bits)");
  const int64_t g = psamd::tpf_groups(n, bits);
  auto need = [&](const Tensor& t, at::ScalarType dt, const char* name, int64_t m) {
    if (partial && t.numel() == 0) return;
    chk(t, dt, name);
    check(t.numel() >= m, std::string(what) + ": " + name + " smaller than the geometry");
  };
  need(f.cnt, at::kInt, "cnt", 4 * g);
  need(f.uniqf, at::kLong, "uniqf", g * psamd::tpf_key_region());
  need(f.ent_pos, at::kInt, "ent_pos", g * psamd::tpf_entry_region());
  need(f.ent_j, at::kShort, "ent_j", g * psamd::tpf_entry_region());
  need(f.slot_u, at::kInt, "slot_u", g * psamd::tpf_key_region());
}

// filt (the fused tail filter, tploc.hip tpf_filter_unit): (cells int32 [the sketch's
// byte cells as words], rsize, rshift, k, vmax, freq, ecnt uint8 [>= tpf_stride_max(n)],
// w_ent float32 [the FlatLoc's tile-entry weights][, cnt_pre int32 [like cnt]: the
// unfiltered counts])
Launch make_localize_tpf(Tensor keys, int64_t n, int bits, Tensor temp, Tensor dcnt, Tensor rep,
                         Tensor uniqf, Tensor ent_pos, Tensor ent_j, Tensor cnt, Tensor err,
                         bool sorted, optional<py::tuple> filt = {}, int stage = 0) {
  check(stage >= 0 && stage <= 4,
        "localize_tpf: stage 0 (all), 1 (tile), 2 (bucket), 3 (tail filter), 4 (tile + bucket)");
  chk(keys, at::kLong, "keys");
  chk(temp, at::kByte, "temp");
  chk(dcnt, at::kInt, "dcnt");
  chk(rep, at::kShort, "rep");
  chk(err, at::kInt, "err");
  check(n > 0 && keys.numel() >= n, "localize_tpf: n keys");
  check_tpf(TpfBufs{cnt, uniqf, ent_pos, ent_j, ent_pos}, n, bits, "localize_tpf");
  const int64_t T = psamd::tpf_stride(n) / psamd::tploc_tile();
  check(dcnt.numel() >= T && rep.numel() >= n, "localize_tpf: dcnt / rep");
  check((size_t)temp.numel() >= psamd::tpf_temp_bytes(n, bits), "localize_tpf: temp too small");
  const psamd::KeyMix km = make_keymix(bits);
  std::vector<Tensor> keep{keys, temp, dcnt, rep, uniqf, ent_pos, ent_j, cnt, err};
  bool has_f = false;
  psamd::CmArgs ca{};
  Tensor ecnt, w_ent, cnt_pre;
  if (filt && !filt->is_none()) {
    const py::tuple& f = *filt;
    check(f.size() == 8 || f.size() == 9,
          "localize_tpf filt: (cells, rsize, rshift, k, vmax, freq, ecnt, w_ent[, cnt_pre])");
    if (f.size() == 9 && !f[8].is_none()) {
      cnt_pre = f[8].cast<Tensor>();
      chk(cnt_pre, at::kInt, "filt cnt_pre");
      check(cnt_pre.numel() >= cnt.numel(), "localize_tpf filt: cnt_pre smaller than cnt");
      keep.push_back(cnt_pre);
    }
    Tensor cells = f[0].cast<Tensor>();
    ecnt = f[6].cast<Tensor>();
    w_ent = f[7].cast<Tensor>();
    chk(cells, at::kInt, "filt cells");
    chk(ecnt, at::kByte, "filt ecnt");
    chk(w_ent, at::kFloat, "filt w_ent");
    ca.rsize = f[1].cast<uint64_t>();
    ca.rshift = f[2].cast<int>();
    ca.k = f[3].cast<int>();
    ca.vmax = f[4].cast<uint32_t>();
    ca.freq = f[5].cast<int>();
    check(ca.k >= 1 && ca.k <= 30 && ca.vmax >= 1 && ca.vmax <= 255 && ca.freq >= 0 &&
              ca.freq < 255,
          "localize_tpf filt: k / vmax / freq");
    check(ca.rsize > 0 && ca.rsize % 64 == 0 && ca.rshift >= 0 && ca.rshift <= bits &&
              bits - ca.rshift <= 30 &&
              (ca.rsize << (bits - ca.rshift)) <= (uint64_t)cells.numel() * 4,
          "localize_tpf filt: sketch regions exceed the cells");
    check(ecnt.numel() >= psamd::tpf_stride_max(n), "localize_tpf filt: ecnt too small");
    check(w_ent.numel() >= psamd::tpf_stride(n), "localize_tpf filt: w_ent too small");
    ca.cells = ptr<uint32_t>(cells);
    ca.ncells32 = (uint64_t)cells.numel() * 4 <= ((uint64_t)1 << 32) ? 1 : 0;
    keep.push_back(cells);
    keep.push_back(ecnt);
    keep.push_back(w_ent);
    has_f = true;
  }
  return [=, keep = std::move(keep)](hipStream_t st) {
    psamd::localize_tpf(ptr<uint64_t>(keys), n, km, temp.data_ptr(), (size_t)temp.numel(),
                        ptr<int32_t>(dcnt), ptr<uint16_t>(rep), ptr<uint64_t>(uniqf),
                        ptr<int32_t>(ent_pos), ptr<uint16_t>(ent_j), ptr<int32_t>(cnt),
                        ptr<int32_t>(err), sorted, st, has_f ? &ca : nullptr,
                        has_f ? ptr<uint8_t>(ecnt) : nullptr, has_f ? ptr<float>(w_ent) : nullptr,
                        has_f ? w_ent.numel() : 0,
                        cnt_pre.defined() ? ptr<int32_t>(cnt_pre) : nullptr, stage);
  };
}

// The flat step boundary: update A (optional) then pull B (optional), same n.
Launch make_tpf_step(int64_t n, int bits, optional<TpfBufs> A, optional<Tensor> psum,
                     optional<TpfBufs> B, optional<Tensor> w_ent, Tensor slots, int init_type,
                     double init_v, double init_s, uint64_t seed, optional<Tensor> err,
                     optional<Tensor> inserted, uint64_t home_base, uint64_t home_m, int algo,
                     int lr_type, double alpha, double beta, double l1, double l2,
                     double grad_scale, double max_delta, optional<Tensor> stats,
                     optional<Tensor> hist, optional<Tensor> metrics,
                     optional<Tensor> step_counter) {
  const int64_t cap = slot_capacity(slots);
  check(cap <= ((int64_t)1 << 32), "tpf_step: u32 slot ids need <= 2^32 slots");
  check(A.has_value() || B.has_value(), "tpf_step: nothing to do");
  check(alpha > 0, "learning rate alpha must be > 0");
  const int64_t N = psamd::tpf_stride(n);
  if (A) {
    check_tpf(*A, n, bits, "tpf_step A");
    check(psum.has_value(), "tpf_step: update needs psum");
    chk(*psum, at::kFloat, "psum");
    check(psum->numel() >= N, "tpf_step: psum < stride");
  }
  if (B) {
    check_tpf(*B, n, bits, "tpf_step B");
    check(w_ent.has_value(), "tpf_step: pull needs w_ent");
    chk(*w_ent, at::kFloat, "w_ent");
    check(w_ent->numel() >= N, "tpf_step: w_ent < stride");
  }
  uint32_t* hp = optr<uint32_t>(hist, at::kInt, "hist");
  double* mp = optr<double>(metrics, at::kDouble, "metrics");
  constexpr int kBins = 2048;
  if (hp) check(mp && hist->numel() % (2 * kBins) == 0 && hist->numel() / (2 * kBins) <= 8,
                "tpf_step: hist = stripes x 2 x 2048 (<= 8 stripes) with metrics");
  double* sp = optr<double>(stats, at::kDouble, "stats");
  const int sstripes = acc_stripes_of(stats);
  const int hstripes = hp ? (int)(hist->numel() / (2 * kBins)) : 1;
  int64_t* cp = optr<int64_t>(step_counter, at::kLong, "step_counter");
  int32_t* ep = optr<int32_t>(err, at::kInt, "err");
  int32_t* ip = optr<int32_t>(inserted, at::kInt, "inserted");
  std::vector<optional<Tensor>> keep{psum, w_ent, slots, err, inserted, stats, hist, metrics,
                                     step_counter};
  for (const auto* f : {A ? &*A : nullptr, B ? &*B : nullptr})
    if (f) keep.insert(keep.end(), {f->cnt, f->uniqf, f->ent_pos, f->ent_j, f->slot_u});
  const TpfBufs* a = A ? &*A : nullptr;
  const TpfBufs* b = B ? &*B : nullptr;
  auto p32 = [](const TpfBufs* f, Tensor TpfBufs::*m) -> int32_t* {
    return f ? reinterpret_cast<int32_t*>((f->*m).data_ptr()) : nullptr;
  };
  int32_t *ca = p32(a, &TpfBufs::cnt), *pa = p32(a, &TpfBufs::ent_pos);
  uint16_t* ja = reinterpret_cast<uint16_t*>(p32(a, &TpfBufs::ent_j));
  uint32_t* sa = reinterpret_cast<uint32_t*>(p32(a, &TpfBufs::slot_u));
  int32_t *cb = p32(b, &TpfBufs::cnt), *pb = p32(b, &TpfBufs::ent_pos);
  uint16_t* jb = reinterpret_cast<uint16_t*>(p32(b, &TpfBufs::ent_j));
  uint32_t* sb = reinterpret_cast<uint32_t*>(p32(b, &TpfBufs::slot_u));
  uint64_t* ub = reinterpret_cast<uint64_t*>(p32(b, &TpfBufs::uniqf));
  float* ps = A ? ptr<float>(*psum) : nullptr;
  float* we = B ? ptr<float>(*w_ent) : nullptr;
  const int64_t pcap = A ? psum->numel() : 0, wcap = B ? w_ent->numel() : 0;
  return [=](hipStream_t st) {
    (void)keep;
    psamd::tpf_step(n, bits, ca, pa, ja, sa, ps, pcap, cb, ub, pb, jb, sb, we, wcap,
                    slots.data_ptr(), cap, home_base, home_m, init_type, (float)init_v,
                    (float)init_s, seed, ep, ip, algo, lr_type, (float)alpha, (float)beta,
                    (float)l1, (float)l2, (float)grad_scale, (float)max_delta, sp, sstripes, hp,
                    kBins, hstripes, mp, cp, st);
  };
}

// Synthetic minibatch generator with a row cursor kept in the launcher: run k uses rows
// [row0 + k * row_step, + B) (a prepared-minibatch buffer is refilled every row_step / B
// minibatches), so a launch list regenerates fresh data on every run with the row offset
// as a plain launch argument (no device counter, no extra launch).
Launch make_criteo_gen(uint64_t seed, int64_t row0, int64_t row_step, int64_t B,
                       uint64_t num_features, double alpha, Tensor keys, Tensor labels) {
  chk(keys, at::kLong, "keys");
  chk(labels, at::kFloat, "labels");
  check(keys.numel() >= B * 39 && labels.numel() >= B, "criteo_gen buffers too small");
  check(alpha > 1.0, "power-law alpha must be > 1");
  check(num_features > 0 && B > 0, "num_features > 0, B > 0");
  auto cursor = std::make_shared<int64_t>(row0);
  return [=, keep = std::vector<Tensor>{keys, labels}](hipStream_t st) {
    psamd::criteo_gen(seed, *cursor, nullptr, 1, B, num_features, (float)alpha,
                      ptr<uint64_t>(keys), ptr<float>(labels), nullptr, st);
    *cursor += row_step;
  };
}

// (cnt, uniqf, ent_pos, ent_j, slot_u) from Python
optional<TpfBufs> tpf_bufs(const optional<py::tuple>& t) {
  if (!t.has_value() || t->is_none()) return c10::nullopt;
  check(t->size() == 5, "flat buffers: (cnt, uniqf, ent_pos, ent_j, slot_u)");
  return TpfBufs{(*t)[0].cast<Tensor>(), (*t)[1].cast<Tensor>(), (*t)[2].cast<Tensor>(),
                 (*t)[3].cast<Tensor>(), (*t)[4].cast<Tensor>()};
}

hipEvent_t list_event(const py::object& ev, const char* what) {
  const uint64_t v = py::isinstance<py::int_>(ev) ? ev.cast<uint64_t>()
                                                  : ev.attr("cuda_event").cast<uint64_t>();
  check(v != 0, std::string(what) + ": event not created yet (record it once first)");
  return reinterpret_cast<hipEvent_t>(v);
}

}  // namespace

PYBIND11_MODULE(_hipops, m) {
  m.doc() = "parameter_server_amd HIP kernels (gfx950)";

  // Event record / wait on the current stream with the EXTERNAL flags: inside a stream
  // capture they become event record / wait nodes of the graph (cross-graph ordering
  // between graphs replayed on different streams, no host-side event call per replay);
  // outside a capture they act like hipEventRecord / hipStreamWaitEvent.
  m.def("event_record_ext", [](py::object event) {
    PSAMD_HIP_CHECK(hipEventRecordWithFlags(list_event(event, "event_record_ext"), cur_stream(),
                                            hipEventRecordExternal));
  });
  m.def("event_wait_ext", [](py::object event) {
    PSAMD_HIP_CHECK(hipStreamWaitEvent(cur_stream(), list_event(event, "event_wait_ext"),
                                       hipEventWaitExternal));
  });

  m.def("keymix_params", [](int bits) {
    auto k = make_keymix(bits);
    return py::make_tuple(k.mask, k.a, k.b, k.ai, k.bi, k.s, k.bits);
  });

  // ---------------- KV table ----------------
  m.def("kv_init", [](Tensor slots) {
    psamd::kv_init(slots.data_ptr(), slot_capacity(slots), cur_stream());
  });
  m.def("kv_resolve", [](Tensor slots, Tensor keys, optional<Tensor> n_dev, Tensor out_slot,
                         optional<Tensor> out_w, bool insert, int init_type, double init_v,
                         double init_s, uint64_t seed, optional<Tensor> err,
                         optional<Tensor> inserted, uint64_t home_base, uint64_t home_m) {
    make_kv_resolve(slots, keys, n_dev, out_slot, out_w, insert, init_type, init_v, init_s, seed,
                    err, inserted, home_base, home_m)(cur_stream());
  }, py::arg("slots"), py::arg("keys"), py::arg("n_dev"), py::arg("out_slot"),
     py::arg("out_w"), py::arg("insert"), py::arg("init_type"), py::arg("init_v"),
     py::arg("init_s"), py::arg("seed"), py::arg("err"), py::arg("inserted"),
     py::arg("home_base") = 0, py::arg("home_m") = 0);
  // ---------------- factorization machine (fm.hip) ----------------
  m.def("fm_fwd_bwd", [](Tensor X0, optional<Tensor> vals, int64_t B, int S, Tensor local_col,
                         Tensor w_local, Tensor labels, Tensor coef, Tensor dX0, Tensor metrics,
                         optional<Tensor> hist, int nbins) {
    chk(X0, at::kBFloat16, "X0");
    chk(dX0, at::kBFloat16, "dX0");
    chk(local_col, at::kInt, "local_col");
    chk(w_local, at::kFloat, "w_local");
    chk(labels, at::kFloat, "labels");
    chk(coef, at::kFloat, "coef");
    chk(metrics, at::kDouble, "metrics");
    check(X0.dim() == 2 && X0.size(1) <= 128 && X0.size(1) > 0, "X0 must be [B*S, D<=128]");
    check(S > 0 && S <= 64, "1..64 keys per example");
    const int D = (int)X0.size(1);
    check(X0.size(0) >= B * S && dX0.numel() >= B * S * D, "X0/dX0 too small");
    check(local_col.numel() >= B * S && labels.numel() >= B && coef.numel() >= B, "too small");
    check(metrics.numel() >= 3, "metrics[3]");
    const float* v = optr<float>(vals, at::kFloat, "vals");
    if (v) check(vals->numel() >= B * S, "vals too small");
    uint32_t* h = optr<uint32_t>(hist, at::kInt, "hist");
    if (h) check(hist->numel() >= 2 * nbins, "hist too small");
    psamd::fm_fwd_bwd(X0.data_ptr(), nullptr, nullptr, 0, 0, v, B, S, D, ptr<int32_t>(local_col),
                      ptr<float>(w_local),
                      w_local.numel(), ptr<float>(labels), ptr<float>(coef), dX0.data_ptr(),
                      ptr<double>(metrics), h, nbins, acc_stripes_of(metrics), cur_stream());
  });
  m.def("fm_fwd_bwd_gather", [](Tensor rows, optional<Tensor> idx, optional<Tensor> vals, int64_t B,
                                int S, Tensor local_col, Tensor w_local, Tensor labels, Tensor coef,
                                Tensor dX0, Tensor metrics, optional<Tensor> hist, int nbins) {
    // rows [R, D] bf16 read through local_col (and idx) -- no expanded X0
    chk(rows, at::kBFloat16, "rows");
    chk(dX0, at::kBFloat16, "dX0");
    chk(local_col, at::kInt, "local_col");
    chk(w_local, at::kFloat, "w_local");
    chk(labels, at::kFloat, "labels");
    chk(coef, at::kFloat, "coef");
    chk(metrics, at::kDouble, "metrics");
    check(rows.dim() == 2, "rows [R, D]");
    const int D = (int)rows.size(1);
    check(D == 8 || D == 16 || D == 32, "row gather: D in {8, 16, 32}");
    check(S > 0 && S <= 64, "1..64 keys per example");
    check(dX0.numel() >= B * S * D, "dX0 too small");
    check(local_col.numel() >= B * S && labels.numel() >= B && coef.numel() >= B, "too small");
    check(metrics.numel() >= 3, "metrics[3]");
    const int64_t* ip = optr<int64_t>(idx, at::kLong, "idx");
    const float* v = optr<float>(vals, at::kFloat, "vals");
    if (v) check(vals->numel() >= B * S, "vals too small");
    uint32_t* h = optr<uint32_t>(hist, at::kInt, "hist");
    if (h) check(hist->numel() >= 2 * nbins, "hist too small");
    psamd::fm_fwd_bwd(nullptr, rows.data_ptr(), ip, ip ? idx->numel() : 0, rows.size(0), v, B, S,
                      D, ptr<int32_t>(local_col), ptr<float>(w_local), w_local.numel(),
                      ptr<float>(labels), ptr<float>(coef), dX0.data_ptr(), ptr<double>(metrics),
                      h, nbins, acc_stripes_of(metrics), cur_stream());
  });
  m.def("fm_l2", [](Tensor dE, Tensor rows, optional<Tensor> idx, optional<Tensor> n_dev,
                    int64_t u_cap, double lambda) {
    chk(dE, at::kFloat, "dE");
    chk(rows, at::kBFloat16, "rows");
    check(rows.dim() == 2, "rows [n, D]");
    const int D = (int)rows.size(1);
    check(dE.numel() >= u_cap * D, "dE too small");
    const int64_t* ip = optr<int64_t>(idx, at::kLong, "idx");
    if (ip) check(idx->numel() >= u_cap, "idx too small");
    else check(rows.size(0) >= u_cap, "rows too small");
    psamd::fm_l2(ptr<float>(dE), rows.data_ptr(), ip, rows.size(0),
                 optr<int32_t>(n_dev, at::kInt, "n_dev"), u_cap, D, (float)lambda, cur_stream());
  });
  // ---------------- one-sided peer-HBM exchange (p2p.hip) ----------------
  m.def("ipc_export", [](Tensor t) {
    check(t.is_cuda(), "ipc_export: device tensor");
    std::string out(72, '\0');
    psamd::ipc_export(t.data_ptr(), reinterpret_cast<uint8_t*>(&out[0]));
    return py::bytes(out);
  });
  m.def("ipc_import", [](py::bytes b) {
    std::string s = b;
    check(s.size() == 72, "ipc_import: 72-byte handle");
    return (int64_t) reinterpret_cast<intptr_t>(psamd::ipc_import(reinterpret_cast<const uint8_t*>(s.data())));
  });
  m.def("ipc_close", [](int64_t ptr, int64_t off) {
    psamd::ipc_close(reinterpret_cast<void*>(static_cast<intptr_t>(ptr)), off);
  });
  m.def("p2p_lookup_rows", [](Tensor tabs, int G, int self, Tensor send, int64_t H, int64_t C, int kw,
                              Tensor wout, Tensor slot_out, int init_type, double init_v,
                              double init_s, uint64_t seed, Tensor err,
                              optional<Tensor> inserted) {
    chk(tabs, at::kLong, "tabs");
    chk(send, at::kInt, "send");
    chk(wout, at::kFloat, "wout");
    chk(slot_out, at::kLong, "slot_out");
    chk(err, at::kInt, "err");
    check(G >= 1 && G <= 64 && self >= 0 && self < G, "p2p: 1..64 ranks");
    check(tabs.numel() == 5 * G, "tabs: 5 int64 per rank");
    check(kw == 1 || kw == 2, "kw 1 or 2");
    check(H >= 4 + C * kw, "row too short (header + C keys)");
    check(send.numel() >= G * H && wout.numel() >= G * C && slot_out.numel() >= G * C,
          "p2p_lookup_rows buffers too small");
    psamd::p2p_lookup_rows(tabs.data_ptr(), G, self, ptr<int32_t>(send), H, C, kw, ptr<float>(wout),
                           ptr<int64_t>(slot_out), init_type, (float)init_v, (float)init_s, seed,
                           ptr<int32_t>(err), optr<int32_t>(inserted, at::kInt, "inserted"),
                           cur_stream());
  });
  // rings: per peer the base of its inbox = G x Q entries of H words + G x Q sequence words
  m.def("p2p_post", [](Tensor send, int64_t H, int64_t C, int kw, int nb, int G, int self,
                       int64_t seq, int Q, Tensor rings, Tensor applied, Tensor ok, Tensor err,
                       optional<Tensor> err_host, int64_t spin) {
    chk(send, at::kInt, "send");
    chk(rings, at::kLong, "rings");
    chk(applied, at::kLong, "applied");
    chk(ok, at::kInt, "ok");
    chk(err, at::kInt, "err");
    check(G >= 1 && G <= 64 && self >= 0 && self < G, "p2p: 1..64 ranks");
    check(nb >= 0 && nb <= 7, "p2p_post: FixingFloat 0..7 bytes");
    check(rings.numel() == G && applied.numel() == G && ok.numel() >= G, "p2p_post: G pointers");
    const int64_t gw = nb ? (C * nb + 3) / 4 : C;
    check(send.numel() >= G * H && H >= 4 + C * kw + gw, "p2p_post: send rows");
    check(seq >= 1 && seq < (int64_t(1) << 31) && Q >= 1, "p2p_post: 1 <= seq < 2^31, Q >= 1");
    int32_t* eh = nullptr;
    if (err_host.has_value() && err_host->defined()) {
      check(err_host->device().is_cpu() && err_host->is_pinned() &&
                err_host->scalar_type() == at::kInt && err_host->numel() >= 1,
            "err_host must be a pinned int32 host tensor");
      void* dptr = nullptr;
      PSAMD_HIP_CHECK(hipHostGetDevicePointer(&dptr, err_host->data_ptr(), 0));
      eh = reinterpret_cast<int32_t*>(dptr);
    }
    psamd::p2p_post(ptr<int32_t>(send), H, C, kw, nb, G, self, (int32_t)seq, Q,
                    reinterpret_cast<void* const*>(rings.data_ptr()),
                    reinterpret_cast<void* const*>(applied.data_ptr()), ptr<int32_t>(ok),
                    ptr<int32_t>(err), eh, spin, cur_stream());
  });
  m.def("p2p_gather", [](Tensor inbox, Tensor applied, int G, int self, int Q, int64_t H, int64_t C,
                         int kw, int nb, Tensor stage, Tensor ready) {
    chk(inbox, at::kInt, "inbox");
    chk(applied, at::kInt, "applied");
    chk(stage, at::kInt, "stage");
    chk(ready, at::kInt, "ready");
    check(G >= 1 && G <= 64 && self >= 0 && self < G, "p2p: 1..64 ranks");
    check(nb >= 0 && nb <= 7, "p2p_gather: FixingFloat 0..7 bytes");
    check(inbox.numel() >= (int64_t)G * Q * (H + 1) && stage.numel() >= G * H,
          "p2p_gather: inbox = G x Q x (H + 1) words");
    check(applied.numel() >= G && ready.numel() >= G, "p2p_gather: counters");
    psamd::p2p_gather(ptr<int32_t>(inbox), ptr<int32_t>(applied), G, self, Q, H, C, kw, nb,
                      ptr<int32_t>(stage), ptr<int32_t>(ready), cur_stream());
  });
  // a zeroed FINE-GRAINED device buffer (cross-device coherent while kernels run; IPC
  // exportable) as a uint8 tensor that frees itself
  // raw HIP events for native launch lists (handle as an integer; the caller destroys it)
  m.def("event_create", []() {
    hipEvent_t e = nullptr;
    PSAMD_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return reinterpret_cast<uint64_t>(e);
  });
  m.def("event_destroy", [](uint64_t e) {
    if (e) PSAMD_HIP_CHECK(hipEventDestroy(reinterpret_cast<hipEvent_t>(e)));
  });
  m.def("fine_empty", [](int64_t nbytes) {
    check(nbytes > 0, "fine_empty: nbytes > 0");
    int dev = 0;
    PSAMD_HIP_CHECK(hipGetDevice(&dev));
    void* p = psamd::p2p_fine_alloc((size_t)nbytes);
    return torch::from_blob(p, {nbytes}, [](void* q) { psamd::p2p_fine_free(q); },
                            torch::TensorOptions().dtype(at::kByte).device(at::kCUDA, dev));
  });
  m.def("p2p_commit", [](Tensor applied, Tensor ready, int G, optional<Tensor> total) {
    chk(applied, at::kInt, "applied");
    chk(ready, at::kInt, "ready");
    check(G >= 1 && G <= 64 && applied.numel() >= G && ready.numel() >= G, "p2p_commit");
    psamd::p2p_commit(ptr<int32_t>(applied), ptr<int32_t>(ready), G,
                      optr<int64_t>(total, at::kLong, "total"), cur_stream());
  });
  // ---------------- tile dedup + bucket partition localisation (tploc.hip) ----------------
  m.def("tploc_stride", [](int64_t n) { return psamd::tploc_stride(n); });
  // flat layout: entry stride of n keys / bound over minibatches of <= n keys / log2 tile
  m.def("tpf_stride", [](int64_t n) { return psamd::tpf_stride(n); });
  m.def("tpf_stride_max", [](int64_t n) { return psamd::tpf_stride_max(n); });
  m.def("tpf_tile_log2", [](int64_t n) { return psamd::tpf_tile_log2(n); });
  m.def("tploc_buckets", [](int64_t n, int bits) { return psamd::tploc_buckets(n, bits); });
  m.def("tploc_supported", [](int64_t n, int bits) { return psamd::tploc_supported(n, bits); });
  m.def("tploc_temp_bytes", [](int64_t n, int bits) { return (int64_t)psamd::tploc_temp_bytes(n, bits); });
  m.def("localize_tp", [](Tensor keys, int bits, Tensor temp, Tensor dcnt, Tensor rep, Tensor pos_s,
                          Tensor segid, Tensor uniq, Tensor seg_start, Tensor ent_uid,
                          optional<Tensor> local_col, Tensor n_uniq, Tensor n_ent, Tensor grad,
                          optional<Tensor> pieces, Tensor err, optional<Tensor> prof) {
    chk(keys, at::kLong, "keys");
    chk(temp, at::kByte, "temp");
    chk(dcnt, at::kInt, "dcnt");
    chk(rep, at::kShort, "rep");
    chk(pos_s, at::kInt, "pos_s");
    chk(segid, at::kInt, "segid");
    chk(uniq, at::kLong, "uniq");
    chk(seg_start, at::kInt, "seg_start");
    chk(ent_uid, at::kInt, "ent_uid");
    int32_t* lc = optr<int32_t>(local_col, at::kInt, "local_col");
    chk(n_uniq, at::kInt, "n_uniq");
    chk(n_ent, at::kInt, "n_ent");
    chk(grad, at::kFloat, "grad");
    chk(err, at::kInt, "err");
    const int64_t n = keys.numel();
    check(psamd::tploc_supported(n, bits), "tp localisation: 2..34 key bits, n <= 5.2M");
    if (lc) check(local_col->numel() >= n, "local_col too small");
    const int64_t N = psamd::tploc_stride(n);
    const int64_t T = N / psamd::tploc_tile();
    check(pos_s.numel() >= N && segid.numel() >= N && uniq.numel() >= N &&
              seg_start.numel() >= N + 1 && ent_uid.numel() >= N && grad.numel() >= N,
          "tp localisation buffers < stride");
    check(dcnt.numel() >= T && rep.numel() >= n, "tp buffers too small");
    check((size_t)temp.numel() >= psamd::tploc_temp_bytes(n, bits), "tp temp too small");
    psamd::localize_tp(ptr<uint64_t>(keys), n, make_keymix(bits), temp.data_ptr(),
                       (size_t)temp.numel(), ptr<int32_t>(dcnt), ptr<uint16_t>(rep),
                       ptr<int32_t>(pos_s), ptr<int32_t>(segid), ptr<uint64_t>(uniq),
                       ptr<int32_t>(seg_start), ptr<int32_t>(ent_uid), lc,
                       ptr<int32_t>(n_uniq), ptr<int32_t>(n_ent), ptr<float>(grad),
                       reinterpret_cast<unsigned long long*>(optr<int64_t>(pieces, at::kLong, "pieces")),
                       ptr<int32_t>(err), uniq.numel(),
                       reinterpret_cast<uint64_t*>(optr<int64_t>(prof, at::kLong, "prof")),
                       cur_stream());
  });
  m.def("tp_backward", [](Tensor rep, Tensor dcnt, int64_t n, optional<Tensor> rows, int width,
                          optional<Tensor> vals, Tensor coef, Tensor psum, Tensor pos_s,
                          Tensor segid, Tensor n_ent, Tensor grad) {
    chk(rep, at::kShort, "rep");
    chk(dcnt, at::kInt, "dcnt");
    chk(coef, at::kFloat, "coef");
    chk(psum, at::kFloat, "psum");
    chk(pos_s, at::kInt, "pos_s");
    chk(segid, at::kInt, "segid");
    chk(n_ent, at::kInt, "n_ent");
    chk(grad, at::kFloat, "grad");
    const int64_t N = psamd::tploc_stride(n);
    check(n > 0 && rep.numel() >= n && dcnt.numel() >= N / psamd::tploc_tile(), "tp backward: rep / dcnt");
    check(psum.numel() >= N && pos_s.numel() >= N && segid.numel() >= N, "tp backward buffers");
    const int32_t* r = optr<int32_t>(rows, at::kInt, "rows");
    if (r) check(rows->numel() >= n, "rows too small");
    else check(width > 0, "width must be > 0 without rows");
    const float* v = optr<float>(vals, at::kFloat, "vals");
    if (v) check(vals->numel() >= n, "vals too small");
    psamd::tp_backward(ptr<uint16_t>(rep), ptr<int32_t>(dcnt), n, r, width, v, ptr<float>(coef),
                       coef.numel(), ptr<float>(psum), ptr<int32_t>(pos_s), ptr<int32_t>(segid),
                       ptr<int32_t>(n_ent), ptr<float>(grad), grad.numel(), cur_stream());
  });
  m.def("tp_seg_update", [](Tensor pos_s, Tensor segid, int64_t n, Tensor n_ent, Tensor psum,
                            Tensor seg_start, Tensor n_uniq, Tensor pieces,
                            Tensor slot_idx, Tensor slots, int algo, int lr_type, double alpha,
                            double beta, double l1, double l2, double grad_scale,
                            double max_delta, optional<Tensor> stats, optional<Tensor> hist,
                            optional<Tensor> metrics, optional<Tensor> step_counter) {
    make_tp_seg_update(pos_s, segid, n, n_ent, psum, seg_start, n_uniq, pieces, slot_idx, slots,
                       algo, lr_type, alpha, beta, l1, l2, grad_scale, max_delta, stats, hist,
                       metrics, step_counter)(cur_stream());
  });
  m.def("tp_gather", [](Tensor rep, Tensor ent_uid, int64_t n, Tensor local_col) {
    chk(rep, at::kShort, "rep");
    chk(ent_uid, at::kInt, "ent_uid");
    chk(local_col, at::kInt, "local_col");
    check(n > 0 && rep.numel() >= n && local_col.numel() >= n &&
              ent_uid.numel() >= psamd::tploc_stride(n), "tp gather buffers");
    psamd::tp_gather(ptr<uint16_t>(rep), ptr<int32_t>(ent_uid), n, ptr<int32_t>(local_col),
                     cur_stream());
  });
  m.def("tp_fwd_bwd_supported", [](int width) { return psamd::tp_fwd_bwd_supported(width); });
  // ---- flat 1-GPU layout (tploc.hip "tpf")
  m.def("tpf_groups", [](int64_t n, int bits) { return psamd::tpf_groups(n, bits); });
  m.def("tpf_key_region", []() { return psamd::tpf_key_region(); });
  m.def("tpf_entry_region", []() { return psamd::tpf_entry_region(); });
  m.def("tpf_temp_bytes", [](int64_t n, int bits) { return psamd::tpf_temp_bytes(n, bits); });
  m.def("localize_tpf", [](Tensor keys, int bits, Tensor temp, Tensor dcnt, Tensor rep,
                           Tensor uniqf, Tensor ent_pos, Tensor ent_j, Tensor cnt, Tensor err,
                           bool sorted, optional<py::tuple> filt, int stage) {
    make_localize_tpf(keys, keys.numel(), bits, temp, dcnt, rep, uniqf, ent_pos, ent_j, cnt,
                      err, sorted, filt, stage)(cur_stream());
  }, py::arg("keys"), py::arg("bits"), py::arg("temp"), py::arg("dcnt"), py::arg("rep"),
     py::arg("uniqf"), py::arg("ent_pos"), py::arg("ent_j"), py::arg("cnt"), py::arg("err"),
     py::arg("sorted"), py::arg("filt") = py::none(), py::arg("stage") = 0);
  // ---- the padded multi-GPU exchange on the flat layout (rows as in exchange.hip)
  m.def("tpf_exchange_ok", [](int64_t n, int bits, int G) {
    return psamd::tpf_exchange_ok(n, bits, G);
  });
  m.def("tpf_pack_keys", [](int64_t n, int bits, int G, Tensor cnt, Tensor uniqf, int64_t C, int kw,
                            int64_t H, Tensor send, optional<Tensor> ovf, optional<Tensor> homes,
                            int64_t b0, int lgP) {
    check_tpf(TpfBufs{cnt, uniqf, cnt.new_empty({0}, at::kInt), cnt.new_empty({0}, at::kShort),
                      cnt.new_empty({0}, at::kInt)}, n, bits, "tpf_pack_keys", true);
    chk(send, at::kInt, "send");
    check(psamd::tpf_exchange_ok(n, bits, G), "tpf_pack_keys: G a power of two dividing groups");
    check((kw == 1 || kw == 2) && C > 0 && H >= 4 + C * kw + 1 && send.numel() >= G * H,
          "tpf_pack_keys: row geometry");
    const uint64_t* hp = check_homes(homes, G, H, b0, lgP, 4 + C * kw);
    psamd::tpf_pack_keys(n, bits, G, ptr<int32_t>(cnt), ptr<uint64_t>(uniqf), C, kw, H,
                         ptr<int32_t>(send), optr<int32_t>(ovf, at::kInt, "ovf"), hp, b0, lgP,
                         cur_stream());
  }, py::arg("n"), py::arg("bits"), py::arg("G"), py::arg("cnt"), py::arg("uniqf"), py::arg("C"),
     py::arg("kw"), py::arg("H"), py::arg("send"), py::arg("ovf"),
     py::arg("homes") = py::none(), py::arg("b0") = 0, py::arg("lgP") = 0);
  m.def("tpf_unpack_w", [](int64_t n, int bits, int G, Tensor cnt, Tensor ent_pos, Tensor ent_j,
                           int64_t C, Tensor wrecv, Tensor w_ent, int64_t wstride) {
    // wstride: row stride of wrecv (0 = C; the merged exchange reads the weights in
    // place from the received rows)
    const int64_t ws = wstride > 0 ? wstride : C;
    check_tpf(TpfBufs{cnt, cnt.new_empty({0}, at::kLong), ent_pos, ent_j,
                      cnt.new_empty({0}, at::kInt)}, n, bits, "tpf_unpack_w", true);
    chk(wrecv, at::kFloat, "wrecv");
    chk(w_ent, at::kFloat, "w_ent");
    check(psamd::tpf_exchange_ok(n, bits, G), "tpf_unpack_w: G a power of two dividing groups");
    check(C > 0 && ws >= C && wrecv.numel() >= (G - 1) * ws + C &&
          w_ent.numel() >= psamd::tpf_stride(n), "tpf_unpack_w: buffers");
    psamd::tpf_unpack_w(n, bits, G, ptr<int32_t>(cnt), ptr<int32_t>(ent_pos),
                        ptr<uint16_t>(ent_j), C, ptr<float>(wrecv), ws, ptr<float>(w_ent),
                        w_ent.numel(), cur_stream());
  }, py::arg("n"), py::arg("bits"), py::arg("G"), py::arg("cnt"), py::arg("ent_pos"),
     py::arg("ent_j"), py::arg("C"), py::arg("wrecv"), py::arg("w_ent"), py::arg("wstride") = 0);
  m.def("tpf_pack_grads", [](int64_t n, int bits, int G, Tensor cnt, Tensor ent_pos, Tensor ent_j,
                             int64_t C, int kw, int64_t H, Tensor psum, Tensor send,
                             optional<Tensor> gstage, optional<Tensor> hist,
                             optional<Tensor> metrics, optional<Tensor> step_counter,
                             optional<Tensor> ovf, optional<Tensor> ovf_host) {
    check_tpf(TpfBufs{cnt, cnt.new_empty({0}, at::kLong), ent_pos, ent_j,
                      cnt.new_empty({0}, at::kInt)}, n, bits, "tpf_pack_grads", true);
    chk(psum, at::kFloat, "psum");
    chk(send, at::kInt, "send");
    check(psamd::tpf_exchange_ok(n, bits, G), "tpf_pack_grads: G a power of two dividing groups");
    check((kw == 1 || kw == 2) && C > 0 && H >= 4 + C * kw + 1 && send.numel() >= G * H,
          "tpf_pack_grads: row geometry");
    check(psum.numel() >= psamd::tpf_stride(n), "tpf_pack_grads: psum < stride");
    float* gs = optr<float>(gstage, at::kFloat, "gstage");
    if (gs)  // (+ 2 floats per bucket group: the workgroups' min / max partials)
      check(gstage->numel() >= G * C + 2 * (int64_t)psamd::tpf_groups(n, bits),
            "tpf_pack_grads: gstage < G * C + 2 * groups");
    else check(H >= 4 + C * kw + C, "tpf_pack_grads: f32 gradient rows");
    uint32_t* hp = optr<uint32_t>(hist, at::kInt, "hist");
    double* mp = optr<double>(metrics, at::kDouble, "metrics");
    if (hp) check(mp && hist->numel() % 4096 == 0 && hist->numel() / 4096 <= 8,
                  "tpf_pack_grads: hist = stripes x 2 x 2048 with metrics");
    int32_t* op = optr<int32_t>(ovf, at::kInt, "ovf");
    int32_t* oh = nullptr;
    if (ovf_host.has_value() && ovf_host->defined()) {
      check(op && ovf_host->device().is_cpu() && ovf_host->is_pinned() &&
                ovf_host->scalar_type() == at::kInt,
            "ovf_host: pinned int32 host tensor (with ovf)");
      void* dptr = nullptr;
      PSAMD_HIP_CHECK(hipHostGetDevicePointer(&dptr, ovf_host->data_ptr(), 0));
      oh = reinterpret_cast<int32_t*>(dptr);
    }
    psamd::tpf_pack_grads(n, bits, G, ptr<int32_t>(cnt), ptr<int32_t>(ent_pos),
                          ptr<uint16_t>(ent_j), C, kw, H, ptr<float>(psum), psum.numel(),
                          ptr<int32_t>(send), gs != nullptr, gs, hp,
                          hp ? (int)(hist->numel() / 4096) : 1, mp,
                          optr<int64_t>(step_counter, at::kLong, "step_counter"), op, oh,
                          cur_stream());
  });
  m.def("tpf_step", [](int64_t n, int bits, optional<py::tuple> A, optional<Tensor> psum,
                       optional<py::tuple> B, optional<Tensor> w_ent, Tensor slots, int init_type,
                       double init_v, double init_s, uint64_t seed, optional<Tensor> err,
                       optional<Tensor> inserted, uint64_t home_base, uint64_t home_m, int algo,
                       int lr_type, double alpha, double beta, double l1, double l2,
                       double grad_scale, double max_delta, optional<Tensor> stats,
                       optional<Tensor> hist, optional<Tensor> metrics,
                       optional<Tensor> step_counter) {
    make_tpf_step(n, bits, tpf_bufs(A), psum, tpf_bufs(B), w_ent, slots, init_type, init_v,
                  init_s, seed, err, inserted, home_base, home_m, algo, lr_type, alpha, beta, l1,
                  l2, grad_scale, max_delta, stats, hist, metrics, step_counter)(cur_stream());
  });
  // phase marks of the fused kernel (tuning aid): 16 int64 per tile, or None to disable
  m.def("tp_fb_set_prof", [](optional<Tensor> prof) {
    uint64_t* p = nullptr;
    if (prof) {
      chk(*prof, at::kLong, "prof");
      p = reinterpret_cast<uint64_t*>(prof->data_ptr<int64_t>());
    }
    psamd::tp_fb_set_prof(p);
  });
  // phase marks of the tile kernel (tuning aid): 16 int64 per tile, or None to disable
  m.def("tp_tile_set_prof", [](optional<Tensor> prof) {
    uint64_t* p = nullptr;
    if (prof) {
      chk(*prof, at::kLong, "prof");
      p = reinterpret_cast<uint64_t*>(prof->data_ptr<int64_t>());
    }
    psamd::tp_tile_set_prof(p);
  });
  m.def("tp_fwd_bwd", [](Tensor rep, Tensor dcnt, optional<Tensor> ent_uid, int64_t n, int width,
                         optional<Tensor> vals, Tensor w_local, Tensor labels, int64_t B,
                         int loss_type, Tensor coef, optional<Tensor> metrics,
                         optional<Tensor> hist, int nbins, Tensor psum, optional<Tensor> pos_s,
                         optional<Tensor> segid, optional<Tensor> n_ent, optional<Tensor> grad,
                         bool reduce) {
    make_tp_fwd_bwd(rep, dcnt, ent_uid, n, width, vals, w_local, labels, B, loss_type, coef,
                    metrics, hist, nbins, psum, pos_s, segid, n_ent, grad, reduce)(cur_stream());
  });
  m.def("tp_fwd_bwd_csr", [](Tensor rep, Tensor dcnt, optional<Tensor> ent_uid, int64_t n,
                             Tensor row_ptr, Tensor rows, optional<Tensor> vals, Tensor w_local,
                             Tensor labels, int64_t B, int loss_type, Tensor coef,
                             optional<Tensor> metrics, optional<Tensor> hist, int nbins,
                             Tensor psum, optional<Tensor> pos_s, optional<Tensor> segid,
                             optional<Tensor> n_ent, optional<Tensor> grad, bool reduce) {
    make_tp_fwd_bwd_csr(rep, dcnt, ent_uid, n, row_ptr, rows, vals, w_local, labels, B,
                        loss_type, coef, metrics, hist, nbins, psum, pos_s, segid, n_ent, grad,
                        reduce)(cur_stream());
  });
  // A validate-once launch list: the add_* calls check their arguments exactly as the
  // single ops above and keep the tensors alive; run() issues every launch in order on
  // the current stream with no per-call argument conversion. The 1-GPU sparse-LR step
  // (resolve, fused forward + backward, fused scan + update) runs from one per
  // minibatch buffer: three pybind crossings with 60 tensor / scalar arguments cost
  // ~10 us of host issue time per step (profiles/r3_s3_host_issue.log).
  py::class_<GraphChain>(m, "GraphChain")
      .def(py::init<>())
      .def("add_child", [](GraphChain& c, py::object torch_graph) {
        check(c.ex == nullptr, "GraphChain: already instantiated");
        const py::object h = torch_graph.attr("raw_cuda_graph")();
        const hipGraph_t child = reinterpret_cast<hipGraph_t>(h.cast<uint64_t>());
        check(child != nullptr, "GraphChain.add_child: capture with keep_graph=True");
        hipGraphNode_t n;
        PSAMD_HIP_CHECK(hipGraphAddChildGraphNode(&n, c.g, c.deps(), c.ndeps(), child));
        c.chain(n);
        c.keep.push_back(torch_graph);
      })
      .def("add_wait", [](GraphChain& c, py::object event) {
        check(c.ex == nullptr, "GraphChain: already instantiated");
        hipGraphNode_t n;
        PSAMD_HIP_CHECK(hipGraphAddEventWaitNode(&n, c.g, c.deps(), c.ndeps(),
                                                 list_event(event, "GraphChain.add_wait")));
        c.chain(n);
        c.keep.push_back(event);
      })
      .def("add_record", [](GraphChain& c, py::object event) {
        check(c.ex == nullptr, "GraphChain: already instantiated");
        hipGraphNode_t n;
        PSAMD_HIP_CHECK(hipGraphAddEventRecordNode(&n, c.g, c.deps(), c.ndeps(),
                                                   list_event(event, "GraphChain.add_record")));
        c.chain(n);
        c.keep.push_back(event);
      })
      .def("instantiate", [](GraphChain& c) {
        if (!c.ex) PSAMD_HIP_CHECK(hipGraphInstantiate(&c.ex, c.g, nullptr, nullptr, 0));
      })
      .def("launch", [](GraphChain& c) {
        check(c.ex != nullptr, "GraphChain: instantiate first");
        PSAMD_HIP_CHECK(hipGraphLaunch(c.ex, cur_stream()));
      })
      // (like CUDAGraph.reset: frees the executable graph; the caller synchronised)
      .def("reset", [](GraphChain& c) {
        if (c.ex) PSAMD_HIP_CHECK(hipGraphExecDestroy(c.ex));
        c.ex = nullptr;
        c.keep.clear();
      });

  py::class_<LaunchList>(m, "LaunchList")
      .def(py::init<>())
      .def("add_chain", [](LaunchList& l, py::object chain) {
        GraphChain& c = chain.cast<GraphChain&>();
        check(c.ex != nullptr, "add_chain: instantiate the GraphChain first");
        const hipGraphExec_t ex = c.ex;
        l.keep.push_back(chain);
        l.push_op([ex](hipStream_t& s) { PSAMD_HIP_CHECK(hipGraphLaunch(ex, s)); }, "chain");
      })
      .def("add_kv_resolve", [](LaunchList& l, Tensor slots, Tensor keys, optional<Tensor> n_dev,
                                Tensor out_slot, optional<Tensor> out_w, bool insert,
                                int init_type, double init_v, double init_s, uint64_t seed,
                                optional<Tensor> err, optional<Tensor> inserted,
                                uint64_t home_base, uint64_t home_m) {
        l.push(make_kv_resolve(slots, keys, n_dev, out_slot, out_w, insert, init_type,
                                        init_v, init_s, seed, err, inserted, home_base, home_m), "kv_resolve");
      })
      .def("add_tp_fwd_bwd", [](LaunchList& l, Tensor rep, Tensor dcnt, optional<Tensor> ent_uid,
                                int64_t n, int width, optional<Tensor> vals, Tensor w_local,
                                Tensor labels, int64_t B, int loss_type, Tensor coef,
                                optional<Tensor> metrics, optional<Tensor> hist, int nbins,
                                Tensor psum, optional<Tensor> pos_s, optional<Tensor> segid,
                                optional<Tensor> n_ent, optional<Tensor> grad, bool reduce) {
        l.push(make_tp_fwd_bwd(rep, dcnt, ent_uid, n, width, vals, w_local, labels, B,
                                        loss_type, coef, metrics, hist, nbins, psum, pos_s, segid,
                                        n_ent, grad, reduce), "tp_fwd_bwd");
      })
      .def("add_tp_seg_update", [](LaunchList& l, Tensor pos_s, Tensor segid, int64_t n,
                                   Tensor n_ent, Tensor psum, Tensor seg_start, Tensor n_uniq,
                                   Tensor pieces, Tensor slot_idx, Tensor slots, int algo,
                                   int lr_type, double alpha, double beta, double l1, double l2,
                                   double grad_scale, double max_delta, optional<Tensor> stats,
                                   optional<Tensor> hist, optional<Tensor> metrics,
                                   optional<Tensor> step_counter) {
        l.push(make_tp_seg_update(pos_s, segid, n, n_ent, psum, seg_start, n_uniq, pieces,
                                           slot_idx, slots, algo, lr_type, alpha, beta, l1, l2,
                                           grad_scale, max_delta, stats, hist, metrics,
                                           step_counter), "tp_seg_update");
      })
      .def("add_localize_tpf", [](LaunchList& l, Tensor keys, int64_t n, int bits, Tensor temp,
                                  Tensor dcnt, Tensor rep, Tensor uniqf, Tensor ent_pos,
                                  Tensor ent_j, Tensor cnt, Tensor err, bool sorted,
                                  optional<py::tuple> filt, int stage) {
        l.push(make_localize_tpf(keys, n, bits, temp, dcnt, rep, uniqf, ent_pos, ent_j,
                                          cnt, err, sorted, filt, stage), "localize_tpf");
      }, py::arg("keys"), py::arg("n"), py::arg("bits"), py::arg("temp"), py::arg("dcnt"),
         py::arg("rep"), py::arg("uniqf"), py::arg("ent_pos"), py::arg("ent_j"), py::arg("cnt"),
         py::arg("err"), py::arg("sorted"), py::arg("filt") = py::none(), py::arg("stage") = 0)
      .def("add_tpf_step", [](LaunchList& l, int64_t n, int bits, optional<py::tuple> A,
                              optional<Tensor> psum, optional<py::tuple> B,
                              optional<Tensor> w_ent, Tensor slots, int init_type, double init_v,
                              double init_s, uint64_t seed, optional<Tensor> err,
                              optional<Tensor> inserted, uint64_t home_base, uint64_t home_m,
                              int algo, int lr_type, double alpha, double beta, double l1,
                              double l2, double grad_scale, double max_delta,
                              optional<Tensor> stats, optional<Tensor> hist,
                              optional<Tensor> metrics, optional<Tensor> step_counter) {
        l.push(make_tpf_step(n, bits, tpf_bufs(A), psum, tpf_bufs(B), w_ent, slots,
                                      init_type, init_v, init_s, seed, err, inserted, home_base,
                                      home_m, algo, lr_type, alpha, beta, l1, l2, grad_scale,
                                      max_delta, stats, hist, metrics, step_counter), "tpf_step");
      })
      .def("add_criteo_gen", [](LaunchList& l, uint64_t seed, int64_t row0, int64_t row_step,
                                int64_t B, uint64_t num_features, double alpha, Tensor keys,
                                Tensor labels) {
        l.push(make_criteo_gen(seed, row0, row_step, B, num_features, alpha, keys,
                                        labels), "criteo_gen");
      })
      // control ops: a torch.cuda.Stream / torch.cuda.Event (the list keeps a reference:
      // a torch Event destroys its HIP event with the object, and a raw handle left in a
      // list then fails on the next run) or a raw handle the caller owns (event_create).
      // Events must exist already (torch creates them lazily: record once first).
      .def("add_stream", [](LaunchList& l, py::object stream) {
        const uint64_t v = py::isinstance<py::int_>(stream)
                               ? stream.cast<uint64_t>()
                               : stream.attr("cuda_stream").cast<uint64_t>();
        const hipStream_t h = reinterpret_cast<hipStream_t>(v);
        l.keep.push_back(stream);
        l.push_op([h](hipStream_t& s) { s = h; }, "stream");
      })
      .def("add_wait", [](LaunchList& l, py::object event) {
        const hipEvent_t e = list_event(event, "add_wait");
        l.keep.push_back(event);
        l.push_op([e](hipStream_t& s) { PSAMD_HIP_CHECK(hipStreamWaitEvent(s, e, 0)); }, "wait");
      })
      .def("add_record", [](LaunchList& l, py::object event) {
        const hipEvent_t e = list_event(event, "add_record");
        l.keep.push_back(event);
        l.push_op([e](hipStream_t& s) { PSAMD_HIP_CHECK(hipEventRecord(e, s)); }, "record");
      })
      // replay of a captured torch.cuda.CUDAGraph (the list keeps the graph alive):
      // hipGraphLaunch of its executable graph on the list's current stream. Only for
      // graphs whose kernels draw nothing from torch's RNG (torch's replay() also
      // advances the captured generator offsets; ours use their own counters)
      .def("add_graph", [](LaunchList& l, py::object graph) {
        const py::object h = graph.attr("raw_cuda_graph_exec")();
        if (!py::isinstance<py::int_>(h))
          throw std::invalid_argument("add_graph: raw_cuda_graph_exec() is not an int handle");
        const hipGraphExec_t ex = reinterpret_cast<hipGraphExec_t>(h.cast<uint64_t>());
        if (!ex) throw std::invalid_argument("add_graph: graph not instantiated");
        l.keep.push_back(graph);
        l.push_op([ex](hipStream_t& s) { PSAMD_HIP_CHECK(hipGraphLaunch(ex, s)); }, "graph");
      })
      // the ops of another list, SHARED (a generator's row cursor advances for both)
      .def("extend", [](LaunchList& l, const LaunchList& o) {
        l.ops.insert(l.ops.end(), o.ops.begin(), o.ops.end());
        l.names.insert(l.names.end(), o.names.begin(), o.names.end());
        l.keep.insert(l.keep.end(), o.keep.begin(), o.keep.end());
      })
      .def("__len__", [](const LaunchList& l) { return l.ops.size(); })
      .def("run", [](const LaunchList& l) {
        hipStream_t st = cur_stream();
        size_t i = 0;
        try {
          for (; i < l.ops.size(); ++i) l.ops[i](st);
        } catch (const std::exception& e) {
          throw std::runtime_error("LaunchList op " + std::to_string(i) + " of " +
                                   std::to_string(l.ops.size()) + " (" + l.names[i] +
                                   "): " + e.what());
        }
      });
  // ---------------- fixed-capacity exchange (exchange.hip) ----------------
  // buffers: send/recv int32 [G * H]; row layout documented in exchange.hip
  m.def("kv_resolve_rows", [](Tensor slots, Tensor recv, int64_t H, int64_t C, int kw,
                              Tensor out_slot, Tensor out_w, bool insert, int init_type,
                              double init_v, double init_s, uint64_t seed, optional<Tensor> err,
                              optional<Tensor> inserted, uint64_t home_base, uint64_t home_m,
                              optional<Tensor> out_key, optional<Tensor> bnd, int lgP,
                              int64_t wstride) {
    const int64_t cap = slot_capacity(slots);
    const int64_t ws = wstride > 0 ? wstride : C;
    chk(recv, at::kInt, "recv");
    chk(out_slot, at::kLong, "out_slot");
    chk(out_w, at::kFloat, "out_w");
    check(kw == 1 || kw == 2, "kw must be 1 (u32 keys) or 2 (u64 keys)");
    check(C > 0 && H >= 4 + C * kw + 1 && H % 4 == 0, "bad exchange row geometry");
    check(recv.numel() % H == 0, "recv is not a whole number of rows");
    const int G = (int)(recv.numel() / H);
    check(G >= 1 && G <= 64, "1..64 peers");
    check(ws >= C && out_slot.numel() >= G * C && out_w.numel() >= (G - 1) * ws + C,
          "out_slot < G*C or out_w < (G-1)*wstride + C");
    int64_t* ok = optr<int64_t>(out_key, at::kLong, "out_key");
    if (ok) check(out_key->numel() >= G * C, "out_key < G*C");
    int32_t* bp = optr<int32_t>(bnd, at::kInt, "bnd");
    check(lgP >= 0 && lgP <= 20, "lgP in 0..20");
    if (bp) check(bnd->numel() >= G * ((1 << lgP) + 1), "bnd < G*(P+1)");
    psamd::kv_resolve_rows(slots.data_ptr(), cap, ptr<int32_t>(recv), G, H, C, kw,
                           ptr<int64_t>(out_slot), ptr<float>(out_w), ws, insert, init_type,
                           (float)init_v, (float)init_s, seed, optr<int32_t>(err, at::kInt, "err"),
                           optr<int32_t>(inserted, at::kInt, "inserted"), home_base, home_m,
                           reinterpret_cast<uint64_t*>(ok), bp, lgP, cur_stream());
  }, py::arg("slots"), py::arg("recv"), py::arg("H"), py::arg("C"), py::arg("kw"),
     py::arg("out_slot"), py::arg("out_w"), py::arg("insert"), py::arg("init_type"),
     py::arg("init_v"), py::arg("init_s"), py::arg("seed"), py::arg("err"), py::arg("inserted"),
     py::arg("home_base"), py::arg("home_m"), py::arg("out_key") = py::none(),
     py::arg("bnd") = py::none(), py::arg("lgP") = 0, py::arg("wstride") = 0);
  // per-push apply of every source row, partitioned by key range (see kv_apply_part_kernel)
  m.def("kv_apply_part", [](Tensor slots, Tensor slot_idx, Tensor keys, Tensor grad,
                            int64_t gstride, Tensor recv, int64_t H, int64_t C, Tensor bnd, int lgP,
                            int algo, int lr_type, double alpha, double beta, double l1, double l2,
                            double grad_scale, double max_delta, optional<Tensor> stats,
                            int ff_nb, int kw) {
    const int64_t cap = slot_capacity(slots);
    chk(slot_idx, at::kLong, "slot_idx");
    chk(keys, at::kLong, "keys");
    chk(grad, at::kFloat, "grad");
    chk(recv, at::kInt, "recv");
    chk(bnd, at::kInt, "bnd");
    check(C > 0 && H > 4 && recv.numel() % H == 0, "bad exchange row geometry");
    const int G = (int)(recv.numel() / H);
    check(G >= 1 && G <= 64, "1..64 peers");
    // ff_nb > 0: the gradients are the rows' FixingFloat codes (grad unused)
    check(ff_nb >= 0 && ff_nb <= 7 && (kw == 1 || kw == 2), "kv_apply_part: ff_nb / kw");
    if (ff_nb) check(H >= 4 + C * kw + (C * ff_nb + 3) / 4, "kv_apply_part: FixingFloat rows");
    else check(gstride >= C && grad.numel() >= (G - 1) * gstride + C, "grad rows out of bounds");
    check(slot_idx.numel() >= G * C && keys.numel() >= G * C, "slot_idx/keys < G*C");
    check(lgP >= 0 && lgP <= 20, "lgP in 0..20");
    check(bnd.numel() >= G * ((1 << lgP) + 1), "bnd < G*(P+1)");
    double* st = optr<double>(stats, at::kDouble, "stats");
    const int stripes = acc_stripes_of(stats);
    psamd::kv_apply_part(slots.data_ptr(), cap, ptr<int64_t>(slot_idx),
                         reinterpret_cast<const uint64_t*>(keys.data_ptr<int64_t>()),
                         ptr<float>(grad), gstride, ptr<int32_t>(recv), G, H, C, ptr<int32_t>(bnd),
                         lgP, algo, lr_type, (float)alpha, (float)beta, (float)l1, (float)l2,
                         (float)grad_scale, (float)max_delta, st, stripes, ff_nb, kw,
                         cur_stream());
  }, py::arg("slots"), py::arg("slot_idx"), py::arg("keys"), py::arg("grad"), py::arg("gstride"),
     py::arg("recv"), py::arg("H"), py::arg("C"), py::arg("bnd"), py::arg("lgP"), py::arg("algo"),
     py::arg("lr_type"), py::arg("alpha"), py::arg("beta"), py::arg("l1"), py::arg("l2"),
     py::arg("grad_scale"), py::arg("max_delta"), py::arg("stats"), py::arg("ff_nb") = 0,
     py::arg("kw") = 1);
  // aggregated pushes of every source row in one launch; grad row s at grad[s*gstride]
  m.def("kv_accumulate_rows", [](Tensor slots, Tensor slot_idx, Tensor grad, int64_t gstride,
                                 Tensor recv, int64_t H, int64_t C, Tensor touched,
                                 Tensor n_touched) {
    const int64_t cap = slot_capacity(slots);
    chk(slot_idx, at::kLong, "slot_idx");
    chk(grad, at::kFloat, "grad");
    chk(recv, at::kInt, "recv");
    chk(touched, at::kLong, "touched");
    chk(n_touched, at::kInt, "n_touched");
    check(C > 0 && H > 4 && recv.numel() % H == 0, "bad exchange row geometry");
    const int G = (int)(recv.numel() / H);
    check(G >= 1 && G <= 64, "1..64 peers");
    check(gstride >= C && grad.numel() >= (G - 1) * gstride + C, "grad rows out of bounds");
    check(slot_idx.numel() >= G * C, "slot_idx < G*C");
    psamd::kv_accumulate_rows(slots.data_ptr(), cap, ptr<int64_t>(slot_idx), ptr<float>(grad),
                              gstride, ptr<int32_t>(recv), G, H, C, ptr<int64_t>(touched),
                              ptr<int32_t>(n_touched), touched.numel(), cur_stream());
  });
  m.def("kv_update_rows", [](Tensor slots, Tensor slot_idx, Tensor grad, int64_t gstride,
                             Tensor recv, int64_t H, int64_t C, Tensor link, Tensor nxt, int algo,
                             int lr_type, double alpha, double beta, double l1, double l2,
                             double grad_scale, double max_delta, optional<Tensor> stats) {
    const int64_t cap = slot_capacity(slots);
    chk(slot_idx, at::kLong, "slot_idx");
    chk(grad, at::kFloat, "grad");
    chk(recv, at::kInt, "recv");
    chk(link, at::kLong, "link");
    chk(nxt, at::kInt, "nxt");
    check(C > 0 && H > 4 && recv.numel() % H == 0, "bad exchange row geometry");
    const int G = (int)(recv.numel() / H);
    check(G >= 1 && G <= 64, "1..64 peers");
    check(gstride >= C && grad.numel() >= (G - 1) * gstride + C, "grad rows out of bounds");
    check(slot_idx.numel() >= G * C, "slot_idx < G*C");
    check(nxt.numel() >= G * C, "nxt < G*C");
    const int64_t L = link.numel();
    check(L >= 2 * G * C && (L & (L - 1)) == 0, "link: power of two >= 2*G*C");
    double* st = optr<double>(stats, at::kDouble, "stats");
    const int stripes = acc_stripes_of(stats);
    psamd::kv_update_rows(slots.data_ptr(), cap, ptr<int64_t>(slot_idx), ptr<float>(grad), gstride,
                          ptr<int32_t>(recv), G, H, C,
                          reinterpret_cast<unsigned long long*>(link.data_ptr<int64_t>()), L,
                          ptr<int32_t>(nxt), algo, lr_type, (float)alpha, (float)beta, (float)l1,
                          (float)l2, (float)grad_scale, (float)max_delta, st, stripes,
                          cur_stream());
  });
  // ---------------- 256x256 LDS-DMA bf16 GEMM, K-major operands (gemm256.hip) ----------------
  m.def("gemm_nt256", [](Tensor A, Tensor B, int64_t M, int64_t N, int64_t K,
                         optional<Tensor> bias, bool relu, optional<Tensor> C,
                         optional<Tensor> Cf, int variant) {
    chk(A, at::kBFloat16, "A");
    chk(B, at::kBFloat16, "B");
    check(M > 0 && N > 0 && K > 0 && K % 64 == 0, "gemm_nt256: K must be a multiple of 64");
    check(A.numel() >= M * K && B.numel() >= N * K, "gemm_nt256: A [M, K], B [N, K]");
    check(((uintptr_t)A.data_ptr() % 16) == 0 && ((uintptr_t)B.data_ptr() % 16) == 0,
          "gemm_nt256: 16-B aligned operands");
    const float* bp = optr<float>(bias, at::kFloat, "bias");
    if (bp) check(bias->numel() >= N, "bias too small");
    __bf16* cp = C.has_value() && C->defined() ? (chk(*C, at::kBFloat16, "C"), ptr<__bf16>(*C)) : nullptr;
    float* fp = optr<float>(Cf, at::kFloat, "Cf");
    check(cp || fp, "gemm_nt256: need an output");
    if (cp) check(C->numel() >= M * N, "C too small");
    if (fp) check(Cf->numel() >= M * N, "Cf too small");
    check(variant >= 0 && variant <= 6,
          "variant: 0 = one barrier per K-step, 1 = ping-pong, 2 = ping-pong with 2-step "
          "prefetch, 3 = 0 with fragment reads interleaved into the MFMA rows, 4 = 4-slot "
          "LDS ring, 5 = 4 waves of 128 x 128, 6 = 4 with 32x32x16 MFMAs");
    psamd::gemm_nt256(ptr<__bf16>(A), K, ptr<__bf16>(B), K, (int)M, (int)N, (int)K, bp, relu, cp, N,
                      fp, N, variant, cur_stream());
  }, py::arg("A"), py::arg("B"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("bias"),
     py::arg("relu"), py::arg("C"), py::arg("Cf"), py::arg("variant") = 0);
  // C [M, N] f32 = beta C + A^T B for MN-major A [K, M], B [K, N] (the weight gradient):
  // split-K partials into part [splits, M, N], then a fixed-order sum (gemm256.hip)
  m.def("gemm_tn256", [](Tensor A, Tensor B, int64_t M, int64_t N, int64_t K, int64_t splits,
                         Tensor part, Tensor C, double beta, int phase,
                         optional<Tensor> tile_ctr) {
    chk(A, at::kBFloat16, "A");
    chk(B, at::kBFloat16, "B");
    chk(part, at::kFloat, "part");
    chk(C, at::kFloat, "C");
    check(M > 0 && N > 0 && K > 0 && K % 64 == 0 && M % 8 == 0 && N % 8 == 0,
          "gemm_tn256: K % 64, M % 8, N % 8");
    check(splits >= 1 && splits <= K / 64, "gemm_tn256: 1 <= splits <= K / 64");
    check(A.numel() >= K * M && B.numel() >= K * N, "gemm_tn256: A [K, M], B [K, N]");
    check(part.numel() >= splits * M * N && C.numel() >= M * N, "gemm_tn256: part / C size");
    check(((uintptr_t)A.data_ptr() % 16) == 0 && ((uintptr_t)B.data_ptr() % 16) == 0 &&
              ((uintptr_t)C.data_ptr() % 16) == 0 && ((uintptr_t)part.data_ptr() % 16) == 0,
          "gemm_tn256: 16-B aligned operands");
    check(phase >= 0 && phase <= 3,
          "gemm_tn256: phase 0 (both) / 1 (GEMM) / 2 (reduce) / 3 (reduce in the GEMM)");
    auto* tc = reinterpret_cast<unsigned int*>(optr<int32_t>(tile_ctr, at::kInt, "tile_ctr"));
    if (phase == 3)
      check(tc && tile_ctr->numel() >= ((M + 255) / 256) * ((N + 255) / 256),
            "gemm_tn256 phase 3: tile_ctr, one zeroed int32 per 256 x 256 tile");
    psamd::gemm_tn256(ptr<__bf16>(A), M, ptr<__bf16>(B), N, (int)M, (int)N, (int)K, (int)splits,
                      ptr<float>(part), ptr<float>(C), (float)beta, phase, tc, cur_stream());
  }, py::arg("A"), py::arg("B"), py::arg("M"), py::arg("N"), py::arg("K"), py::arg("splits"),
     py::arg("part"), py::arg("C"), py::arg("beta"), py::arg("phase") = 0,
     py::arg("tile_ctr") = py::none());
  m.def("transpose_bf16", [](Tensor in, Tensor out) {
    chk(in, at::kBFloat16, "in");
    chk(out, at::kBFloat16, "out");
    check(in.dim() == 2 && out.numel() >= in.numel(), "transpose_bf16: in [R, C], out [C, R]");
    const int64_t R = in.size(0), C = in.size(1);
    check(R % 64 == 0 && C % 64 == 0, "transpose_bf16: R, C multiples of 64");
    psamd::transpose_bf16(in.data_ptr(), (int)R, (int)C, out.data_ptr(), cur_stream());
  });
  // ---------------- k-value push / pull API (kvapi.hip) ----------------
  // rows [hdr 4 | keys C*kw | values C*k f32] of H words (pull rows: no values)
  m.def("kvv_pack_vals", [](Tensor vals, int64_t k, Tensor pos_s, Tensor seg_start, Tensor n_uniq,
                            Tensor off, int64_t C, int kw, int64_t H, Tensor send) {
    chk(vals, at::kFloat, "vals");
    chk(pos_s, at::kInt, "pos_s");
    chk(seg_start, at::kInt, "seg_start");
    chk(n_uniq, at::kInt, "n_uniq");
    chk(off, at::kLong, "off");
    chk(send, at::kInt, "send");
    const int G = (int)off.numel() - 1;
    check(G >= 1 && G <= 64, "1..64 peers");
    check(k >= 1 && vals.numel() % k == 0, "vals must be [nnz, k]");
    const int64_t nnz = vals.numel() / k;
    check(pos_s.numel() >= nnz, "pos_s < nnz");
    const int64_t u_cap = std::min<int64_t>(seg_start.numel() - 1, nnz);
    check(u_cap >= 1, "seg_start too small");
    check(kw >= 0 && kw <= 2, "kw must be 0 (key-less row of a registered key set), 1 or 2");
    check(C > 0 && H >= 4 + C * kw + C * k && H % 4 == 0, "bad push row geometry");
    check(send.numel() == G * H, "send must be [G * H]");
    psamd::kvv_pack_vals(ptr<float>(vals), (int)k, ptr<int32_t>(pos_s), ptr<int32_t>(seg_start),
                         ptr<int32_t>(n_uniq), u_cap, nnz, ptr<int64_t>(off), G, C, kw, H,
                         ptr<int32_t>(send), cur_stream());
  });
  m.def("kvv_serve", [](Tensor recv, int64_t H, int64_t C, Tensor slot, Tensor vals, Tensor rec) {
    chk(recv, at::kInt, "recv");
    chk(slot, at::kLong, "slot");
    chk(vals, at::kFloat, "vals");
    chk(rec, at::kFloat, "rec");
    check(H >= 4 && C > 0 && recv.numel() % H == 0, "bad exchange row geometry");
    const int G = (int)(recv.numel() / H);
    check(G >= 1 && G <= 64, "1..64 peers");
    check(vals.dim() == 2, "vals must be [capacity, k]");
    const int64_t k = vals.size(1);
    check(slot.numel() >= G * C && rec.numel() >= G * C * k, "slot / rec < G*C(*k)");
    psamd::kvv_serve(ptr<int32_t>(recv), G, H, C, ptr<int64_t>(slot), ptr<float>(vals),
                     vals.size(0), (int)k, k, ptr<float>(rec), cur_stream());
  });
  // scalar tables (optimizer rules): serve the w field of the 32-B KV slots
  m.def("kv_serve_w", [](Tensor recv, int64_t H, int64_t C, Tensor slot, Tensor slots, Tensor rec) {
    chk(recv, at::kInt, "recv");
    chk(slot, at::kLong, "slot");
    chk(rec, at::kFloat, "rec");
    const int64_t cap = slot_capacity(slots);
    check(H >= 4 && C > 0 && recv.numel() % H == 0, "bad exchange row geometry");
    const int G = (int)(recv.numel() / H);
    check(G >= 1 && G <= 64, "1..64 peers");
    check(slot.numel() >= G * C && rec.numel() >= G * C, "slot / rec < G*C");
    const float* w = reinterpret_cast<const float*>(static_cast<const char*>(slots.data_ptr()) + 8);
    psamd::kvv_serve(ptr<int32_t>(recv), G, H, C, ptr<int64_t>(slot), w, cap, 1, 8,
                     ptr<float>(rec), cur_stream());
  });
  m.def("kvv_apply", [](Tensor recv, int64_t H, int64_t C, int kw, Tensor slot, Tensor vals,
                        int op) {
    chk(recv, at::kInt, "recv");
    chk(slot, at::kLong, "slot");
    chk(vals, at::kFloat, "vals");
    check(op == 0 || op == 1, "op: 0 = add, 1 = assign");
    check(vals.dim() == 2, "vals must be [capacity, k]");
    const int64_t k = vals.size(1);
    check(kw >= 0 && kw <= 2, "kw must be 0 (key-less row), 1 or 2");
    check(C > 0 && H >= 4 + C * kw + C * k && recv.numel() % H == 0, "bad push row geometry");
    const int G = (int)(recv.numel() / H);
    check(G >= 1 && G <= 64, "1..64 peers");
    check(slot.numel() >= G * C, "slot < G*C");
    psamd::kvv_apply(ptr<int32_t>(recv), G, H, C, kw, ptr<int64_t>(slot), ptr<float>(vals),
                     vals.size(0), (int)k, op, cur_stream());
  });
  m.def("kvv_unpack", [](Tensor rec, int64_t C, int64_t k, Tensor off, Tensor local_col,
                         Tensor out) {
    chk(rec, at::kFloat, "rec");
    chk(off, at::kLong, "off");
    chk(local_col, at::kInt, "local_col");
    chk(out, at::kFloat, "out");
    const int G = (int)off.numel() - 1;
    check(G >= 1 && G <= 64, "1..64 peers");
    check(k >= 1 && C > 0 && rec.numel() >= G * C * k, "rec < G*C*k");
    const int64_t nnz = local_col.numel();
    check(out.numel() >= nnz * k, "out < nnz*k");
    psamd::kvv_unpack(ptr<float>(rec), C, (int)k, ptr<int64_t>(off), G, ptr<int32_t>(local_col),
                      nnz, ptr<float>(out), cur_stream());
  });
  m.def("kvv_single_off", [](Tensor n_uniq, Tensor off) {
    chk(n_uniq, at::kInt, "n_uniq");
    chk(off, at::kLong, "off");
    check(off.numel() == 2, "off must be [2]");
    psamd::kvv_single_off(ptr<int32_t>(n_uniq), ptr<int64_t>(off), cur_stream());
  });
  // device-visible pointer of a pinned int32 host flag (nullptr when absent)
  auto host_flag = [](const optional<Tensor>& src, const optional<Tensor>& host_dst) -> int32_t* {
    if (!host_dst.has_value() || !host_dst->defined()) return nullptr;
    check(src.has_value() && src->defined(), "ovf_host needs ovf");
    check(host_dst->device().is_cpu() && host_dst->is_pinned() &&
              host_dst->scalar_type() == at::kInt && host_dst->numel() >= 1,
          "ovf_host must be a pinned int32 host tensor");
    void* dptr = nullptr;
    PSAMD_HIP_CHECK(hipHostGetDevicePointer(&dptr, host_dst->data_ptr(), 0));
    return reinterpret_cast<int32_t*>(dptr);
  };
  m.def("xchg_publish", [](Tensor src, Tensor host_dst) {
    chk(src, at::kInt, "src");
    check(host_dst.device().is_cpu() && host_dst.is_pinned() && host_dst.scalar_type() == at::kInt &&
              host_dst.numel() >= 1,
          "host_dst must be a pinned int32 host tensor");
    void* dptr = nullptr;
    PSAMD_HIP_CHECK(hipHostGetDevicePointer(&dptr, host_dst.data_ptr(), 0));
    psamd::xchg_publish(ptr<int32_t>(src), reinterpret_cast<int32_t*>(dptr), cur_stream());
  });
  m.def("xchg_pack_keys", [](Tensor ukeys, Tensor n_uniq, Tensor off, int64_t C, int kw,
                             int64_t H, Tensor send, optional<Tensor> ovf,
                             optional<Tensor> homes, int64_t b0, int lgP) {
    chk(ukeys, at::kLong, "ukeys");
    chk(n_uniq, at::kInt, "n_uniq");
    chk(off, at::kLong, "off");
    chk(send, at::kInt, "send");
    const int G = (int)off.numel() - 1;
    check(G >= 1 && G <= 64, "1..64 peers");
    check(kw == 1 || kw == 2, "kw must be 1 or 2");
    check(C > 0 && H >= 4 + C * kw + 1 && H % 4 == 0, "bad exchange row geometry");
    check(send.numel() == G * H, "send must be [G * H]");
    const uint64_t* hp = check_homes(homes, G, H, b0, lgP, 4 + C * kw);
    psamd::xchg_pack_keys(ptr<uint64_t>(ukeys), ptr<int32_t>(n_uniq), ukeys.numel(),
                          ptr<int64_t>(off), G, C, kw, H, ptr<int32_t>(send),
                          optr<int32_t>(ovf, at::kInt, "ovf"), hp, b0, lgP, cur_stream());
  }, py::arg("ukeys"), py::arg("n_uniq"), py::arg("off"), py::arg("C"), py::arg("kw"),
     py::arg("H"), py::arg("send"), py::arg("ovf"), py::arg("homes") = py::none(),
     py::arg("b0") = 0, py::arg("lgP") = 0);
  // The owner's half of a merged exchange in one launch (kv_table.hip kv_owner_part_kernel):
  // resolve of the pulled keys (bounds from the rows, weights into the next send rows at
  // word w0, stride H) and the per-source push apply of an earlier pull, per partition.
  m.def("kv_owner_part", [](Tensor slots, Tensor recv, int64_t H, int64_t C, int kw, int64_t b0,
                            int lgP, Tensor slot_out, Tensor key_out, Tensor bnd_out, Tensor wout,
                            int init_type, double init_v, double init_s, uint64_t seed,
                            optional<Tensor> err, optional<Tensor> inserted, uint64_t home_base,
                            uint64_t home_m, optional<Tensor> slot_idx, optional<Tensor> keys,
                            optional<Tensor> grad, int64_t gstride, optional<Tensor> bnd_in,
                            bool post, int algo, int lr_type, double alpha, double beta,
                            double l1, double l2, double grad_scale, double max_delta,
                            optional<Tensor> stats) {
    const int64_t cap = slot_capacity(slots);
    chk(recv, at::kInt, "recv");
    chk(slot_out, at::kLong, "slot_out");
    chk(key_out, at::kLong, "key_out");
    chk(bnd_out, at::kInt, "bnd_out");
    chk(wout, at::kFloat, "wout");
    check(kw == 1 || kw == 2, "kw must be 1 or 2");
    check(recv.numel() % H == 0, "recv is not a whole number of rows");
    const int G = (int)(recv.numel() / H);
    const int P = 1 << lgP;
    check(G >= 1 && G <= 64 && lgP >= 0 && lgP <= 20, "1..64 rows, lgP 0..20");
    check(C > 0 && b0 >= 4 + C * kw && b0 + P + 1 <= H, "kv_owner_part: row geometry");
    check(slot_out.numel() >= G * C && key_out.numel() >= G * C &&
          bnd_out.numel() >= G * (P + 1) && wout.numel() >= (G - 1) * H + C,
          "kv_owner_part: output sizes");
    const bool apply = slot_idx.has_value();
    if (apply) {
      chk(*slot_idx, at::kLong, "slot_idx");
      chk(*keys, at::kLong, "keys");
      chk(*grad, at::kFloat, "grad");
      chk(*bnd_in, at::kInt, "bnd_in");
      check(slot_idx->numel() >= G * C && keys->numel() >= G * C &&
            bnd_in->numel() >= G * (P + 1) && grad->numel() >= (G - 1) * gstride + C,
            "kv_owner_part: apply inputs");
      check(alpha > 0, "learning rate alpha must be > 0");
    }
    double* sp = optr<double>(stats, at::kDouble, "stats");
    psamd::kv_owner_part(
        slots.data_ptr(), cap, home_base, home_m, ptr<int32_t>(recv), G, H, C, kw, b0, lgP,
        ptr<int64_t>(slot_out), reinterpret_cast<uint64_t*>(key_out.data_ptr<int64_t>()),
        ptr<int32_t>(bnd_out), ptr<float>(wout), init_type, (float)init_v, (float)init_s, seed,
        optr<int32_t>(err, at::kInt, "err"), optr<int32_t>(inserted, at::kInt, "inserted"),
        apply ? ptr<int64_t>(*slot_idx) : nullptr,
        apply ? reinterpret_cast<const uint64_t*>(keys->data_ptr<int64_t>()) : nullptr,
        apply ? ptr<float>(*grad) : nullptr, gstride, apply ? ptr<int32_t>(*bnd_in) : nullptr,
        apply, post, algo, lr_type, (float)alpha, (float)beta, (float)l1, (float)l2,
        (float)grad_scale, (float)max_delta, sp, acc_stripes_of(stats), cur_stream());
  });
  m.def("xchg_pack_grads", [host_flag](Tensor grad, optional<Tensor> perm, Tensor n_uniq, Tensor off,
                              int64_t C, int kw, int64_t H, Tensor send, optional<Tensor> hist,
                              optional<Tensor> metrics, optional<Tensor> step_counter,
                              optional<Tensor> ovf, optional<Tensor> ovf_host) {
    chk(grad, at::kFloat, "grad");
    chk(n_uniq, at::kInt, "n_uniq");
    chk(off, at::kLong, "off");
    chk(send, at::kInt, "send");
    const int G = (int)off.numel() - 1;
    check(G >= 1 && G <= 64, "1..64 peers");
    check(C > 0 && H >= 4 + C * (kw + 1) && H % 4 == 0, "bad exchange row geometry");
    check(send.numel() == G * H, "send must be [G * H]");
    const int32_t* pp = optr<int32_t>(perm, at::kInt, "perm");
    if (pp) check(perm->numel() >= grad.numel(), "perm shorter than grad");
    // optional: the step's AUC histogram (stripes x 2 x 2048) -> metrics in block 0
    uint32_t* hp = optr<uint32_t>(hist, at::kInt, "hist");
    double* mp = optr<double>(metrics, at::kDouble, "metrics");
    if (hp) check(mp && hist->numel() % 4096 == 0 && hist->numel() / 4096 <= 8,
                  "xchg_pack_grads: hist = stripes x 2 x 2048 (<= 8 stripes) with metrics");
    psamd::xchg_pack_grads(ptr<float>(grad), pp, ptr<int32_t>(n_uniq), grad.numel(),
                           ptr<int64_t>(off), G, C, kw, H, ptr<int32_t>(send), hp,
                           hp ? (int)(hist->numel() / 4096) : 1, mp,
                           optr<int64_t>(step_counter, at::kLong, "step_counter"),
                           optr<int32_t>(ovf, at::kInt, "ovf"), host_flag(ovf, ovf_host),
                           cur_stream());
  }, py::arg("grad"), py::arg("perm"), py::arg("n_uniq"), py::arg("off"), py::arg("C"),
     py::arg("kw"), py::arg("H"), py::arg("send"), py::arg("hist") = py::none(),
     py::arg("metrics") = py::none(), py::arg("step_counter") = py::none(),
     py::arg("ovf") = py::none(), py::arg("ovf_host") = py::none());
  m.def("xchg_ff_pack_grads", [](Tensor grad, optional<Tensor> perm, Tensor n_uniq, Tensor off,
                                 int64_t C, int kw, int64_t H, int nb, uint64_t seed,
                                 optional<Tensor> step, Tensor send, Tensor gstage) {
    chk(grad, at::kFloat, "grad");
    chk(n_uniq, at::kInt, "n_uniq");
    chk(off, at::kLong, "off");
    chk(send, at::kInt, "send");
    chk(gstage, at::kFloat, "gstage");
    const int G = (int)off.numel() - 1;
    check(G >= 1 && G <= 64, "1..64 peers");
    check(kw == 1 || kw == 2, "kw must be 1 or 2");
    check(nb >= 1 && nb <= 7, "FixingFloat bytes in [1, 7]");
    check(C > 0 && H >= 4 + C * kw + (C * nb + 3) / 4 && H % 4 == 0, "bad exchange row geometry");
    check(send.numel() == G * H, "send must be [G * H]");
    check(gstage.numel() >= G * C, "gstage < G*C");
    const int32_t* pp = optr<int32_t>(perm, at::kInt, "perm");
    if (pp) check(perm->numel() >= grad.numel(), "perm shorter than grad");
    psamd::xchg_ff_pack_grads(ptr<float>(grad), pp, ptr<int32_t>(n_uniq), grad.numel(),
                              ptr<int64_t>(off), G, C, kw, H, nb, seed,
                              optr<int64_t>(step, at::kLong, "step"), ptr<int32_t>(send),
                              ptr<float>(gstage), cur_stream());
  });
  m.def("xchg_ff_init", [](Tensor send, int64_t H) {
    chk(send, at::kInt, "send");
    check(H > 4 && send.numel() % H == 0, "send is not a whole number of rows");
    const int G = (int)(send.numel() / H);
    check(G >= 1 && G <= 64, "1..64 peers");
    psamd::xchg_ff_init(ptr<int32_t>(send), G, H, cur_stream());
  });
  m.def("xchg_ff_encode", [](Tensor gstage, int64_t C, int kw, int64_t H, int nb, uint64_t seed,
                             optional<Tensor> step, Tensor send, int per) {
    chk(gstage, at::kFloat, "gstage");
    chk(send, at::kInt, "send");
    check(kw == 1 || kw == 2, "kw must be 1 or 2");
    check(nb >= 1 && nb <= 7, "FixingFloat bytes in [1, 7]");
    check(C > 0 && H >= 4 + C * kw + (C * nb + 3) / 4 && send.numel() % H == 0,
          "bad exchange row geometry");
    const int G = (int)(send.numel() / H);
    check(G >= 1 && G <= 64 && gstage.numel() >= G * C, "gstage < G*C");
    check(per >= 0 && gstage.numel() >= G * C + 2 * (int64_t)G * per,
          "xchg_ff_encode: gstage < G*C + the producers' partials");
    psamd::xchg_ff_encode(ptr<float>(gstage), G, C, kw, H, nb, seed,
                          optr<int64_t>(step, at::kLong, "step"), ptr<int32_t>(send), per,
                          cur_stream());
  }, py::arg("gstage"), py::arg("C"), py::arg("kw"), py::arg("H"), py::arg("nb"), py::arg("seed"),
     py::arg("step"), py::arg("send"), py::arg("per") = 0);
  m.def("xchg_ff_decode", [](Tensor recv, int64_t C, int kw, int64_t H, int nb, Tensor gin) {
    chk(recv, at::kInt, "recv");
    chk(gin, at::kFloat, "gin");
    check(kw == 1 || kw == 2, "kw must be 1 or 2");
    check(nb >= 1 && nb <= 7, "FixingFloat bytes in [1, 7]");
    check(C > 0 && H >= 4 + C * kw + (C * nb + 3) / 4 && H % 4 == 0, "bad exchange row geometry");
    check(recv.numel() % H == 0, "recv is not a whole number of rows");
    const int G = (int)(recv.numel() / H);
    check(G >= 1 && G <= 64, "1..64 peers");
    check(gin.numel() >= G * C, "gin < G*C");
    psamd::xchg_ff_decode(ptr<int32_t>(recv), G, C, kw, H, nb, ptr<float>(gin), cur_stream());
  });
  m.def("xchg_clear_counts", [](Tensor send, int64_t H, bool keys, bool grads) {
    chk(send, at::kInt, "send");
    check(H > 4 && send.numel() % H == 0, "send is not a whole number of rows");
    const int G = (int)(send.numel() / H);
    check(G >= 1 && G <= 64, "1..64 peers");
    psamd::xchg_clear_counts(ptr<int32_t>(send), G, H, keys, grads, cur_stream());
  });
  m.def("xchg_unpack_w", [](Tensor recv_w, optional<Tensor> perm, Tensor n_uniq, Tensor off,
                            int64_t C, Tensor w_local, int64_t wstride) {
    const int64_t ws = wstride > 0 ? wstride : C;
    chk(recv_w, at::kFloat, "recv_w");
    chk(n_uniq, at::kInt, "n_uniq");
    chk(off, at::kLong, "off");
    chk(w_local, at::kFloat, "w_local");
    const int G = (int)off.numel() - 1;
    check(G >= 1 && G <= 64, "1..64 peers");
    check(ws >= C && recv_w.numel() >= (G - 1) * ws + C, "recv_w < (G-1)*wstride + C");
    const int32_t* pp = optr<int32_t>(perm, at::kInt, "perm");
    if (pp) check(perm->numel() >= w_local.numel(), "perm shorter than w_local");
    psamd::xchg_unpack_w(ptr<float>(recv_w), pp, ptr<int32_t>(n_uniq), w_local.numel(),
                         ptr<int64_t>(off), G, C, ws, ptr<float>(w_local), cur_stream());
  }, py::arg("recv_w"), py::arg("perm"), py::arg("n_uniq"), py::arg("off"), py::arg("C"),
     py::arg("w_local"), py::arg("wstride") = 0);
  m.def("kv_gather", [](Tensor slots, Tensor slot_idx, optional<Tensor> n_dev, Tensor out,
                        int field) {
    const int64_t cap = slot_capacity(slots);
    chk(slot_idx, at::kLong, "slot_idx");
    chk(out, at::kFloat, "out");
    check(field >= 0 && field < 4, "field in [0,4): w,z,n,acc");
    check(out.numel() >= slot_idx.numel(), "out too small");
    psamd::kv_gather(slots.data_ptr(), cap, ptr<int64_t>(slot_idx), slot_idx.numel(),
                     optr<int32_t>(n_dev, at::kInt, "n_dev"), ptr<float>(out), field,
                     cur_stream());
  });
  m.def("kv_set", [](Tensor slots, Tensor slot_idx, optional<Tensor> w, optional<Tensor> z,
                     optional<Tensor> nn) {
    const int64_t cap = slot_capacity(slots);
    chk(slot_idx, at::kLong, "slot_idx");
    const int64_t n = slot_idx.numel();
    for (auto* t : {&w, &z, &nn})
      if (t->has_value()) check((*t)->numel() >= n, "value array too small");
    psamd::kv_set(slots.data_ptr(), cap, ptr<int64_t>(slot_idx), n, optr<float>(w, at::kFloat, "w"),
                  optr<float>(z, at::kFloat, "z"), optr<float>(nn, at::kFloat, "n"),
                  cur_stream());
  });
  m.def("kv_update", [](Tensor slots, Tensor slot_idx, Tensor grad, optional<Tensor> n_dev,
                        int algo, int lr_type, double alpha, double beta, double l1, double l2,
                        double grad_scale, double max_delta, optional<Tensor> stats,
                        optional<Tensor> hist, optional<Tensor> metrics,
                        optional<Tensor> step_counter) {
    const int64_t cap = slot_capacity(slots);
    chk(slot_idx, at::kLong, "slot_idx");
    chk(grad, at::kFloat, "grad");
    check(grad.numel() >= slot_idx.numel(), "grad too small");
    check(alpha > 0, "learning rate alpha must be > 0");
    // optional: the step's AUC histogram -> metrics (auc_from_hist folded into block 0)
    uint32_t* hp = optr<uint32_t>(hist, at::kInt, "hist");
    double* mp = optr<double>(metrics, at::kDouble, "metrics");
    constexpr int kBins = 2048;
    if (hp) check(mp && hist->numel() % (2 * kBins) == 0 && hist->numel() / (2 * kBins) <= 8,
                  "kv_update: hist = stripes x 2 x 2048 (<= 8 stripes) with metrics");
    psamd::kv_update(slots.data_ptr(), cap, ptr<int64_t>(slot_idx), ptr<float>(grad),
                     slot_idx.numel(), optr<int32_t>(n_dev, at::kInt, "n_dev"), algo, lr_type,
                     (float)alpha, (float)beta, (float)l1, (float)l2, (float)grad_scale,
                     (float)max_delta, optr<double>(stats, at::kDouble, "stats"),
                     acc_stripes_of(stats), hp, kBins,
                     hp ? (int)(hist->numel() / (2 * kBins)) : 1, mp,
                     optr<int64_t>(step_counter, at::kLong, "step_counter"), cur_stream());
  }, py::arg("slots"), py::arg("slot_idx"), py::arg("grad"), py::arg("n_dev"), py::arg("algo"),
     py::arg("lr_type"), py::arg("alpha"), py::arg("beta"), py::arg("l1"), py::arg("l2"),
     py::arg("grad_scale"), py::arg("max_delta"), py::arg("stats"), py::arg("hist") = py::none(),
     py::arg("metrics") = py::none(), py::arg("step_counter") = py::none());
  m.def("kv_accumulate", [](Tensor slots, Tensor slot_idx, Tensor grad, optional<Tensor> n_dev,
                            Tensor touched, Tensor n_touched) {
    const int64_t cap = slot_capacity(slots);
    chk(slot_idx, at::kLong, "slot_idx");
    chk(grad, at::kFloat, "grad");
    chk(touched, at::kLong, "touched");
    chk(n_touched, at::kInt, "n_touched");
    check(touched.numel() >= slot_idx.numel(), "touched buffer too small");
    psamd::kv_accumulate(slots.data_ptr(), cap, ptr<int64_t>(slot_idx), ptr<float>(grad),
                         slot_idx.numel(), optr<int32_t>(n_dev, at::kInt, "n_dev"),
                         ptr<int64_t>(touched), ptr<int32_t>(n_touched), touched.numel(),
                         cur_stream());
  });
  m.def("kv_apply_accumulated", [](Tensor slots, Tensor touched, Tensor n_touched, int algo,
                                   int lr_type, double alpha, double beta, double l1, double l2,
                                   double grad_scale, double max_delta, optional<Tensor> stats) {
    const int64_t cap = slot_capacity(slots);
    chk(touched, at::kLong, "touched");
    chk(n_touched, at::kInt, "n_touched");
    psamd::kv_apply_accumulated(slots.data_ptr(), cap, ptr<int64_t>(touched), ptr<int32_t>(n_touched),
                                touched.numel(), algo, lr_type, (float)alpha, (float)beta,
                                (float)l1, (float)l2, (float)grad_scale, (float)max_delta,
                                optr<double>(stats, at::kDouble, "stats"), acc_stripes_of(stats),
                                cur_stream());
  });
  m.def("kv_census", [](Tensor slots) {
    const int64_t cap = slot_capacity(slots);
    auto out = torch::zeros({2}, slots.options().dtype(at::kLong));
    psamd::kv_census(slots.data_ptr(), cap, ptr<unsigned long long>(out), cur_stream());
    return out;
  });

  // ---------------- localisation ----------------
  m.def("mix_iota", [](Tensor keys, int bits, Tensor h, Tensor pos) {
    chk(keys, at::kLong, "keys");
    chk(h, at::kLong, "h");
    chk(pos, at::kInt, "pos");
    const int64_t n = keys.numel();
    check(h.numel() >= n && pos.numel() >= n, "outputs too small");
    psamd::mix_iota(ptr<uint64_t>(keys), n, make_keymix(bits), ptr<uint64_t>(h), ptr<int32_t>(pos),
                    cur_stream());
  });
  m.def("mix_keys", [](Tensor keys, int bits, Tensor out, bool inverse) {
    chk(keys, at::kLong, "keys");
    chk(out, at::kLong, "out");
    check(out.numel() >= keys.numel(), "out too small");
    psamd::mix_keys(ptr<uint64_t>(keys), keys.numel(), make_keymix(bits), ptr<uint64_t>(out),
                    inverse, cur_stream());
  });
  m.def("sort_pairs_temp_bytes", [](int64_t n, int end_bit, bool rocprim) {
    return (int64_t)(rocprim ? psamd::rocprim_sort_temp_bytes(n, end_bit)
                             : psamd::radix_sort_temp_bytes(n));
  }, py::arg("n"), py::arg("end_bit"), py::arg("rocprim") = false);
  m.def("sort_pairs", [](Tensor temp, Tensor k_in, Tensor k_out, Tensor v_in, Tensor v_out,
                         int64_t n, int end_bit, bool rocprim) {
    chk(temp, at::kByte, "temp");
    chk(k_in, at::kLong, "k_in");
    chk(k_out, at::kLong, "k_out");
    chk(v_in, at::kInt, "v_in");
    chk(v_out, at::kInt, "v_out");
    check(n >= 0 && k_in.numel() >= n && k_out.numel() >= n && v_in.numel() >= n &&
              v_out.numel() >= n, "sort buffers too small");
    check(n < (int64_t)INT32_MAX, "sort size must fit int32");
    check(end_bit >= 1 && end_bit <= 64, "end_bit in [1,64]");
    check(k_in.data_ptr() != k_out.data_ptr() && v_in.data_ptr() != v_out.data_ptr(),
          "sort input and output must not alias");
    const size_t need = rocprim ? psamd::rocprim_sort_temp_bytes(n, end_bit)
                                : psamd::radix_sort_temp_bytes(n);
    check((size_t)temp.numel() >= need, "sort temp storage too small");
    if (rocprim)
      psamd::rocprim_sort_pairs(temp.data_ptr(), (size_t)temp.numel(), ptr<uint64_t>(k_in),
                                ptr<uint64_t>(k_out), ptr<int32_t>(v_in), ptr<int32_t>(v_out), n,
                                end_bit, cur_stream());
    else
      psamd::radix_sort_pairs(temp.data_ptr(), (size_t)temp.numel(), ptr<uint64_t>(k_in),
                              ptr<uint64_t>(k_out), ptr<int32_t>(v_in), ptr<int32_t>(v_out), n,
                              end_bit, cur_stream());
  }, py::arg("temp"), py::arg("k_in"), py::arg("k_out"), py::arg("v_in"), py::arg("v_out"),
     py::arg("n"), py::arg("end_bit"), py::arg("rocprim") = false);
  m.def("scan_temp_bytes", [](int64_t n) { return (int64_t)psamd::scan_temp_bytes(n); });
  m.def("inclusive_scan_i32", [](Tensor temp, Tensor in, Tensor out, int64_t n) {
    chk(temp, at::kByte, "temp");
    chk(in, at::kInt, "in");
    chk(out, at::kInt, "out");
    check(in.numel() >= n && out.numel() >= n, "scan buffers too small");
    check((size_t)temp.numel() >= psamd::scan_temp_bytes(n), "scan temp too small");
    psamd::inclusive_scan_i32(temp.data_ptr(), (size_t)temp.numel(), ptr<int32_t>(in),
                              ptr<int32_t>(out), n, cur_stream());
  });
  m.def("rle", [](Tensor hs, Tensor pos_s, int64_t n, Tensor flags, Tensor segid, Tensor scan_temp,
                  Tensor uniq, Tensor seg_start, Tensor local_col, Tensor n_uniq,
                  optional<Tensor> zero_a, optional<Tensor> zero_b) {
    chk(hs, at::kLong, "hs");
    chk(pos_s, at::kInt, "pos_s");
    chk(flags, at::kInt, "flags");
    chk(segid, at::kInt, "segid");
    chk(scan_temp, at::kByte, "scan_temp");
    chk(uniq, at::kLong, "uniq");
    chk(seg_start, at::kInt, "seg_start");
    chk(local_col, at::kInt, "local_col");
    chk(n_uniq, at::kInt, "n_uniq");
    check(n >= 1, "rle needs n >= 1");
    check(hs.numel() >= n && pos_s.numel() >= n && flags.numel() >= n && segid.numel() >= n &&
              uniq.numel() >= n && seg_start.numel() >= n + 1 && local_col.numel() >= n,
          "rle buffers too small");
    float* za = optr<float>(zero_a, at::kFloat, "zero_a");
    float* zb = optr<float>(zero_b, at::kFloat, "zero_b");
    if (za) check(zero_a->numel() >= n, "zero_a too small");
    if (zb) check(zero_b->numel() >= n, "zero_b too small");
    check((size_t)scan_temp.numel() >= psamd::scan_temp_bytes(n), "scan temp too small");
    psamd::rle(ptr<uint64_t>(hs), ptr<int32_t>(pos_s), n, ptr<int32_t>(flags), ptr<int32_t>(segid),
               scan_temp.data_ptr(), (size_t)scan_temp.numel(), ptr<uint64_t>(uniq),
               ptr<int32_t>(seg_start), ptr<int32_t>(local_col), ptr<int32_t>(n_uniq), za, zb,
               cur_stream());
  });
  m.def("localize32_temp_bytes", [](int64_t n) { return (int64_t)psamd::localize32_temp_bytes(n); });
  m.def("sort40_temp_bytes", [](int64_t n) { return (int64_t)psamd::sort40_temp_bytes(n); });
  m.def("sort40", [](Tensor keys, int bits, Tensor temp, Tensor hs, Tensor pos_s) {
    chk(keys, at::kLong, "keys");
    chk(temp, at::kByte, "temp");
    chk(hs, at::kLong, "hs");
    chk(pos_s, at::kInt, "pos_s");
    const int64_t n = keys.numel();
    check(n >= 1 && n < (int64_t(1) << 22), "sort40: 1 <= n < 2^22");
    check(bits > 30 && bits <= 40, "sort40 needs 30 < key bits <= 40");
    check(hs.numel() >= n && pos_s.numel() >= n, "sort40 buffers too small");
    check((size_t)temp.numel() >= psamd::sort40_temp_bytes(n), "sort40 temp too small");
    psamd::sort40(ptr<uint64_t>(keys), n, make_keymix(bits), temp.data_ptr(),
                  (size_t)temp.numel(), ptr<uint64_t>(hs), ptr<int32_t>(pos_s), cur_stream());
  });
  m.def("localize32", [](Tensor keys, int bits, Tensor temp, Tensor hs, Tensor pos_s, Tensor segid,
                         Tensor uniq, Tensor seg_start, Tensor local_col, Tensor n_uniq,
                         optional<Tensor> zero_a, optional<Tensor> zero_b, int digit_bits) {
    check(digit_bits == 8 || digit_bits == 10, "localize32 digit_bits: 8 or 10");
    chk(keys, at::kLong, "keys");
    chk(temp, at::kByte, "temp");
    chk(hs, at::kInt, "hs");
    chk(pos_s, at::kInt, "pos_s");
    chk(segid, at::kInt, "segid");
    chk(uniq, at::kLong, "uniq");
    chk(seg_start, at::kInt, "seg_start");
    chk(local_col, at::kInt, "local_col");
    chk(n_uniq, at::kInt, "n_uniq");
    const int64_t n = keys.numel();
    check(n >= 1 && n < (int64_t)INT32_MAX, "localize32: 1 <= n < 2^31");
    check(bits >= 2 && bits <= 32, "localize32 needs key bits <= 32");
    check(hs.numel() >= n && pos_s.numel() >= n && segid.numel() >= n && uniq.numel() >= n &&
              seg_start.numel() >= n + 1 && local_col.numel() >= n, "localize32 buffers too small");
    check((size_t)temp.numel() >= psamd::localize32_temp_bytes(n), "localize32 temp too small");
    float* za = optr<float>(zero_a, at::kFloat, "zero_a");
    float* zb = optr<float>(zero_b, at::kFloat, "zero_b");
    if (za) check(zero_a->numel() >= n, "zero_a too small");
    if (zb) check(zero_b->numel() >= n, "zero_b too small");
    psamd::localize32(ptr<uint64_t>(keys), n, make_keymix(bits), temp.data_ptr(),
                      (size_t)temp.numel(), ptr<uint32_t>(hs), ptr<int32_t>(pos_s),
                      ptr<int32_t>(segid), ptr<uint64_t>(uniq), ptr<int32_t>(seg_start),
                      ptr<int32_t>(local_col), ptr<int32_t>(n_uniq), za, zb, digit_bits,
                      cur_stream());
  }, py::arg("keys"), py::arg("bits"), py::arg("temp"), py::arg("hs"), py::arg("pos_s"),
     py::arg("segid"), py::arg("uniq"), py::arg("seg_start"), py::arg("local_col"),
     py::arg("n_uniq"), py::arg("zero_a"), py::arg("zero_b"), py::arg("digit_bits") = 8);
  m.def("partloc_temp_bytes", [](int64_t n, int bits) {
    return (int64_t)psamd::partloc_temp_bytes(n, bits);
  });
  m.def("partloc_supported", [](int64_t n, int bits) { return psamd::partloc_supported(n, bits); });
  m.def("localize_part", [](Tensor keys, int bits, Tensor temp, Tensor pos_s, Tensor segid,
                            Tensor uniq, Tensor seg_start, Tensor local_col, Tensor n_uniq,
                            optional<Tensor> zero_a, optional<Tensor> zero_b, Tensor err) {
    chk(keys, at::kLong, "keys");
    chk(temp, at::kByte, "temp");
    chk(pos_s, at::kInt, "pos_s");
    chk(segid, at::kInt, "segid");
    chk(uniq, at::kLong, "uniq");
    chk(seg_start, at::kInt, "seg_start");
    chk(local_col, at::kInt, "local_col");
    chk(n_uniq, at::kInt, "n_uniq");
    chk(err, at::kInt, "err");
    const int64_t n = keys.numel();
    check(psamd::partloc_supported(n, bits), "localize_part: needs bits <= 32 and n <= 10M");
    check(pos_s.numel() >= n && segid.numel() >= n && uniq.numel() >= n &&
              seg_start.numel() >= n + 1 && local_col.numel() >= n,
          "localize_part buffers too small");
    check((size_t)temp.numel() >= psamd::partloc_temp_bytes(n, bits), "localize_part temp too small");
    float* za = optr<float>(zero_a, at::kFloat, "zero_a");
    float* zb = optr<float>(zero_b, at::kFloat, "zero_b");
    if (za) check(zero_a->numel() >= n, "zero_a too small");
    if (zb) check(zero_b->numel() >= n, "zero_b too small");
    psamd::localize_part(ptr<uint64_t>(keys), n, make_keymix(bits), temp.data_ptr(),
                         (size_t)temp.numel(), ptr<int32_t>(pos_s), ptr<int32_t>(segid),
                         ptr<uint64_t>(uniq), ptr<int32_t>(seg_start), ptr<int32_t>(local_col),
                         ptr<int32_t>(n_uniq), za, zb, ptr<int32_t>(err), uniq.numel(),
                         cur_stream());
  });
  m.def("owner_split", [](Tensor uniq, optional<Tensor> n_uniq, Tensor bounds, Tensor offsets) {
    chk(uniq, at::kLong, "uniq");
    chk(bounds, at::kLong, "bounds");
    chk(offsets, at::kLong, "offsets");
    const int G = (int)bounds.numel() - 1;
    check(G >= 1 && offsets.numel() >= G + 1, "bounds/offsets size mismatch");
    psamd::owner_split(ptr<uint64_t>(uniq), optr<int32_t>(n_uniq, at::kInt, "n_uniq"),
                       uniq.numel(), ptr<uint64_t>(bounds), G, ptr<int64_t>(offsets),
                       cur_stream());
  });
  m.def("owner_of", [](Tensor h, Tensor bounds, Tensor owner) {
    chk(h, at::kLong, "h");
    chk(bounds, at::kLong, "bounds");
    chk(owner, at::kInt, "owner");
    const int G = (int)bounds.numel() - 1;
    check(G >= 1 && owner.numel() >= h.numel(), "owner_of sizes");
    psamd::owner_of(ptr<uint64_t>(h), h.numel(), ptr<uint64_t>(bounds), G, ptr<int32_t>(owner),
                    cur_stream());
  });

  // ---------------- linear model ----------------
  m.def("linear_fwd", [](optional<Tensor> row_ptr, int64_t B, int width, Tensor local_col,
                         optional<Tensor> vals, Tensor w_local, Tensor labels, int loss_type,
                         optional<Tensor> xw, Tensor coef, optional<Tensor> coef2,
                         optional<Tensor> metrics, optional<Tensor> hist, int nbins) {
    chk(local_col, at::kInt, "local_col");
    chk(w_local, at::kFloat, "w_local");
    chk(labels, at::kFloat, "labels");
    chk(coef, at::kFloat, "coef");
    check(labels.numel() >= B && coef.numel() >= B, "labels/coef too small");
    const int64_t* rp = optr<int64_t>(row_ptr, at::kLong, "row_ptr");
    if (rp) check(row_ptr->numel() >= B + 1, "row_ptr too small");
    else check(width > 0 && local_col.numel() >= B * width, "fixed width layout too small");
    const float* v = optr<float>(vals, at::kFloat, "vals");
    if (v) check(vals->numel() >= local_col.numel(), "vals too small");
    uint32_t* hp = optr<uint32_t>(hist, at::kInt, "hist");
    if (hp) check(nbins > 0 && nbins <= 8192 && hist->numel() >= 2 * nbins, "hist size");
    float* xp = optr<float>(xw, at::kFloat, "xw");
    if (xp) check(xw->numel() >= B, "xw too small");
    float* c2 = optr<float>(coef2, at::kFloat, "coef2");
    if (c2) check(coef2->numel() >= B, "coef2 too small");
    double* mp = optr<double>(metrics, at::kDouble, "metrics");
    if (mp) check(metrics->numel() >= 5, "metrics needs >= 5 slots");
    psamd::linear_fwd(rp, B, width, ptr<int32_t>(local_col), v, ptr<float>(w_local),
                      w_local.numel(), ptr<float>(labels), loss_type, xp, ptr<float>(coef), c2, mp, hp, nbins,
                      acc_stripes_of(metrics),
                      hp ? (int)std::max<int64_t>(1, hist->numel() / (2 * nbins)) : 1,
                      cur_stream());
  });
  m.def("linear_bwd", [](Tensor pos_s, Tensor segid, int64_t n, optional<Tensor> rows, int width,
                         optional<Tensor> vals, Tensor coef, optional<Tensor> coef2, Tensor grad,
                         optional<Tensor> hess) {
    chk(pos_s, at::kInt, "pos_s");
    chk(segid, at::kInt, "segid");
    chk(coef, at::kFloat, "coef");
    chk(grad, at::kFloat, "grad");
    check(pos_s.numel() >= n && segid.numel() >= n, "bwd inputs too small");
    const int32_t* r = optr<int32_t>(rows, at::kInt, "rows");
    if (r) check(rows->numel() >= n, "rows too small");
    else check(width > 0, "need rows or a fixed width");
    float* h = optr<float>(hess, at::kFloat, "hess");
    const float* c2 = optr<float>(coef2, at::kFloat, "coef2");
    check(!h || c2, "hess requires coef2");
    if (h) check(hess->numel() >= grad.numel(), "hess smaller than grad");
    psamd::linear_bwd(ptr<int32_t>(pos_s), ptr<int32_t>(segid), n, r, width,
                      optr<float>(vals, at::kFloat, "vals"), ptr<float>(coef), coef.numel(), c2,
                      ptr<float>(grad), h, grad.numel(), cur_stream());
  });
  m.def("auc_from_hist", [](Tensor hist, int nbins, Tensor metrics,
                            optional<Tensor> step_counter) {
    chk(hist, at::kInt, "hist");
    chk(metrics, at::kDouble, "metrics");
    check(hist.numel() >= 2 * nbins && metrics.numel() >= 5, "auc sizes");
    check(nbins == 2048, "auc_from_hist: 2048 bins (256 threads x 8)");
    const int stripes = (int)std::max<int64_t>(1, hist.numel() / (2 * nbins));
    check(stripes <= 8, "auc_from_hist: at most 8 histogram stripes");
    psamd::auc_from_hist(ptr<uint32_t>(hist), nbins, stripes, ptr<double>(metrics),
                         optr<int64_t>(step_counter, at::kLong, "step_counter"), cur_stream());
  }, py::arg("hist"), py::arg("nbins"), py::arg("metrics"),
     py::arg("step_counter") = py::none());
  m.def("csr_rows", [](Tensor row_ptr, Tensor rows) {
    chk(row_ptr, at::kLong, "row_ptr");
    chk(rows, at::kInt, "rows");
    psamd::csr_rows(ptr<int64_t>(row_ptr), row_ptr.numel() - 1, ptr<int32_t>(rows),
                    cur_stream());
  });
  m.def("criteo_set_tables", [](std::vector<uint32_t> cards, std::vector<float> gauss) {
    check(cards.size() == 26, "need 26 cardinalities");
    check(gauss.size() == 256, "need 256 Gaussian quantiles");
    psamd::criteo_set_tables(cards.data(), gauss.data());
  });
  m.def("add_i64", [](Tensor p, int64_t v) {
    chk(p, at::kLong, "p");
    psamd::add_i64(ptr<int64_t>(p), v, cur_stream());
  });
  m.def("criteo_gen", [](uint64_t seed, int64_t row0, int64_t B, uint64_t num_features,
                         double alpha, Tensor keys, Tensor labels, optional<Tensor> row0_dev,
                         int64_t row_scale, optional<Tensor> row0_out) {
    // row0_out: the kernel writes row0_dev + 1 there (the cursor of the next launch, which
    // reads row0_out and writes row0_dev: a captured graph pair alternating the two
    // words generates fresh rows on every replay, no separate add)
    int64_t* op = optr<int64_t>(row0_out, at::kLong, "row0_out");
    if (op) check(row0_dev.has_value() && row0_dev->defined() && row0_out->numel() >= 1 &&
                      row0_dev->numel() >= 1 && op != row0_dev->data_ptr<int64_t>(),
                  "row0_out: a word of its own next to row0_dev");
    chk(keys, at::kLong, "keys");
    chk(labels, at::kFloat, "labels");
    check(keys.numel() >= B * 39 && labels.numel() >= B, "criteo_gen buffers too small");
    check(alpha > 1.0, "power-law alpha must be > 1");
    check(num_features > 0, "num_features > 0");
    psamd::criteo_gen(seed, row0, optr<int64_t>(row0_dev, at::kLong, "row0_dev"), row_scale, B,
                      num_features, (float)alpha, ptr<uint64_t>(keys), ptr<float>(labels),
                      op, cur_stream());
  }, py::arg("seed"), py::arg("row0"), py::arg("B"), py::arg("num_features"), py::arg("alpha"),
     py::arg("keys"), py::arg("labels"), py::arg("row0_dev") = py::none(),
     py::arg("row_scale") = 1, py::arg("row0_out") = py::none());

  // ---------------- filters ----------------
  // CountMin over byte cells packed in int32 words: one region of all cells, or (rshift
  // < 64) regions of rsize cells selected by key >> rshift (countmin.cuh)
  auto cm_rsize = [](const Tensor& table, int64_t rsize, int rshift, int key_bits) {
    const uint64_t n = (uint64_t)table.numel() * 4;
    if (rshift >= 64) return rsize > 0 ? std::min<uint64_t>((uint64_t)rsize, n) : n;
    check(rsize > 0 && rsize % 64 == 0,
          "countmin: region size must be a positive multiple of 64 (one block)");
    check(rshift >= 0 && key_bits >= rshift && key_bits - rshift <= 30 &&
              ((uint64_t)rsize << (key_bits - rshift)) <= n,
          "countmin: regions exceed the cell table");
    return (uint64_t)rsize;
  };
  m.def("cm_insert", [cm_rsize](Tensor table, int k, int vmax, Tensor keys, optional<Tensor> counts,
                                optional<Tensor> n_dev, int64_t rsize, int rshift, int key_bits) {
    chk(table, at::kInt, "table");
    chk(keys, at::kLong, "keys");
    check(k >= 1 && k <= 30 && vmax >= 1 && vmax <= 255, "countmin k/vmax");
    const uint8_t* c = optr<uint8_t>(counts, at::kByte, "counts");
    if (c) check(counts->numel() >= keys.numel(), "counts too small");
    psamd::cm_insert(ptr<uint32_t>(table), cm_rsize(table, rsize, rshift, key_bits), rshift, k,
                     (uint32_t)vmax, ptr<uint64_t>(keys), c, keys.numel(),
                     optr<int32_t>(n_dev, at::kInt, "n_dev"), cur_stream());
  }, py::arg("table"), py::arg("k"), py::arg("vmax"), py::arg("keys"), py::arg("counts"),
     py::arg("n_dev"), py::arg("rsize") = 0, py::arg("rshift") = 64, py::arg("key_bits") = 64);
  m.def("cm_query", [cm_rsize](Tensor table, int k, int vmax, Tensor keys, optional<Tensor> n_dev,
                               int freq, optional<Tensor> keep, optional<Tensor> out_count,
                               int64_t rsize, int rshift, int key_bits) {
    chk(table, at::kInt, "table");
    chk(keys, at::kLong, "keys");
    int32_t* kp = optr<int32_t>(keep, at::kInt, "keep");
    uint8_t* cp = optr<uint8_t>(out_count, at::kByte, "out_count");
    if (kp) check(keep->numel() >= keys.numel(), "keep too small");
    if (cp) check(out_count->numel() >= keys.numel(), "out_count too small");
    psamd::cm_query(ptr<uint32_t>(table), cm_rsize(table, rsize, rshift, key_bits), rshift, k,
                    (uint32_t)vmax, ptr<uint64_t>(keys), keys.numel(),
                    optr<int32_t>(n_dev, at::kInt, "n_dev"), freq, kp, cp, cur_stream());
  }, py::arg("table"), py::arg("k"), py::arg("vmax"), py::arg("keys"), py::arg("n_dev"),
     py::arg("freq"), py::arg("keep"), py::arg("out_count"), py::arg("rsize") = 0,
     py::arg("rshift") = 64, py::arg("key_bits") = 64);
  m.def("compact_kept", [](Tensor keep, Tensor incl, optional<Tensor> n_dev, Tensor kept_idx,
                           Tensor n_kept, optional<Tensor> remap, optional<Tensor> keys_in,
                           optional<Tensor> keys_out) {
    chk(keep, at::kInt, "keep");
    chk(incl, at::kInt, "incl");
    chk(kept_idx, at::kInt, "kept_idx");
    chk(n_kept, at::kInt, "n_kept");
    check(kept_idx.numel() >= keep.numel() && incl.numel() >= keep.numel(), "compact sizes");
    const uint64_t* ki = optr<uint64_t>(keys_in, at::kLong, "keys_in");
    uint64_t* ko = optr<uint64_t>(keys_out, at::kLong, "keys_out");
    check((ki == nullptr) == (ko == nullptr), "keys_in and keys_out go together");
    if (ki) check(keys_in->numel() >= keep.numel() && keys_out->numel() >= keep.numel(),
                  "compact key buffers too small");
    psamd::compact_kept(ptr<int32_t>(keep), ptr<int32_t>(incl), keep.numel(),
                        optr<int32_t>(n_dev, at::kInt, "n_dev"), ptr<int32_t>(kept_idx),
                        ptr<int32_t>(n_kept), optr<int32_t>(remap, at::kInt, "remap"), ki, ko,
                        cur_stream());
  });
  m.def("cm_insert_seg", [cm_rsize](Tensor table, int k, int vmax, Tensor keys, Tensor seg_start,
                                    optional<Tensor> n_dev, int64_t rsize, int rshift,
                                    int key_bits) {
    chk(table, at::kInt, "table");
    chk(keys, at::kLong, "keys");
    chk(seg_start, at::kInt, "seg_start");
    check(k >= 1 && k <= 30 && vmax >= 1 && vmax <= 255, "countmin k/vmax");
    check(seg_start.numel() >= keys.numel() + 1 || n_dev.has_value(), "seg_start too small");
    const int64_t n = std::min<int64_t>(keys.numel(), seg_start.numel() - 1);
    psamd::cm_insert_seg(ptr<uint32_t>(table), cm_rsize(table, rsize, rshift, key_bits), rshift,
                         k, (uint32_t)vmax, ptr<uint64_t>(keys), ptr<int32_t>(seg_start), n,
                         optr<int32_t>(n_dev, at::kInt, "n_dev"), cur_stream());
  }, py::arg("table"), py::arg("k"), py::arg("vmax"), py::arg("keys"), py::arg("seg_start"),
     py::arg("n_dev"), py::arg("rsize") = 0, py::arg("rshift") = 64, py::arg("key_bits") = 64);
  m.def("ff_minmax", [](Tensor x, Tensor mm) {
    chk(x, at::kFloat, "x");
    chk(mm, at::kFloat, "mm");
    check(mm.numel() >= 2, "mm needs 2 floats");
    psamd::ff_minmax(ptr<float>(x), x.numel(), ptr<float>(mm), cur_stream());
  });
  m.def("ff_encode", [](Tensor x, Tensor mm, int nbytes, uint64_t seed, Tensor out) {
    chk(x, at::kFloat, "x");
    chk(mm, at::kFloat, "mm");
    chk(out, at::kByte, "out");
    check(nbytes >= 1 && nbytes <= 7, "nbytes in [1,7]");
    check(out.numel() >= x.numel() * nbytes, "out too small");
    psamd::ff_encode(ptr<float>(x), x.numel(), ptr<float>(mm), nbytes, seed, ptr<uint8_t>(out),
                     cur_stream());
  });
  m.def("ff_decode", [](Tensor code, Tensor mm, int nbytes, Tensor out) {
    chk(code, at::kByte, "code");
    chk(mm, at::kFloat, "mm");
    chk(out, at::kFloat, "out");
    check(nbytes >= 1 && nbytes <= 7, "nbytes in [1,7]");
    check(code.numel() >= out.numel() * nbytes, "code too small");
    psamd::ff_decode(ptr<uint8_t>(code), out.numel(), ptr<float>(mm), nbytes, ptr<float>(out),
                     cur_stream());
  });
  m.def("key_signature", [](Tensor keys, Tensor sig) {
    chk(keys, at::kLong, "keys");
    chk(sig, at::kLong, "sig");
    psamd::key_signature(ptr<uint64_t>(keys), keys.numel(), ptr<unsigned long long>(sig),
                         cur_stream());
  });

  // ---------------------------------------------------------------- Darlin BCD
  // CSC of one rank: col/row int32 per nnz (sorted by col), val f32 per nnz or None
  // (binary). Block = nnz range [p0, p1) holding global columns [c0, c0 + ncols).
  auto csc_check = [](const Tensor& col, const Tensor& row, const optional<Tensor>& val,
                      int64_t p0, int64_t p1) {
    chk(col, at::kInt, "col");
    chk(row, at::kInt, "row");
    check(col.numel() == row.numel(), "col/row size mismatch");
    check(0 <= p0 && p0 <= p1 && p1 <= col.numel(), "nnz range outside the matrix");
    if (val.has_value() && val->defined()) {
      chk(*val, at::kFloat, "val");
      check(val->numel() == col.numel(), "val size mismatch");
    }
  };
  m.def("bcd_grad_chunked", [](Tensor col, Tensor row, optional<Tensor> val, Tensor chunks,
                                int64_t c0, int64_t ncols, Tensor ym, Tensor y, Tensor delta,
                                Tensor active, Tensor G, Tensor U, bool zeroed,
                                optional<Tensor> rowq, bool rowq_ready,
                                optional<Tensor> urows) {
    // chunks: [n + 1] int64 entry offsets (bit 62 = hot chunk), built and range-checked
    // on the host once per block (models/darlin.py build_chunks)
    chk(col, at::kInt, "col");
    chk(row, at::kInt, "row");
    chk(chunks, at::kLong, "chunks");
    check(chunks.numel() >= 1, "chunks needs the end sentinel");
    chk(ym, at::kDouble, "ym");
    chk(y, at::kFloat, "y");
    chk(delta, at::kDouble, "delta");
    chk(active, at::kByte, "active");
    chk(G, at::kDouble, "G");
    chk(U, at::kDouble, "U");
    check(row.numel() == col.numel(), "col/row size mismatch");
    const float* vp = optr<float>(val, at::kFloat, "val");
    if (vp) check(val->numel() == col.numel(), "val size mismatch");
    check(y.numel() == ym.numel(), "y/ym size mismatch");
    check(delta.numel() == active.numel(), "delta/active size mismatch");
    check(c0 >= 0 && ncols >= 0 && c0 + ncols <= delta.numel(), "column block outside model");
    check(G.numel() >= ncols && U.numel() >= ncols, "G/U too small");
    double* rq = optr<double>(rowq, at::kDouble, "rowq");
    if (rq) check(rowq->numel() >= 2 * ym.numel(), "rowq: 2 doubles per example");
    // urows: the block's distinct examples (the rowq packing covers only them; entries
    // outside the list would read stale factors: built from the block's rows, darlin.py)
    const int32_t* ur = optr<int32_t>(urows, at::kInt, "urows");
    if (ur) check(rq != nullptr, "urows needs rowq");
    psamd::bcd_grad_chunked(ptr<int32_t>(col), ptr<int32_t>(row), vp, ptr<int64_t>(chunks),
                            chunks.numel() - 1, c0, ncols, ptr<double>(ym), ptr<float>(y),
                            ym.numel(), ptr<double>(delta), ptr<uint8_t>(active), rq,
                            ptr<double>(G), ptr<double>(U), zeroed, rq != nullptr && rowq_ready,
                            ur, ur ? urows->numel() : 0, cur_stream());
  }, py::arg("col"), py::arg("row"), py::arg("val"), py::arg("chunks"), py::arg("c0"),
     py::arg("ncols"), py::arg("ym"), py::arg("y"), py::arg("delta"), py::arg("active"),
     py::arg("G"), py::arg("U"), py::arg("zeroed"), py::arg("rowq"), py::arg("rowq_ready"),
     py::arg("urows") = py::none());
  // Darlin row pass over dense per-row block layouts (bcd.hip bcd_rowpass): the pending
  // dual update of block j (jcol: [rows] int32 column relative to the block, -1 none)
  // fused with block k's gradient (narrow: part/G/U; wide: rowq).
  m.def("bcd_rowpass", [](Tensor ym, Tensor y, optional<Tensor> jcol, optional<Tensor> jval,
                          optional<Tensor> jdw, int64_t jncols, optional<Tensor> kcol,
                          optional<Tensor> kval, int64_t c0, int64_t ncols, Tensor delta,
                          Tensor active, int k2, int W, optional<Tensor> part,
                          optional<Tensor> G, optional<Tensor> U, optional<Tensor> rowq,
                          optional<Tensor> hcols, optional<Tensor> part2, bool tau32) {
    chk(ym, at::kDouble, "ym");
    chk(y, at::kFloat, "y");
    chk(delta, at::kDouble, "delta");
    chk(active, at::kByte, "active");
    const int64_t n = ym.numel();
    check(y.numel() == n, "y/ym size mismatch");
    const int32_t* jc = optr<int32_t>(jcol, at::kInt, "jcol");
    const float* jv = optr<float>(jval, at::kFloat, "jval");
    const double* jd = optr<double>(jdw, at::kDouble, "jdw");
    if (jc) {
      check(jcol->numel() == n, "jcol: one int32 per example");
      check(jd != nullptr && jncols >= 0 && jdw->numel() >= jncols, "jdw too small");
      if (jv) check(jval->numel() == n, "jval: one float per example");
    }
    const int32_t* kc = optr<int32_t>(kcol, at::kInt, "kcol");
    const float* kv = optr<float>(kval, at::kFloat, "kval");
    if (kc) {
      check(kcol->numel() == n, "kcol: one int32 per example");
      if (kv) check(kval->numel() == n, "kval: one float per example");
      check(c0 >= 0 && ncols >= 0 && c0 + ncols <= delta.numel(), "column block outside model");
    }
    long long* pp = optr<long long>(part, at::kLong, "part");
    double* Gp = optr<double>(G, at::kDouble, "G");
    double* Up = optr<double>(U, at::kDouble, "U");
    double* rq = optr<double>(rowq, at::kDouble, "rowq");
    const int32_t* hc = optr<int32_t>(hcols, at::kInt, "hcols");
    const int64_t nhot = hc ? hcols->numel() : 0;
    if (pp) {
      check(kc != nullptr, "LDS row pass needs kcol");
      const int64_t nl = hc ? nhot : ncols;
      check(nl <= psamd::bcd_rows_max_cols(), "bcd_rowpass: <= 2048 LDS columns");
      check(W >= 1 && part->numel() >= (int64_t)(W + psamd::bcd_part_segments()) * 2 * nl,
            "part: (W + bcd_part_segments) x 2 x LDS columns int64");
      check(Gp && Up && G->numel() >= ncols && U->numel() >= ncols, "G/U too small");
      check(k2 >= 0 && k2 <= 62, "fixed-point shift");
      // hot columns of a wide block (the reduce stores G[hcols[h]]): range-checked once
      // where they are built (ops/bcd.py hot_layout), not per call (no host sync here)
      if (hc) check(rq != nullptr && rowq->numel() >= 2 * n, "rowq: 2 doubles per example");
      if (part2.has_value() && part2->defined())
        check(part2->numel() >= (int64_t)psamd::bcd_part_segments() * 2 * nl,
              "part2: segments x 2 x LDS columns int64");
    } else if (kc) {
      check(rq != nullptr && rowq->numel() >= 2 * n, "rowq: 2 doubles per example");
    }
    psamd::bcd_rowpass(n, ptr<double>(ym), ptr<float>(y), jc, jv, jd, jncols, kc, kv, c0, ncols,
                       ptr<double>(delta), ptr<uint8_t>(active), k2, W, pp, Gp, Up, rq, hc, nhot,
                       optr<long long>(part2, at::kLong, "part2"), tau32, cur_stream());
  }, py::arg("ym"), py::arg("y"), py::arg("jcol"), py::arg("jval"), py::arg("jdw"),
     py::arg("jncols"), py::arg("kcol"), py::arg("kval"), py::arg("c0"), py::arg("ncols"),
     py::arg("delta"), py::arg("active"), py::arg("k2"), py::arg("W"), py::arg("part"),
     py::arg("G"), py::arg("U"), py::arg("rowq"), py::arg("hcols"), py::arg("part2"),
     py::arg("tau32") = false);
  m.def("bcd_grad", [csc_check](Tensor col, Tensor row, optional<Tensor> val, int64_t p0,
                                int64_t p1, int64_t c0, int64_t ncols, Tensor ym, Tensor y,
                                Tensor delta, Tensor active, Tensor G, Tensor U) {
    csc_check(col, row, val, p0, p1);
    chk(ym, at::kDouble, "ym");
    chk(y, at::kFloat, "y");
    chk(delta, at::kDouble, "delta");
    chk(active, at::kByte, "active");
    chk(G, at::kDouble, "G");
    chk(U, at::kDouble, "U");
    check(y.numel() == ym.numel(), "y/ym size mismatch");
    check(delta.numel() == active.numel(), "delta/active size mismatch");
    check(c0 >= 0 && ncols >= 0 && c0 + ncols <= delta.numel(), "column block outside model");
    check(G.numel() >= ncols && U.numel() >= ncols, "G/U too small");
    psamd::bcd_grad(ptr<int32_t>(col), ptr<int32_t>(row), optr<float>(val, at::kFloat, "val"), p0,
                    p1, c0, ncols, ptr<double>(ym), ptr<float>(y), ym.numel(), ptr<double>(delta),
                    ptr<uint8_t>(active), ptr<double>(G), ptr<double>(U), cur_stream());
  });
  m.def("bcd_update", [](int64_t c0, int64_t ncols, Tensor G, Tensor U, Tensor w, Tensor delta,
                         Tensor active, Tensor dw, double eta, double lambda, double delta_max,
                         double kkt_thr, Tensor vio_bits, bool consume, bool nan_filtered,
                         optional<Tensor> part2, int k2) {
    chk(G, at::kDouble, "G");
    chk(U, at::kDouble, "U");
    chk(w, at::kDouble, "w");
    chk(delta, at::kDouble, "delta");
    chk(active, at::kByte, "active");
    chk(dw, at::kDouble, "dw");
    chk(vio_bits, at::kLong, "vio_bits");
    check(w.numel() == delta.numel() && w.numel() == active.numel(), "model arrays mismatch");
    check(c0 >= 0 && ncols >= 0 && c0 + ncols <= w.numel(), "column block outside model");
    check(G.numel() >= ncols && U.numel() >= ncols && dw.numel() >= ncols, "G/U/dw too small");
    check(eta > 0, "eta must be > 0");
    const long long* p2 = optr<long long>(part2, at::kLong, "part2");
    if (p2)
      check(part2->numel() >= (int64_t)psamd::bcd_part_segments() * 2 * ncols && k2 >= 0 &&
                k2 <= 62,
            "part2: segments x 2 x ncols int64 (a narrow row pass's sums)");
    psamd::bcd_update(c0, ncols, ptr<double>(G), ptr<double>(U), ptr<double>(w),
                      ptr<double>(delta), ptr<uint8_t>(active), ptr<double>(dw), eta, lambda,
                      delta_max, kkt_thr, ptr<unsigned long long>(vio_bits), consume,
                      nan_filtered, p2, k2, cur_stream());
  });
  m.def("bcd_replica", [](int64_t c0, int64_t ncols, int64_t own0, int64_t own1, Tensor dw,
                          Tensor w, Tensor delta, Tensor active, double delta_max) {
    chk(dw, at::kDouble, "dw");
    chk(w, at::kDouble, "w");
    chk(delta, at::kDouble, "delta");
    chk(active, at::kByte, "active");
    check(w.numel() == delta.numel() && w.numel() == active.numel(), "model arrays mismatch");
    check(c0 >= 0 && ncols >= 0 && c0 + ncols <= w.numel(), "column block outside model");
    check(dw.numel() >= ncols, "dw too small");
    psamd::bcd_replica(c0, ncols, own0, own1, ptr<double>(dw), ptr<double>(w), ptr<double>(delta),
                       ptr<uint8_t>(active), delta_max, cur_stream());
  });
  m.def("bcd_dual", [csc_check](Tensor col, Tensor row, optional<Tensor> val, int64_t p0,
                                int64_t p1, int64_t c0, int64_t ncols, Tensor dw, Tensor y,
                                Tensor ym, bool unique_rows) {
    csc_check(col, row, val, p0, p1);
    chk(dw, at::kDouble, "dw");
    chk(y, at::kFloat, "y");
    chk(ym, at::kDouble, "ym");
    check(y.numel() == ym.numel(), "y/ym size mismatch");
    check(ncols >= 0 && dw.numel() >= ncols, "dw too small");
    psamd::bcd_dual(ptr<int32_t>(col), ptr<int32_t>(row), optr<float>(val, at::kFloat, "val"), p0,
                    p1, c0, ncols, ptr<double>(dw), ptr<float>(y), ptr<double>(ym), ym.numel(),
                    unique_rows, cur_stream());
  });
  m.def("bcd_rows_max_cols", []() { return psamd::bcd_rows_max_cols(); });
  m.def("bcd_part_segments", []() { return psamd::bcd_part_segments(); });
  m.def("bcd_grad_rows", [csc_check](Tensor col, Tensor row, optional<Tensor> val, int64_t p0,
                                     int64_t p1, int64_t c0, int64_t ncols, Tensor ym, Tensor y,
                                     Tensor delta, Tensor active, int k2, int W, Tensor part,
                                     Tensor G, Tensor U, optional<Tensor> w,
                                     optional<Tensor> dw, optional<Tensor> vio_bits,
                                     optional<Tensor> counter, double eta, double lambda,
                                     double delta_max, double kkt_thr) {
    csc_check(col, row, val, p0, p1);
    chk(ym, at::kDouble, "ym");
    chk(y, at::kFloat, "y");
    chk(delta, at::kDouble, "delta");
    chk(active, at::kByte, "active");
    chk(part, at::kLong, "part");
    chk(G, at::kDouble, "G");
    chk(U, at::kDouble, "U");
    check(y.numel() == ym.numel(), "y/ym size mismatch");
    check(ncols >= 0 && ncols <= psamd::bcd_rows_max_cols(), "bcd_grad_rows: ncols <= 2048");
    check(c0 >= 0 && c0 + ncols <= delta.numel() && delta.numel() == active.numel(),
          "block columns out of range");
    check(G.numel() >= ncols && U.numel() >= ncols, "G/U too small");
    check(W >= 1 && W <= 65535 &&
              part.numel() >= (int64_t)(dw.has_value() && dw->defined() ? 1 : W) * 2 * ncols,
          "partials buffer (fused update: the block's 2 x ncols accumulator)");
    check(k2 >= 0 && k2 <= 62, "fixed-point scale 2^0..2^62");
    // fused update (dw given): the last workgroup applies the coordinate step of every
    // column of the block (bcd_update's arithmetic) and writes dw
    double* dwp = optr<double>(dw, at::kDouble, "dw");
    double* wp = optr<double>(w, at::kDouble, "w");
    auto* vp = reinterpret_cast<unsigned long long*>(optr<int64_t>(vio_bits, at::kLong, "vio_bits"));
    auto* cp = reinterpret_cast<unsigned int*>(optr<int32_t>(counter, at::kInt, "counter"));
    if (dwp) {
      check(wp && vp && cp, "fused update needs w, vio_bits and counter");
      check(w->numel() == delta.numel() && dw->numel() >= ncols, "w / dw size");
      check(eta > 0, "eta must be > 0");
    }
    psamd::bcd_grad_rows(ptr<int32_t>(col), ptr<int32_t>(row), optr<float>(val, at::kFloat, "val"),
                         p0, p1, c0, ncols, ptr<double>(ym), ptr<float>(y), ym.numel(),
                         ptr<double>(delta), ptr<uint8_t>(active), k2, W,
                         reinterpret_cast<long long*>(part.data_ptr()), ptr<double>(G),
                         ptr<double>(U), wp, dwp, vp, cp, eta, lambda, delta_max, kkt_thr,
                         cur_stream());
  }, py::arg("col"), py::arg("row"), py::arg("val"), py::arg("p0"), py::arg("p1"), py::arg("c0"),
     py::arg("ncols"), py::arg("ym"), py::arg("y"), py::arg("delta"), py::arg("active"),
     py::arg("k2"), py::arg("W"), py::arg("part"), py::arg("G"), py::arg("U"),
     py::arg("w") = py::none(), py::arg("dw") = py::none(), py::arg("vio_bits") = py::none(),
     py::arg("counter") = py::none(), py::arg("eta") = 1.0, py::arg("lam") = 0.0,
     py::arg("delta_max") = 0.0, py::arg("kkt_thr") = 0.0);
  m.def("bcd_objective", [](Tensor ym, Tensor out) {
    chk(ym, at::kDouble, "ym");
    chk(out, at::kDouble, "out");
    check(out.numel() >= 1, "out needs 1 double");
    psamd::bcd_objective(ptr<double>(ym), ym.numel(), ptr<double>(out), cur_stream());
  });
  m.def("bcd_server_stats", [](Tensor w, Tensor active, int64_t c0, int64_t c1, Tensor out) {
    chk(w, at::kDouble, "w");
    chk(active, at::kByte, "active");
    chk(out, at::kDouble, "out");
    check(w.numel() == active.numel(), "w/active mismatch");
    check(0 <= c0 && c0 <= c1 && c1 <= w.numel(), "range outside model");
    check(out.numel() >= 3, "out needs 3 doubles");
    psamd::bcd_server_stats(ptr<double>(w), ptr<uint8_t>(active), c0, c1, ptr<double>(out),
                            cur_stream());
  });

  // ------------------------------------------------------------------ bf16 GEMM
  // C[m,n] = sum_k A(m,k) B(n,k); A(m,k) = A[m*lda+k] if a_kmajor else A[k*lda+m] (B alike)
  m.def("gemm_bf16", [](Tensor A, bool a_kmajor, int64_t lda, Tensor B, bool b_kmajor,
                        int64_t ldb, int64_t M, int64_t N, int64_t K, int epi,
                        optional<Tensor> bias, optional<Tensor> aux, int64_t ldaux,
                        optional<Tensor> C, int64_t ldc, optional<Tensor> Cf, int64_t ldcf,
                        double beta, int splitk, optional<Tensor> colsum) {
    chk(A, at::kBFloat16, "A");
    chk(B, at::kBFloat16, "B");
    check(M > 0 && N > 0 && K > 0 && M < INT32_MAX && N < INT32_MAX && K < INT32_MAX,
          "bad GEMM shape");
    auto need = [&](const Tensor& t, bool kmaj, int64_t ld, int64_t rows, const char* nm) {
      check(ld % 8 == 0, std::string(nm) + ": leading dimension must be a multiple of 8");
      check(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
            std::string(nm) + ": must be 16-byte aligned");
      if (kmaj) {
        check(K % 8 == 0 && ld >= K, std::string(nm) + ": K-major needs K % 8 == 0, ld >= K");
        check(t.numel() >= (rows - 1) * ld + K, std::string(nm) + ": too small");
      } else {
        check(rows % 8 == 0 && ld >= rows, std::string(nm) + ": MN-major needs rows % 8 == 0");
        check(t.numel() >= (K - 1) * ld + rows, std::string(nm) + ": too small");
      }
    };
    need(A, a_kmajor, lda, M, "A");
    need(B, b_kmajor, ldb, N, "B");
    const float* bp = optr<float>(bias, at::kFloat, "bias");
    if (epi & 1) check(bp && bias->numel() >= N, "EPI_BIAS needs bias[N]");
    const void* xp = nullptr;
    if (epi & 4) {
      check(aux.has_value() && aux->defined(), "EPI_MASK needs aux");
      chk(*aux, at::kBFloat16, "aux");
      check(aux->numel() >= (M - 1) * ldaux + N, "aux too small");
      xp = aux->data_ptr();
    }
    void* cp = nullptr;
    if (C.has_value() && C->defined()) {
      chk(*C, at::kBFloat16, "C");
      check(ldc >= N && C->numel() >= (M - 1) * ldc + N, "C too small");
      cp = C->data_ptr();
    }
    float* cfp = optr<float>(Cf, at::kFloat, "Cf");
    if (cfp) check(ldcf >= N && Cf->numel() >= (M - 1) * ldcf + N, "Cf too small");
    check(cp || cfp, "GEMM needs an output");
    if (splitk > 1)
      check(!cp && cfp && (epi & ~8) == 0 && (beta == 0.0 || beta == 1.0),
            "split-K: fp32 output only, no epilogue, beta 0 or 1");
    float* csp = optr<float>(colsum, at::kFloat, "colsum");
    check(!(epi & 8) || (csp && colsum->numel() >= N), "EPI_COLSUM needs colsum[N]");
    psamd::gemm_bf16(a_kmajor, b_kmajor, A.data_ptr(), (int)lda, B.data_ptr(), (int)ldb, (int)M,
                     (int)N, (int)K, epi, bp, xp, (int)ldaux, cp, (int)ldc, cfp, (int)ldcf,
                     (float)beta, splitk, csp, cur_stream());
  });


  // ------------------------------------------------------------- embeddings
  auto rows_check = [](const Tensor& rows, int64_t cap, int D) {
    chk(rows, at::kBFloat16, "rows");
    check(D > 0 && D % 8 == 0 && D <= 128, "embedding dim must be a multiple of 8, <= 128");
    check(rows.dim() == 2 && rows.size(0) == cap && rows.size(1) == D, "rows must be [cap, D]");
  };
  m.def("emb_init_rows", [rows_check](Tensor slot, Tensor keys, optional<Tensor> n_dev,
                                      Tensor rows, Tensor inited, uint64_t seed, double scale) {
    chk(slot, at::kLong, "slot");
    chk(keys, at::kLong, "keys");
    chk(inited, at::kByte, "inited");
    const int64_t cap = inited.numel();
    rows_check(rows, cap, (int)rows.size(1));
    check(keys.numel() >= slot.numel(), "keys shorter than slot");
    psamd::emb_init_rows(ptr<int64_t>(slot), ptr<uint64_t>(keys), slot.numel(),
                         optr<int32_t>(n_dev, at::kInt, "n_dev"), cap, rows.data_ptr(),
                         ptr<uint8_t>(inited), (int)rows.size(1), seed, (float)scale,
                         cur_stream());
  });
  m.def("emb_gather_rows", [rows_check](Tensor slot, Tensor rows, Tensor out,
                                         optional<Tensor> n_dev) {
    // out[i, :] = rows[slot[i], :] for i < n_dev (device count, clamped) or slot.numel()
    chk(slot, at::kLong, "slot");
    rows_check(rows, rows.size(0), (int)rows.size(1));
    chk(out, at::kBFloat16, "out");
    check(out.numel() >= slot.numel() * rows.size(1), "out too small");
    psamd::emb_gather_rows(ptr<int64_t>(slot), slot.numel(), optr<int32_t>(n_dev, at::kInt, "n_dev"),
                           rows.size(0), rows.data_ptr(), (int)rows.size(1), out.data_ptr(),
                           cur_stream());
  }, py::arg("slot"), py::arg("rows"), py::arg("out"), py::arg("n_dev") = py::none());
  m.def("emb_expand", [](Tensor local_col, int64_t nnz, optional<Tensor> idx, Tensor src,
                         Tensor X0) {
    chk(local_col, at::kInt, "local_col");
    chk(src, at::kBFloat16, "src");
    chk(X0, at::kBFloat16, "X0");
    check(src.dim() == 2 && src.size(1) % 8 == 0, "src must be [rows, D], D % 8 == 0");
    const int D = (int)src.size(1);
    check(local_col.numel() >= nnz && X0.numel() >= nnz * D, "expand buffers too small");
    const int64_t* ip = optr<int64_t>(idx, at::kLong, "idx");
    psamd::emb_expand(ptr<int32_t>(local_col), nnz, ip, ip ? idx->numel() : 0, src.data_ptr(),
                      src.size(0), D, X0.data_ptr(), cur_stream());
  });
  // padded (sync-free) exchange of the embedding models; records [C x D bf16 | C f32]
  // per peer chunk (Q = C*D/2 + C int32 words)
  m.def("emb_padded_serve", [](Tensor recv, int64_t H, int64_t C, int kw, Tensor slot, Tensor w,
                               Tensor rows, Tensor inited, int64_t seed, double scale,
                               Tensor out) {
    chk(recv, at::kInt, "recv");
    chk(slot, at::kLong, "slot");
    chk(w, at::kFloat, "w");
    chk(rows, at::kBFloat16, "rows");
    chk(inited, at::kByte, "inited");
    chk(out, at::kInt, "out");
    check(kw == 1 || kw == 2, "kw 1 or 2");
    check(rows.dim() == 2 && rows.size(1) % 8 == 0, "rows [cap, D], D % 8 == 0");
    const int D = (int)rows.size(1);
    check(C > 0 && C % 4 == 0 && H >= 4 + C * kw, "C % 4 == 0, H >= 4 + C kw");
    const int64_t G = recv.numel() / H;
    check(G >= 1 && recv.numel() == G * H, "recv = G rows of H");
    check(slot.numel() >= G * C && w.numel() >= G * C, "slot / w [G*C]");
    check(inited.numel() >= rows.size(0), "inited [cap]");
    check(out.numel() >= G * (C * (D / 2) + C), "out [G * Q]");
    psamd::emb_padded_serve(ptr<int32_t>(recv), H, C, kw, (int)G, ptr<int64_t>(slot),
                            ptr<float>(w), rows.size(0), rows.data_ptr(), ptr<uint8_t>(inited), D,
                            (uint64_t)seed, (float)scale, ptr<int32_t>(out), cur_stream());
  });
  m.def("emb_unpack_records", [](Tensor in, int64_t C, Tensor off, Tensor n_uniq, Tensor rows_u,
                                 Tensor w_u) {
    chk(in, at::kInt, "in");
    chk(off, at::kLong, "off");
    chk(n_uniq, at::kInt, "n_uniq");
    chk(rows_u, at::kBFloat16, "rows_u");
    chk(w_u, at::kFloat, "w_u");
    check(rows_u.dim() == 2 && rows_u.size(1) % 8 == 0, "rows_u [u_cap, D]");
    const int D = (int)rows_u.size(1);
    const int G = (int)off.numel() - 1;
    check(G >= 1 && C > 0 && C % 4 == 0, "off [G+1], C % 4 == 0");
    check(in.numel() >= (int64_t)G * (C * (D / 2) + C), "in [G * Q]");
    check(w_u.numel() >= rows_u.size(0), "w_u [u_cap]");
    psamd::emb_unpack_records(ptr<int32_t>(in), C, G, ptr<int64_t>(off), ptr<int32_t>(n_uniq),
                              rows_u.size(0), D, rows_u.data_ptr(), ptr<float>(w_u),
                              cur_stream());
  });
  m.def("emb_pack_grads", [](Tensor dE, Tensor g_wide, Tensor off, Tensor n_uniq, int64_t C,
                             Tensor out) {
    chk(dE, at::kFloat, "dE");
    chk(g_wide, at::kFloat, "g_wide");
    chk(off, at::kLong, "off");
    chk(n_uniq, at::kInt, "n_uniq");
    chk(out, at::kInt, "out");
    check(dE.dim() == 2 && dE.size(1) % 8 == 0, "dE [u_cap, D]");
    const int D = (int)dE.size(1);
    const int G = (int)off.numel() - 1;
    check(G >= 1 && C > 0 && C % 4 == 0, "off [G+1], C % 4 == 0");
    check(g_wide.numel() >= dE.size(0), "g_wide [u_cap]");
    check(out.numel() >= (int64_t)G * (C * (D / 2) + C), "out [G * Q]");
    psamd::emb_pack_grads(ptr<float>(dE), ptr<float>(g_wide), ptr<int64_t>(off),
                          ptr<int32_t>(n_uniq), dE.size(0), C, G, D, ptr<int32_t>(out),
                          cur_stream());
  });
  m.def("emb_grad_wide_ok", [](int D) { return psamd::emb_grad_wide_ok(D); });
  m.def("emb_grad_reduce", [](Tensor pos_s, Tensor segid, Tensor seg_start, Tensor n_uniq,
                              int64_t u_cap, int64_t nnz, Tensor dX0, int D, Tensor dE,
                              optional<Tensor> coef, int width, optional<Tensor> g_wide) {
    chk(pos_s, at::kInt, "pos_s");
    chk(segid, at::kInt, "segid");
    check(segid.numel() >= nnz, "segid too small");
    chk(seg_start, at::kInt, "seg_start");
    chk(n_uniq, at::kInt, "n_uniq");
    chk(dX0, at::kBFloat16, "dX0");
    chk(dE, at::kFloat, "dE");
    check(D > 0 && D % 8 == 0, "D % 8 == 0");
    check(seg_start.numel() >= u_cap + 1 && pos_s.numel() >= nnz, "segment arrays too small");
    check(dX0.numel() >= nnz * D && dE.numel() >= u_cap * D, "gradient buffers too small");
    // run partials of the segmented wavefront kernels (D = 128 / 256; from the
    // caching allocator, so graph captures keep it in their pool)
    const int64_t pf = psamd::emb_grad_part_floats(nnz, D);
    Tensor part = pf ? at::empty({pf}, dE.options()) : Tensor();
    // wide & deep: g_wide[u] = sum of coef[row] over u's occurrences (row = pos / width)
    const bool wide = g_wide.has_value();
    if (wide) {
      check(coef.has_value() && width > 0 && nnz % width == 0, "g_wide needs coef and width");
      chk(*coef, at::kFloat, "coef");
      chk(*g_wide, at::kFloat, "g_wide");
      check(coef->numel() >= nnz / width && g_wide->numel() >= u_cap, "coef / g_wide too small");
      check(psamd::emb_grad_wide_ok(D), "g_wide rides along only with D = 128 / 256");
    }
    psamd::emb_grad_reduce(ptr<int32_t>(pos_s), ptr<int32_t>(segid), ptr<int32_t>(seg_start),
                           ptr<int32_t>(n_uniq), u_cap, nnz, dX0.data_ptr(), D, ptr<float>(dE),
                           pf ? ptr<float>(part) : nullptr, wide ? ptr<float>(*coef) : nullptr,
                           wide ? width : 0, wide ? ptr<float>(*g_wide) : nullptr, cur_stream());
  }, py::arg("pos_s"), py::arg("segid"), py::arg("seg_start"), py::arg("n_uniq"),
     py::arg("u_cap"), py::arg("nnz"), py::arg("dX0"), py::arg("D"), py::arg("dE"),
     py::arg("coef") = py::none(), py::arg("width") = 0, py::arg("g_wide") = py::none());
  // wide & deep: wide = (slots, g_wide, algo, lr_type, alpha, beta, l1, l2, grad_scale,
  // max_delta) also applies the keys' wide gradients to their table slots (kv_update's
  // update and stats) in the same pass
  m.def("emb_update", [rows_check](Tensor slot, optional<Tensor> n_dev, optional<Tensor> grad,
                                   optional<Tensor> grad16, Tensor rows, Tensor acc, double lr,
                                   double eps, optional<Tensor> slots, optional<Tensor> g_wide,
                                   std::vector<double> rule, optional<Tensor> stats) {
    chk(slot, at::kLong, "slot");
    chk(acc, at::kFloat, "acc");
    const int64_t cap = acc.numel();
    const int D = (int)rows.size(1);
    rows_check(rows, cap, D);
    const float* gp = optr<float>(grad, at::kFloat, "grad");
    const void* g16 = nullptr;
    if (!gp) {
      check(grad16.has_value() && grad16->defined(), "emb_update needs grad or grad16");
      chk(*grad16, at::kBFloat16, "grad16");
      check(grad16->numel() >= slot.numel() * D, "grad16 too small");
      g16 = grad16->data_ptr();
    } else {
      check(grad->numel() >= slot.numel() * D, "grad too small");
    }
    void* sp = nullptr;
    const float* gw = nullptr;
    int wr[2] = {0, 0};
    float wh[6] = {0, 0, 0, 0, 0, 0};
    if (slots.has_value()) {
      check(slot_capacity(*slots) == cap, "emb_update: slots and rows must be one table");
      chk(*g_wide, at::kFloat, "g_wide");
      check(g_wide->numel() >= slot.numel(), "g_wide too small");
      check(rule.size() == 8, "wide rule = algo, lr_type, alpha, beta, l1, l2, grad_scale, max_delta");
      check(rule[2] > 0, "learning rate alpha must be > 0");
      sp = slots->data_ptr();
      gw = ptr<float>(*g_wide);
      wr[0] = (int)rule[0];
      wr[1] = (int)rule[1];
      for (int q = 0; q < 6; ++q) wh[q] = (float)rule[2 + q];
    }
    psamd::emb_update(ptr<int64_t>(slot), slot.numel(), optr<int32_t>(n_dev, at::kInt, "n_dev"),
                      cap, gp, g16, rows.data_ptr(), ptr<float>(acc), D, (float)lr, (float)eps, sp,
                      gw, wr, wh, optr<double>(stats, at::kDouble, "stats"), acc_stripes_of(stats),
                      cur_stream());
  }, py::arg("slot"), py::arg("n_dev"), py::arg("grad"), py::arg("grad16"), py::arg("rows"),
     py::arg("acc"), py::arg("lr"), py::arg("eps"), py::arg("slots") = py::none(),
     py::arg("g_wide") = py::none(), py::arg("rule") = std::vector<double>{},
     py::arg("stats") = py::none());
  m.def("wd_head", [](Tensor h, Tensor w, Tensor b, Tensor wide_w, Tensor local_col, int S,
                      Tensor labels, Tensor coef, Tensor dh, Tensor dw, Tensor db, Tensor metrics,
                      Tensor hist, int nbins, optional<Tensor> db_h) {
    chk(h, at::kBFloat16, "h");
    chk(w, at::kFloat, "w");
    chk(b, at::kFloat, "b");
    chk(wide_w, at::kFloat, "wide_w");
    chk(local_col, at::kInt, "local_col");
    chk(labels, at::kFloat, "labels");
    chk(coef, at::kFloat, "coef");
    chk(dh, at::kBFloat16, "dh");
    chk(dw, at::kFloat, "dw");
    chk(db, at::kFloat, "db");
    chk(metrics, at::kDouble, "metrics");
    chk(hist, at::kInt, "hist");
    check(h.dim() == 2, "h must be [B, H]");
    const int64_t B = h.size(0);
    const int H = (int)h.size(1);
    check(H > 0 && H <= 512 && w.numel() == H && dw.numel() == H, "head width H in (0, 512]");
    check(S > 0 && S <= 64 && local_col.numel() >= B * S, "S in (0, 64], local_col [B*S]");
    check(labels.numel() >= B && coef.numel() >= B && dh.numel() >= B * H, "head buffers small");
    check(metrics.numel() >= 3 && hist.numel() >= 2 * nbins && nbins > 0, "metrics / hist");
    float* dbh = optr<float>(db_h, at::kFloat, "db_h");
    check(!dbh || db_h->numel() >= H, "db_h [H]");
    check(H % 8 == 0, "head width H % 8 == 0");
    psamd::wd_head(h.data_ptr(), B, H, ptr<float>(w), ptr<float>(b), ptr<float>(wide_w),
                   wide_w.numel(), ptr<int32_t>(local_col), S, ptr<float>(labels),
                   ptr<float>(coef), dh.data_ptr(), ptr<float>(dw), ptr<float>(db), dbh,
                   ptr<double>(metrics), reinterpret_cast<uint32_t*>(hist.data_ptr()), nbins,
                   acc_stripes_of(metrics), cur_stream());
  });
  m.def("colsum_bf16", [](Tensor x, Tensor out) {
    chk(x, at::kBFloat16, "x");
    chk(out, at::kFloat, "out");
    check(x.dim() == 2 && out.numel() >= x.size(1), "colsum: x [B, N], out [N]");
    check(x.size(1) % 8 == 0, "colsum: N % 8 == 0");
    psamd::colred_bf16(x.data_ptr(), x.size(0), (int)x.size(1), nullptr, ptr<float>(out), nullptr,
                       nullptr, cur_stream());
  });
  m.def("adam_update", [](Tensor p, Tensor g, Tensor m_, Tensor v, double lr, double b1,
                          double b2, double eps, int64_t step, double gscale,
                          optional<Tensor> p16, optional<Tensor> step_dev, bool zero_grad) {
    chk(p, at::kFloat, "p");
    chk(g, at::kFloat, "g");
    chk(m_, at::kFloat, "m");
    chk(v, at::kFloat, "v");
    const int64_t n = p.numel();
    check(g.numel() == n && m_.numel() == n && v.numel() == n, "adam buffers mismatch");
    void* p16p = nullptr;
    if (p16.has_value() && p16->defined()) {
      chk(*p16, at::kBFloat16, "p16");
      check(p16->numel() == n, "p16 mismatch");
      p16p = p16->data_ptr();
    }
    const int64_t* sd = nullptr;  // device step clock (graph-captured steps)
    if (step_dev.has_value() && step_dev->defined()) {
      chk(*step_dev, at::kLong, "step_dev");
      sd = step_dev->data_ptr<int64_t>();
    } else {
      check(step >= 1, "adam step >= 1");
    }
    const double s1 = (double)(step >= 1 ? step : 1);
    const double bc1 = 1.0 - std::pow(b1, s1), bc2 = 1.0 - std::pow(b2, s1);
    psamd::adam_update(ptr<float>(p), ptr<float>(g), ptr<float>(m_), ptr<float>(v), n, (float)lr,
                       (float)b1, (float)b2, (float)eps, (float)bc1, (float)bc2, (float)gscale,
                       p16p, sd, zero_grad, cur_stream());
  });
  // SparseMatrix::times (utils/matrix.py): gather (row-reduce) or scatter (atomic) over the
  // compressed major dimension; y = alpha * A x + beta * y.
  m.def("spmv", [](bool scatter, Tensor off, Tensor idx, optional<Tensor> val, Tensor x, Tensor y,
                   double alpha, double beta) {
    chk(off, at::kLong, "offset");
    check(idx.is_cuda() && idx.is_contiguous() &&
              (idx.scalar_type() == at::kInt || idx.scalar_type() == at::kLong),
          "spmv: index must be contiguous int32/int64 on the GPU");
    check(x.is_cuda() && x.is_contiguous() &&
              (x.scalar_type() == at::kFloat || x.scalar_type() == at::kDouble),
          "spmv: x must be contiguous float32/float64 on the GPU");
    chk(y, x.scalar_type(), "y");
    const int64_t n_major = off.numel() - 1, nnz = idx.numel();
    check(n_major >= 0, "spmv: offset must have n_major + 1 entries");
    const void* vp = nullptr;
    if (val.has_value() && val->defined()) {
      chk(*val, x.scalar_type(), "value");
      check(val->numel() == nnz, "spmv: value / index length mismatch");
      vp = val->data_ptr();
    }
    if (scatter) check(x.numel() >= n_major, "spmv(scatter): x shorter than the major dimension");
    else check(y.numel() >= n_major, "spmv(gather): y shorter than the major dimension");
    psamd::spmv(scatter, ptr<int64_t>(off), idx.data_ptr(), (int)idx.element_size(), vp,
                (int)x.element_size(), n_major, nnz, x.data_ptr(), x.numel(), alpha, beta,
                y.data_ptr(), y.numel(), cur_stream());
  });
}
