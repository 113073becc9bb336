// pybind11 module for the host C++ runtime (_pscore). Buffers are passed as raw
// addresses (tensor.data_ptr() / ndarray.ctypes.data) plus element counts so
// this module does not depend on torch.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <stdexcept>

#include "cpu_kernels.h"
#include "module_parts.h"

namespace py = pybind11;
using namespace pscore;

template <typename T>
static T* P(uintptr_t a) { return reinterpret_cast<T*>(a); }

PYBIND11_MODULE(_pscore, m) {
  m.doc() = "parameter_server_amd host runtime (C++17)";

  m.def("keymix_params", [](int bits) {
    auto k = make_keymix(bits);
    return py::make_tuple(k.mask, k.a, k.b, k.ai, k.bi, k.s, k.bits);
  });
  m.def("mix_keys", [](uintptr_t in, uintptr_t out, int64_t n, int bits, bool inverse) {
    auto k = make_keymix(bits);
    const uint64_t* x = P<const uint64_t>(in);
    uint64_t* y = P<uint64_t>(out);
    py::gil_scoped_release rel;
    for (int64_t i = 0; i < n; ++i) y[i] = inverse ? unmix_key(x[i], k) : mix_key(x[i], k);
  });
  m.def("fmix64", [](uint64_t k) { return fmix64(k); });

  m.def("kv_init", [](uintptr_t slots, int64_t cap) {
    py::gil_scoped_release rel;
    kv_init(P<Slot>(slots), cap);
  });
  m.def("kv_resolve", [](uintptr_t slots, int64_t cap, uintptr_t keys, int64_t n,
                         uintptr_t out_slot, uintptr_t out_w, bool insert, int init_type,
                         double init_v, double init_s, uint64_t seed, uint64_t home_base,
                         uint64_t home_m) {
    if (cap <= 0 || (cap & (cap - 1))) throw std::invalid_argument("capacity must be 2^k");
    bool full = false;
    int64_t ins;
    {
      py::gil_scoped_release rel;
      ins = kv_resolve(P<Slot>(slots), cap, P<const uint64_t>(keys), n, P<int64_t>(out_slot),
                       out_w ? P<float>(out_w) : nullptr, insert, init_type, (float)init_v,
                       (float)init_s, seed, &full, home_base, home_m);
    }
    return py::make_tuple(ins, full);
  }, py::arg("slots"), py::arg("cap"), py::arg("keys"), py::arg("n"), py::arg("out_slot"),
     py::arg("out_w"), py::arg("insert"), py::arg("init_type"), py::arg("init_v"),
     py::arg("init_s"), py::arg("seed"), py::arg("home_base") = 0, py::arg("home_m") = 0);
  m.def("kv_gather", [](uintptr_t slots, uintptr_t idx, int64_t n, uintptr_t out, int field) {
    py::gil_scoped_release rel;
    kv_gather(P<const Slot>(slots), P<const int64_t>(idx), n, P<float>(out), field);
  });
  m.def("kv_set", [](uintptr_t slots, uintptr_t idx, int64_t n, uintptr_t w, uintptr_t z,
                     uintptr_t nn) {
    py::gil_scoped_release rel;
    kv_set(P<Slot>(slots), P<const int64_t>(idx), n, w ? P<const float>(w) : nullptr,
           z ? P<const float>(z) : nullptr, nn ? P<const float>(nn) : nullptr);
  });
  m.def("kv_update", [](uintptr_t slots, uintptr_t idx, uintptr_t grad, int64_t n, int algo,
                        int lr_type, double alpha, double beta, double l1, double l2,
                        double grad_scale, double max_delta, uintptr_t stats) {
    if (!(alpha > 0)) throw std::invalid_argument("learning rate alpha must be > 0");
    UpdateParams p{algo, lr_type, (float)alpha, (float)beta, (float)l1, (float)l2,
                   (float)grad_scale, (float)max_delta};
    py::gil_scoped_release rel;
    kv_update(P<Slot>(slots), P<const int64_t>(idx), P<const float>(grad), n, p,
              stats ? P<double>(stats) : nullptr);
  });
  m.def("kv_census", [](uintptr_t slots, int64_t cap) {
    int64_t o, z;
    kv_census(P<const Slot>(slots), cap, &o, &z);
    return py::make_tuple(o, z);
  });
  m.def("sketch_hash", [](uint64_t k) { return sketch_hash(k); });
  m.def("cm_insert", [](uintptr_t cells, uint64_t n_cells, int k, int vmax, uintptr_t keys,
                        uintptr_t counts, int64_t n) {
    py::gil_scoped_release rel;
    cm_insert(P<uint8_t>(cells), n_cells, k, (uint32_t)vmax, P<const uint64_t>(keys),
              counts ? P<const uint8_t>(counts) : nullptr, n);
  });
  m.def("cm_query", [](uintptr_t cells, uint64_t n_cells, int k, int vmax, uintptr_t keys,
                       int64_t n, int freq, uintptr_t keep, uintptr_t out_count) {
    py::gil_scoped_release rel;
    cm_query(P<const uint8_t>(cells), n_cells, k, (uint32_t)vmax, P<const uint64_t>(keys), n,
             freq, keep ? P<int32_t>(keep) : nullptr,
             out_count ? P<uint8_t>(out_count) : nullptr);
  });

  register_util(m);
  register_data(m);
  register_runtime(m);
  register_setops(m);
}
