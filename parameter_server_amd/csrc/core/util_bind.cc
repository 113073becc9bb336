#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "hashing.h"
#include "module_parts.h"

namespace py = pybind11;

namespace pscore {

void register_util(py::module_& m) {
  m.def("crc32c", [](py::bytes b, uint32_t init) {
    std::string s = b;
    return crc32c_extend(init, s.data(), s.size());
  }, py::arg("data"), py::arg("init") = 0u);
  m.def("crc32c_ptr", [](uintptr_t p, size_t n) {
    return crc32c(reinterpret_cast<const void*>(p), n);
  });
  m.def("murmur3_32", [](py::bytes b, uint32_t seed) {
    std::string s = b;
    return murmur3_32(s.data(), s.size(), seed);
  }, py::arg("data"), py::arg("seed") = 0u);
  m.def("murmur3_x64_128", [](py::bytes b, uint32_t seed) {
    std::string s = b;
    uint64_t out[2];
    murmur3_x64_128(s.data(), s.size(), seed, out);
    return py::make_tuple(out[0], out[1]);
  }, py::arg("data"), py::arg("seed") = 0u);
}

}  // namespace pscore
