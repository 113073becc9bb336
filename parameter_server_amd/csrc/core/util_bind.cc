#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <zlib.h>

#include "hashing.h"
#include "textproto.h"
#include "module_parts.h"

namespace py = pybind11;

namespace pscore {

namespace {
py::list tp_to_py(const TPMessage& m) {
  py::list out;
  for (const auto& [name, v] : m.fields) {
    if (v.kind == TPValue::kMessage) {
      out.append(py::make_tuple(name, "message", tp_to_py(*v.msg)));
    } else {
      const char* k = v.kind == TPValue::kNumber ? "number"
                      : v.kind == TPValue::kString ? "string" : "ident";
      out.append(py::make_tuple(name, k, py::bytes(v.text)));
    }
  }
  return out;
}

TPMessage py_to_tp(const py::list& l) {
  TPMessage m;
  for (auto item : l) {
    auto t = item.cast<py::tuple>();
    TPValue v;
    const std::string kind = t[1].cast<std::string>();
    if (kind == "message") {
      v.kind = TPValue::kMessage;
      v.msg = std::make_shared<TPMessage>(py_to_tp(t[2].cast<py::list>()));
    } else {
      v.kind = kind == "number" ? TPValue::kNumber
               : kind == "string" ? TPValue::kString : TPValue::kIdent;
      v.text = t[2].cast<std::string>();
    }
    m.fields.emplace_back(t[0].cast<std::string>(), v);
  }
  return m;
}
}  // namespace

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
  m.def("parse_textproto", [](const std::string& src) {
    try {
      return tp_to_py(parse_textproto(src));
    } catch (const TextProtoError& e) {
      throw py::value_error(e.what());
    }
  });
  m.def("print_textproto", [](const py::list& fields) { return print_textproto(py_to_tp(fields)); });
  m.def("zlib_compress", [](py::bytes b, int level) {
    std::string s = b;
    uLongf n = compressBound(s.size());
    std::string out(n, '\0');
    {
      py::gil_scoped_release rel;
      if (compress2((Bytef*)out.data(), &n, (const Bytef*)s.data(), s.size(), level) != Z_OK)
        throw std::runtime_error("zlib compress failed");
    }
    out.resize(n);
    return py::bytes(out);
  }, py::arg("data"), py::arg("level") = 1);
  m.def("zlib_decompress", [](py::bytes b, size_t raw_size) {
    std::string s = b;
    std::string out(raw_size, '\0');
    uLongf n = raw_size;
    {
      py::gil_scoped_release rel;
      if (uncompress((Bytef*)out.data(), &n, (const Bytef*)s.data(), s.size()) != Z_OK || n != raw_size)
        throw std::runtime_error("zlib decompress failed");
    }
    return py::bytes(out);
  });
}

}  // namespace pscore
