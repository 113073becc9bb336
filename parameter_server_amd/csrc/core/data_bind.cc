#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "data.h"
#include "module_parts.h"

namespace py = pybind11;

namespace pscore {

template <typename T>
static py::array_t<T> to_np(std::vector<T>&& v) {
  auto* heap = new std::vector<T>(std::move(v));
  py::capsule owner(heap, [](void* p) { delete reinterpret_cast<std::vector<T>*>(p); });
  return py::array_t<T>({(py::ssize_t)heap->size()}, {(py::ssize_t)sizeof(T)}, heap->data(), owner);
}

static py::dict batch_to_py(ParsedBatch&& b) {
  py::dict d;
  d["binary"] = b.binary;
  d["bad_lines"] = b.bad_lines;
  py::dict info;
  for (auto& [id, s] : b.info) {
    py::dict x;
    x["min_key"] = s.min_key;
    x["max_key"] = s.max_key;
    x["nnz_ele"] = s.nnz_ele;
    x["nnz_ex"] = s.nnz_ex;
    x["format"] = s.format;
    info[py::int_(id)] = x;
  }
  d["info"] = info;
  d["labels"] = to_np(std::move(b.labels));
  d["row_ptr"] = to_np(std::move(b.row_ptr));
  d["keys"] = to_np(std::move(b.keys));
  d["vals"] = to_np(std::move(b.vals));
  d["slots"] = to_np(std::move(b.slots));
  return d;
}

void register_data(py::module_& m) {
  m.def("parse_text", [](py::bytes data, int format, bool ignore_slot, bool shuffle_fea_id,
                         uint64_t hash_mod, int nthreads, int64_t max_lines) {
    // (parsed in place: the bytes object is immutable and held by this call)
    char* ptr = nullptr;
    Py_ssize_t len = 0;
    if (PyBytes_AsStringAndSize(data.ptr(), &ptr, &len) != 0) throw py::error_already_set();
    ParseOptions opt;
    opt.format = (TextFormat)format;
    opt.ignore_fea_slot = ignore_slot;
    opt.shuffle_fea_id = shuffle_fea_id;
    opt.hash_mod = hash_mod;
    opt.nthreads = nthreads;
    opt.max_lines = max_lines;
    ParsedBatch b;
    {
      py::gil_scoped_release rel;
      b = parse_buffer(ptr, (size_t)len, opt);
    }
    return batch_to_py(std::move(b));
  }, py::arg("data"), py::arg("format"), py::arg("ignore_slot") = false,
     py::arg("shuffle_fea_id") = false, py::arg("hash_mod") = 0, py::arg("nthreads") = 1,
     py::arg("max_lines") = -1);
  m.def("read_file", [](const std::string& path, const std::string& hadoop_home) {
    // a plain local file goes straight into the bytes object (no second copy)
    const bool plain = hadoop_home.empty() && path.rfind("hdfs://", 0) != 0 &&
                       !(path.size() >= 3 && path.compare(path.size() - 3, 3, ".gz") == 0);
    if (plain) {
      FILE* f = fopen(path.c_str(), "rb");
      if (!f) throw std::runtime_error("cannot open " + path);
      fseek(f, 0, SEEK_END);
      const long sz = ftell(f);
      fseek(f, 0, SEEK_SET);
      PyObject* o = PyBytes_FromStringAndSize(nullptr, sz < 0 ? 0 : sz);
      if (!o) {
        fclose(f);
        throw py::error_already_set();
      }
      size_t got = 0;
      {
        py::gil_scoped_release rel;
        got = fread(PyBytes_AS_STRING(o), 1, (size_t)(sz < 0 ? 0 : sz), f);
      }
      fclose(f);
      py::bytes out = py::reinterpret_steal<py::bytes>(o);
      if ((long)got != sz) throw std::runtime_error("short read of " + path);
      return out;
    }
    std::string s;
    {
      py::gil_scoped_release rel;
      s = read_file(path, hadoop_home);
    }
    return py::bytes(s);
  }, py::arg("path"), py::arg("hadoop_home") = "");
  m.def("write_file", [](const std::string& path, py::bytes data, bool gzip) {
    std::string s = data;
    py::gil_scoped_release rel;
    write_file(path, s, gzip);
  }, py::arg("path"), py::arg("data"), py::arg("gzip") = false);
  m.def("list_dir", &list_dir, py::arg("dir"), py::arg("hadoop_home") = "");
  m.def("recordio_pack", [](const std::vector<py::bytes>& recs) {
    std::vector<std::string> v(recs.begin(), recs.end());
    return py::bytes(recordio_pack(v));
  });
  m.def("recordio_unpack", [](py::bytes data) {
    std::vector<py::bytes> out;
    for (auto& r : recordio_unpack(data)) out.emplace_back(r);
    return out;
  });
  m.attr("RECORDIO_MAGIC") = kRecordIOMagic;
}

}  // namespace pscore
