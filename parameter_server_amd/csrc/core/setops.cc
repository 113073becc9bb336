// Sorted-key set algebra and bit sketches for the host runtime.
//
// Reference:
//  * parallelOrderedMatch (src/util/parallel_ordered_match.h:5-86): for two
//    ascending key lists apply op(src_val[i], dst_val[j]) where keys are equal,
//    recursively splitting dst across std::threads; ops assign / plus / or.
//  * parallelUnion (parallel_ordered_match.h:88-112) and SArray::setUnion /
//    setIntersection / findRange (src/util/shared_array_inl.h:150-176).
//  * BloomFilter / BlockBloomFilter (src/util/bloom_filter.h,
//    block_bloom_filter.h) with the Sketch hash (src/util/sketch.h:20-31).
// Here the match splits dst into equal contiguous pieces, one per worker
// thread, each finding its src start with one lower_bound (no recursion); the
// per-key value is a row of `k` elements (KVVector's k-values-per-key layout).
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <exception>
#include <mutex>
#include <type_traits>
#include <stdexcept>
#include <thread>
#include <vector>

#include "cpu_kernels.h"
#include "module_parts.h"

namespace py = pybind11;

namespace pscore {

namespace {

enum MatchOp : int { kAssign = 0, kPlus = 1, kOr = 2, kMinus = 3 };

template <typename V>
inline void apply(int op, const V* s, V* d, int k) {
  switch (op) {
    case kAssign: for (int j = 0; j < k; ++j) d[j] = s[j]; break;
    case kPlus: for (int j = 0; j < k; ++j) d[j] += s[j]; break;
    case kMinus: for (int j = 0; j < k; ++j) d[j] -= s[j]; break;
    case kOr:
      if constexpr (std::is_integral<V>::value) {
        for (int j = 0; j < k; ++j) d[j] |= s[j];
        break;
      }
      throw std::invalid_argument("ordered_match: OR needs an integer value type");
    default: throw std::invalid_argument("ordered_match: unknown op");
  }
}

template <typename V>
int64_t match_range(const uint64_t* sk, int64_t ns, const V* sv, const uint64_t* dk, int64_t d0,
                    int64_t d1, V* dv, int k, int op) {
  if (d0 >= d1 || ns == 0) return 0;
  int64_t i = std::lower_bound(sk, sk + ns, dk[d0]) - sk, j = d0, n = 0;
  while (i < ns && j < d1) {
    if (sk[i] < dk[j]) {
      ++i;
    } else {
      if (sk[i] == dk[j]) {
        apply(op, sv + i * k, dv + j * k, k);
        ++i;
        ++n;
      }
      ++j;
    }
  }
  return n;
}

template <typename V>
int64_t ordered_match_t(const uint64_t* sk, int64_t ns, const V* sv, const uint64_t* dk, int64_t nd,
                        V* dv, int k, int op, int nthreads) {
  if (nd == 0 || ns == 0) return 0;
  // Only the part of dst inside [src.front, src.back] can match (reference findRange).
  const int64_t lo = std::lower_bound(dk, dk + nd, sk[0]) - dk;
  const int64_t hi = std::upper_bound(dk, dk + nd, sk[ns - 1]) - dk;
  const int64_t len = hi - lo;
  const int64_t grain = 1 << 16;
  int t = (int)std::min<int64_t>(std::max(1, nthreads), (len + grain - 1) / grain);
  if (t <= 1) return match_range(sk, ns, sv, dk, lo, hi, dv, k, op);
  std::vector<int64_t> cnt(t, 0);
  std::vector<std::thread> th;
  std::exception_ptr err;
  std::mutex err_mu;
  for (int p = 0; p < t; ++p) {
    th.emplace_back([&, p] {
      try {
        const int64_t a = lo + len * p / t, b = lo + len * (p + 1) / t;
        cnt[p] = match_range(sk, ns, sv, dk, a, b, dv, k, op);
      } catch (...) {
        std::lock_guard<std::mutex> g(err_mu);
        err = std::current_exception();
      }
    });
  }
  for (auto& x : th) x.join();
  if (err) std::rethrow_exception(err);
  int64_t n = 0;
  for (auto c : cnt) n += c;
  return n;
}

// Returns the number of keys written (out must hold na + nb).
int64_t set_union(const uint64_t* a, int64_t na, const uint64_t* b, int64_t nb, uint64_t* out) {
  return std::set_union(a, a + na, b, b + nb, out) - out;
}
int64_t set_intersection(const uint64_t* a, int64_t na, const uint64_t* b, int64_t nb,
                         uint64_t* out) {
  return std::set_intersection(a, a + na, b, b + nb, out) - out;
}

// ------------------------------------------------------------------ bloom filters
// m bits, k probes; double hashing with the rotate-by-17 delta of the reference.
void bloom_insert(uint8_t* bits, uint64_t m, int k, const uint64_t* keys, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    uint32_t h = sketch_hash(keys[i]);
    const uint32_t delta = (h >> 17) | (h << 15);
    for (int j = 0; j < k; ++j) {
      const uint64_t pos = h % m;
      bits[pos >> 3] |= (uint8_t)(1u << (pos & 7));
      h += delta;
    }
  }
}
void bloom_query(const uint8_t* bits, uint64_t m, int k, const uint64_t* keys, int64_t n,
                 uint8_t* out) {
  for (int64_t i = 0; i < n; ++i) {
    uint32_t h = sketch_hash(keys[i]);
    const uint32_t delta = (h >> 17) | (h << 15);
    uint8_t hit = 1;
    for (int j = 0; j < k && hit; ++j) {
      const uint64_t pos = h % m;
      hit = (bits[pos >> 3] >> (pos & 7)) & 1;
      h += delta;
    }
    out[i] = hit;
  }
}
// Block variant: all k probes of a key land in one `bin_bytes` block (one cache line).
void block_bloom_insert(uint8_t* data, uint64_t nbin, int bin_bytes, int k, const uint64_t* keys,
                        int64_t n) {
  const uint32_t bin_bits = (uint32_t)bin_bytes * 8;
  for (int64_t i = 0; i < n; ++i) {
    uint32_t h = sketch_hash(keys[i]);
    const uint32_t delta = (h >> 17) | (h << 15);
    uint8_t* blk = data + (h % nbin) * bin_bytes;
    for (int j = 0; j < k; ++j) {
      const uint32_t pos = h % bin_bits;
      blk[pos >> 3] |= (uint8_t)(1u << (pos & 7));
      h += delta;
    }
  }
}
void block_bloom_query(const uint8_t* data, uint64_t nbin, int bin_bytes, int k,
                       const uint64_t* keys, int64_t n, uint8_t* out) {
  const uint32_t bin_bits = (uint32_t)bin_bytes * 8;
  for (int64_t i = 0; i < n; ++i) {
    uint32_t h = sketch_hash(keys[i]);
    const uint32_t delta = (h >> 17) | (h << 15);
    const uint8_t* blk = data + (h % nbin) * bin_bytes;
    uint8_t hit = 1;
    for (int j = 0; j < k && hit; ++j) {
      const uint32_t pos = h % bin_bits;
      hit = (blk[pos >> 3] >> (pos & 7)) & 1;
      h += delta;
    }
    out[i] = hit;
  }
}

template <typename T>
T* P(uintptr_t a) { return reinterpret_cast<T*>(a); }

}  // namespace

void register_setops(py::module_& m) {
  // vtype: 0 f32, 1 f64, 2 i32, 3 i64, 4 u8
  m.def("ordered_match", [](uintptr_t sk, int64_t ns, uintptr_t sv, uintptr_t dk, int64_t nd,
                            uintptr_t dv, int k, int vtype, int op, int nthreads) {
    if (k < 1) throw std::invalid_argument("ordered_match: k >= 1");
    py::gil_scoped_release nogil;
    const uint64_t* s = P<const uint64_t>(sk);
    const uint64_t* d = P<const uint64_t>(dk);
    switch (vtype) {
      case 0: return ordered_match_t(s, ns, P<const float>(sv), d, nd, P<float>(dv), k, op, nthreads);
      case 1: return ordered_match_t(s, ns, P<const double>(sv), d, nd, P<double>(dv), k, op, nthreads);
      case 2: return ordered_match_t(s, ns, P<const int32_t>(sv), d, nd, P<int32_t>(dv), k, op, nthreads);
      case 3: return ordered_match_t(s, ns, P<const int64_t>(sv), d, nd, P<int64_t>(dv), k, op, nthreads);
      case 4: return ordered_match_t(s, ns, P<const uint8_t>(sv), d, nd, P<uint8_t>(dv), k, op, nthreads);
      default: throw std::invalid_argument("ordered_match: unsupported value type");
    }
  });
  m.def("set_union", [](uintptr_t a, int64_t na, uintptr_t b, int64_t nb, uintptr_t out) {
    py::gil_scoped_release nogil;
    return set_union(P<const uint64_t>(a), na, P<const uint64_t>(b), nb, P<uint64_t>(out));
  });
  m.def("set_intersection", [](uintptr_t a, int64_t na, uintptr_t b, int64_t nb, uintptr_t out) {
    py::gil_scoped_release nogil;
    return set_intersection(P<const uint64_t>(a), na, P<const uint64_t>(b), nb, P<uint64_t>(out));
  });
  m.def("bloom_insert", [](uintptr_t bits, uint64_t mbits, int k, uintptr_t keys, int64_t n) {
    if (mbits == 0) throw std::invalid_argument("bloom: m > 0");
    bloom_insert(P<uint8_t>(bits), mbits, k, P<const uint64_t>(keys), n);
  });
  m.def("bloom_query", [](uintptr_t bits, uint64_t mbits, int k, uintptr_t keys, int64_t n,
                          uintptr_t out) {
    if (mbits == 0) throw std::invalid_argument("bloom: m > 0");
    bloom_query(P<const uint8_t>(bits), mbits, k, P<const uint64_t>(keys), n, P<uint8_t>(out));
  });
  m.def("block_bloom_insert", [](uintptr_t data, uint64_t nbin, int bin_bytes, int k,
                                 uintptr_t keys, int64_t n) {
    if (nbin == 0 || bin_bytes <= 0) throw std::invalid_argument("block bloom: empty");
    block_bloom_insert(P<uint8_t>(data), nbin, bin_bytes, k, P<const uint64_t>(keys), n);
  });
  m.def("block_bloom_query", [](uintptr_t data, uint64_t nbin, int bin_bytes, int k,
                                uintptr_t keys, int64_t n, uintptr_t out) {
    if (nbin == 0 || bin_bytes <= 0) throw std::invalid_argument("block bloom: empty");
    block_bloom_query(P<const uint8_t>(data), nbin, bin_bytes, k, P<const uint64_t>(keys), n,
                      P<uint8_t>(out));
  });
}

}  // namespace pscore
