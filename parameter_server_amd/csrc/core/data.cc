#include "data.h"

#include <dirent.h>
#include <zlib.h>

#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <thread>
#include <unordered_map>

#include "hashing.h"

namespace pscore {

namespace {

// Separator sets as 256-entry tables (one load per character; strchr per character
// was a third of the LIBSVM parse time).
struct Seps {
  bool t[256] = {};
  explicit Seps(const char* s) {
    for (; *s; ++s) t[(unsigned char)*s] = true;
  }
  bool operator()(char c) const { return t[(unsigned char)c]; }
};
const Seps kWs(" \t\r");
const Seps kWsColon(" :\t\r");

inline const Seps& seps_of(const char* s) { return s[1] == ':' ? kWsColon : kWs; }

// Next token in [p, e) delimited by any char of seps; advances p.
inline bool next_tok(const char*& p, const char* e, const Seps& sep, const char*& tb,
                     const char*& te) {
  while (p < e && sep(*p)) ++p;
  if (p >= e) return false;
  tb = p;
  while (p < e && !sep(*p)) ++p;
  te = p;
  return true;
}
inline bool next_tok(const char*& p, const char* e, const char* seps, const char*& tb,
                     const char*& te) {
  return next_tok(p, e, seps_of(seps), tb, te);
}

inline bool to_u64(const char* b, const char* e, uint64_t* v) {
  auto r = std::from_chars(b, e, *v);
  return r.ec == std::errc() && r.ptr == e;
}
inline bool to_i64(const char* b, const char* e, int64_t* v) {
  if (b < e && *b == '+') ++b;
  auto r = std::from_chars(b, e, *v);
  return r.ec == std::errc() && r.ptr == e;
}
inline bool to_f32(const char* b, const char* e, float* v) {
  if (b < e && *b == '+') ++b;
  auto r = std::from_chars(b, e, *v);
  return r.ec == std::errc() && r.ptr == e;
}

inline uint64_t fmix(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33;
  return k;
}

struct Checkpoint {
  size_t labels, row_ptr, keys, vals, slots;
};

// Per-line example sink of one parse_range (reused for every line: no allocation per
// line). Slot statistics go to a flat per-slot array (slot ids < kDenseSlots; a map
// above), merged into the batch's info map once at the end.
class LineSink {
 public:
  static constexpr int kDenseSlots = 4096;
  // mod: every key reduced mod it (the hashing trick, any format; 0 = raw keys)
  explicit LineSink(ParsedBatch* b, uint64_t mod = 0) : b_(b), mod_(mod) {}
  ~LineSink() { flush_info(); }
  void begin() {
    cp_ = {b_->labels.size(), b_->row_ptr.size(), b_->keys.size(), b_->vals.size(),
           b_->slots.size()};
    any_val_ = false;
    nline_ = 0;
  }
  void label(float y) { b_->labels.push_back(y); }
  void add(int slot, uint64_t key, float val, bool has_val) {
    if (mod_) key %= mod_;
    b_->keys.push_back(key);
    b_->vals.push_back(val);
    b_->slots.push_back(slot);
    // (explicit values of exactly 1 -- one-hot "k:1" LIBSVM rows -- are binary features)
    if (has_val && val != 1.f) any_val_ = true;
    SlotStat& s = line_slot(slot);
    s.min_key = std::min(s.min_key, key);
    s.max_key = std::max(s.max_key, key);
    s.nnz_ele++;
    s.format = has_val ? (s.format == 1 ? 1 : 2) : 3;
  }
  void dense_slot(int slot) { line_slot(slot).format = 1; }
  bool commit() {
    b_->row_ptr.push_back((int64_t)b_->keys.size());
    if (any_val_) b_->binary = false;
    for (int i = 0; i < nline_; ++i) {
      const SlotStat& s = lst_[i];
      SlotStat& t = info_of(lid_[i]);
      t.min_key = std::min(t.min_key, s.min_key);
      t.max_key = std::max(t.max_key, s.max_key);
      t.nnz_ele += s.nnz_ele;
      t.nnz_ex += s.nnz_ele > 0;
      if (s.format) t.format = s.format;
    }
    return true;
  }
  bool rollback() {
    b_->labels.resize(cp_.labels);
    b_->row_ptr.resize(cp_.row_ptr);
    b_->keys.resize(cp_.keys);
    b_->vals.resize(cp_.vals);
    b_->slots.resize(cp_.slots);
    b_->bad_lines++;
    return false;
  }

 private:
  // this line's slots (few: a linear scan over the ids seen so far on the line)
  SlotStat& line_slot(int slot) {
    for (int i = nline_ - 1; i >= 0; --i)
      if (lid_[i] == slot) return lst_[i];
    if (nline_ == (int)lid_.size()) {
      lid_.resize(lid_.size() * 2 + 8);
      lst_.resize(lst_.size() * 2 + 8);
    }
    lid_[nline_] = slot;
    lst_[nline_] = SlotStat{};
    return lst_[nline_++];
  }
  SlotStat& info_of(int id) {
    if (id >= 0 && id < kDenseSlots) {
      if (dense_.empty()) {
        dense_.resize(kDenseSlots);
        dense_seen_.assign(kDenseSlots, 0);
      }
      dense_seen_[id] = 1;
      return dense_[id];
    }
    return sparse_[id];
  }
  void flush_info() {
    for (int id = 0; id < (int)dense_seen_.size(); ++id)
      if (dense_seen_[id]) merge(b_->info[id], dense_[id]);
    for (auto& [id, s] : sparse_) merge(b_->info[id], s);
  }
  static void merge(SlotStat& t, const SlotStat& s) {
    t.min_key = std::min(t.min_key, s.min_key);
    t.max_key = std::max(t.max_key, s.max_key);
    t.nnz_ele += s.nnz_ele;
    t.nnz_ex += s.nnz_ex;
    if (s.format) t.format = s.format;
  }

  ParsedBatch* b_;
  uint64_t mod_ = 0;
  Checkpoint cp_{};
  bool any_val_ = false;
  int nline_ = 0;
  std::vector<int> lid_;
  std::vector<SlotStat> lst_;
  std::vector<SlotStat> dense_;
  std::vector<char> dense_seen_;
  std::map<int, SlotStat> sparse_;
};

bool parse_libsvm(const char* p, const char* e, const ParseOptions&, LineSink& s) {
  const char *tb, *te;
  if (!next_tok(p, e, " \t\r", tb, te)) return false;
  float y;
  if (!to_f32(tb, te, &y)) return false;
  s.label(y);
  uint64_t last = 0;
  while (next_tok(p, e, " \t\r", tb, te)) {
    const char* c = std::find(tb, te, ':');
    if (c == te) return false;
    uint64_t idx;
    float v = 1.f;
    if (!to_u64(tb, c, &idx)) return false;
    if (!(te - c == 2 && c[1] == '1') && !to_f32(c + 1, te, &v)) return false;  // ("k:1" fast)
    if (idx < last) return false;  // reference requires non-decreasing indices
    last = idx;
    s.add(1, idx, v, true);
  }
  return true;
}

bool parse_adfea(const char* p, const char* e, const ParseOptions& opt, LineSink& s) {
  // lineid 1 click key:grp key:grp ...
  const char *tb, *te;
  uint64_t key = 0;
  for (int i = 0; next_tok(p, e, " :\t\r", tb, te); ++i) {
    if (i < 2) continue;
    if (i == 2) {
      int64_t c;
      if (!to_i64(tb, te, &c)) return false;
      s.label(c > 0 ? 1.f : -1.f);
    } else if (i % 2 == 1) {
      if (!to_u64(tb, te, &key)) return false;
    } else {
      int64_t g = 1;
      if (!opt.ignore_fea_slot && !to_i64(tb, te, &g)) return false;
      s.add((int)g, key, 1.f, false);
    }
  }
  return true;
}

bool parse_terafea(const char* p, const char* e, const ParseOptions& opt, LineSink& s) {
  // click lineid | key key key ...   (group id = top 10 bits of the key)
  const char *tb, *te;
  for (int i = 0; next_tok(p, e, " \t\r", tb, te); ++i) {
    if (i == 0) {
      int64_t c;
      if (!to_i64(tb, te, &c)) return false;
      s.label(c > 0 ? 1.f : -1.f);
    } else if (i >= 3) {
      uint64_t key;
      if (!to_u64(tb, te, &key)) return false;
      const int g = opt.ignore_fea_slot ? 1 : (int)(key >> 54);
      uint64_t fea = key;
      if (opt.shuffle_fea_id) {
        uint64_t out[2];
        murmur3_x64_128(&fea, 8, 512927377u, out);
        fea = out[0] ^ out[1];
      }
      s.add(g, fea, 1.f, false);
    }
  }
  return true;
}

bool parse_ps(const char* p, const char* e, const ParseOptions& opt, LineSink& s) {
  // label; grp f f f; grp f:w f:w; ...
  const char* q = std::find(p, e, ';');
  int64_t label;
  {
    const char *tb, *te, *pp = p;
    if (!next_tok(pp, q, " \t\r", tb, te) || !to_i64(tb, te, &label)) return false;
  }
  s.label(label > 0 ? 1.f : -1.f);
  p = q;
  int slot_id = -1;
  while (p < e) {
    ++p;  // skip ';'
    const char* ge = std::find(p, e, ';');
    const char *tb, *te, *gp = p;
    if (!next_tok(gp, ge, " \t\r", tb, te)) { p = ge; continue; }
    if (!opt.ignore_fea_slot) {
      int64_t sid;
      if (!to_i64(tb, te, &sid)) return false;
      slot_id = (int)sid;
    } else {
      slot_id = 1;
    }
    if (opt.format == TextFormat::DENSE) s.dense_slot(slot_id);
    uint64_t pending_key = 0, dense_idx = 0;
    for (int i = 0; next_tok(gp, ge, " :\t\r", tb, te); ++i) {
      if (opt.format == TextFormat::DENSE) {
        float v;
        if (!to_f32(tb, te, &v)) return false;
        s.add(slot_id, dense_idx++, v, true);
      } else if (opt.format == TextFormat::SPARSE && (i % 2 == 1)) {
        float v;
        if (!to_f32(tb, te, &v)) return false;
        s.add(slot_id, pending_key, v, true);
      } else {
        uint64_t k;
        if (!to_u64(tb, te, &k)) return false;
        if (opt.format == TextFormat::SPARSE) pending_key = k;
        else s.add(slot_id, k, 1.f, false);
      }
    }
    p = ge;
  }
  return true;
}

bool parse_criteo(const char* p, const char* e, const ParseOptions& opt, LineSink& s) {
  // label \t I1..I13 \t C1..C26 (empty fields allowed)
  int field = 0;
  while (p <= e && field < 40) {
    const char* fe = std::find(p, e, '\t');
    const char* te = fe;
    while (te > p && (te[-1] == '\r' || te[-1] == ' ')) --te;
    if (field == 0) {
      int64_t c;
      if (!to_i64(p, te, &c)) return false;
      s.label(c > 0 ? 1.f : -1.f);
    } else if (te > p) {
      const int j = field - 1;  // slot 0..38
      uint64_t id;
      if (j < 13) {
        int64_t v;
        if (!to_i64(p, te, &v)) return false;
        id = v <= 0 ? 0 : (uint64_t)(2.0 * std::log2(1.0 + (double)v));
      } else {
        uint64_t v;
        auto r = std::from_chars(p, te, v, 16);
        if (r.ec != std::errc() || r.ptr != te) return false;
        id = v;
      }
      const uint64_t key = fmix(((uint64_t)(j + 1) << 48) ^ id);  // (mod in the sink)
      s.add(opt.ignore_fea_slot ? 1 : j + 1, key, 1.f, false);
    }
    ++field;
    if (fe >= e) break;
    p = fe + 1;
  }
  return field >= 1;
}

}  // namespace

void ParsedBatch::append(ParsedBatch&& o) {
  const int64_t base = (int64_t)keys.size();
  labels.insert(labels.end(), o.labels.begin(), o.labels.end());
  for (size_t i = 1; i < o.row_ptr.size(); ++i) row_ptr.push_back(o.row_ptr[i] + base);
  keys.insert(keys.end(), o.keys.begin(), o.keys.end());
  vals.insert(vals.end(), o.vals.begin(), o.vals.end());
  slots.insert(slots.end(), o.slots.begin(), o.slots.end());
  binary = binary && o.binary;
  bad_lines += o.bad_lines;
  for (auto& [id, s] : o.info) {
    auto& t = info[id];
    t.min_key = std::min(t.min_key, s.min_key);
    t.max_key = std::max(t.max_key, s.max_key);
    t.nnz_ele += s.nnz_ele;
    t.nnz_ex += s.nnz_ex;
    if (s.format) t.format = s.format;
  }
}

static bool parse_line_into(const char* b, const char* e, const ParseOptions& opt, LineSink& s) {
  while (e > b && (e[-1] == '\n' || e[-1] == '\r')) --e;
  s.begin();
  bool ok;
  switch (opt.format) {
    case TextFormat::LIBSVM: ok = parse_libsvm(b, e, opt, s); break;
    case TextFormat::ADFEA: ok = parse_adfea(b, e, opt, s); break;
    case TextFormat::TERAFEA: ok = parse_terafea(b, e, opt, s); break;
    case TextFormat::DENSE:
    case TextFormat::SPARSE:
    case TextFormat::SPARSE_BINARY: ok = parse_ps(b, e, opt, s); break;
    case TextFormat::CRITEO: ok = parse_criteo(b, e, opt, s); break;
    default: throw std::invalid_argument("unsupported text format (VW is not implemented)");
  }
  return ok ? s.commit() : s.rollback();
}

bool parse_line(const char* b, const char* e, const ParseOptions& opt, ParsedBatch* out) {
  LineSink s(out, opt.hash_mod);
  return parse_line_into(b, e, opt, s);
}

static ParsedBatch parse_range(const char* p, const char* e, const ParseOptions& opt,
                               int64_t max_lines) {
  ParsedBatch out;
  // (reserve from the byte count: a binary feature is >= 4 bytes of text)
  const size_t guess = (size_t)(e - p) / 8;
  out.keys.reserve(guess);
  out.vals.reserve(guess);
  out.slots.reserve(guess);
  {
    LineSink s(&out, opt.hash_mod);
    int64_t n = 0;
    while (p < e && (max_lines < 0 || n < max_lines)) {
      const char* le = (const char*)std::memchr(p, '\n', e - p);
      if (!le) le = e;
      const char* q = p;
      while (q < le && (*q == ' ' || *q == '\t' || *q == '\r')) ++q;
      if (q < le && *q != '#') {
        parse_line_into(p, le, opt, s);
        ++n;
      }
      p = le + 1;
    }
  }  // (the sink merges its slot statistics into out.info here)
  return out;
}

ParsedBatch parse_buffer(const char* data, size_t len, const ParseOptions& opt) {
  const int T = std::max(1, opt.nthreads);
  if (T == 1 || len < (1u << 20) || opt.max_lines >= 0)
    return parse_range(data, data + len, opt, opt.max_lines);
  std::vector<const char*> cuts{data};
  for (int t = 1; t < T; ++t) {
    const char* c = data + len * t / T;
    if (c < cuts.back()) c = cuts.back();
    const char* nl = (const char*)std::memchr(c, '\n', data + len - c);
    cuts.push_back(nl ? nl + 1 : data + len);
  }
  cuts.push_back(data + len);
  std::vector<ParsedBatch> parts(T);
  std::vector<std::thread> th;
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] { parts[t] = parse_range(cuts[t], cuts[t + 1], opt, -1); });
  for (auto& x : th) x.join();
  // concatenate in parallel: every part copies itself into its slice of the output
  std::vector<size_t> r0(T + 1, 0), k0(T + 1, 0);
  for (int t = 0; t < T; ++t) {
    r0[t + 1] = r0[t] + parts[t].labels.size();
    k0[t + 1] = k0[t] + parts[t].keys.size();
  }
  ParsedBatch out;
  out.labels.resize(r0[T]);
  out.row_ptr.resize(r0[T] + 1);
  out.row_ptr[0] = 0;
  out.keys.resize(k0[T]);
  out.vals.resize(k0[T]);
  out.slots.resize(k0[T]);
  th.clear();
  for (int t = 0; t < T; ++t)
    th.emplace_back([&, t] {
      const ParsedBatch& q = parts[t];
      std::copy(q.labels.begin(), q.labels.end(), out.labels.begin() + r0[t]);
      for (size_t i = 1; i < q.row_ptr.size(); ++i)
        out.row_ptr[r0[t] + i] = q.row_ptr[i] + (int64_t)k0[t];
      std::copy(q.keys.begin(), q.keys.end(), out.keys.begin() + k0[t]);
      std::copy(q.vals.begin(), q.vals.end(), out.vals.begin() + k0[t]);
      std::copy(q.slots.begin(), q.slots.end(), out.slots.begin() + k0[t]);
    });
  for (auto& x : th) x.join();
  for (int t = 0; t < T; ++t) {
    out.binary = out.binary && parts[t].binary;
    out.bad_lines += parts[t].bad_lines;
    for (auto& [id, st] : parts[t].info) {
      auto& d = out.info[id];
      d.min_key = std::min(d.min_key, st.min_key);
      d.max_key = std::max(d.max_key, st.max_key);
      d.nnz_ele += st.nnz_ele;
      d.nnz_ex += st.nnz_ex;
      if (st.format) d.format = st.format;
    }
  }
  return out;
}

// ------------------------------------------------------------------- files
static std::string popen_read(const std::string& cmd) {
  FILE* f = popen(cmd.c_str(), "r");
  if (!f) throw std::runtime_error("popen failed: " + cmd);
  std::string out;
  char buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof(buf), f)) > 0) out.append(buf, n);
  if (pclose(f) != 0) throw std::runtime_error("command failed: " + cmd);
  return out;
}

static bool ends_with(const std::string& s, const std::string& suf) {
  return s.size() >= suf.size() && s.compare(s.size() - suf.size(), suf.size(), suf) == 0;
}

static std::string hadoop_bin(const std::string& home) {
  return (home.empty() ? std::string("hadoop") : home + "/bin/hadoop");
}

std::string read_file(const std::string& path, const std::string& hadoop_home) {
  std::string raw;
  if (path.rfind("hdfs://", 0) == 0 || !hadoop_home.empty()) {
    raw = popen_read(hadoop_bin(hadoop_home) + " fs -cat '" + path + "'");
    if (!ends_with(path, ".gz")) return raw;
  }
  if (ends_with(path, ".gz")) {
    gzFile g = raw.empty() ? gzopen(path.c_str(), "rb") : nullptr;
    std::string out;
    if (g) {
      char buf[1 << 16];
      int n;
      while ((n = gzread(g, buf, sizeof(buf))) > 0) out.append(buf, n);
      gzclose(g);
      return out;
    }
    if (raw.empty()) throw std::runtime_error("cannot open " + path);
    // inflate an in-memory gzip stream (HDFS case)
    z_stream zs{};
    inflateInit2(&zs, 16 + MAX_WBITS);
    zs.next_in = (Bytef*)raw.data();
    zs.avail_in = raw.size();
    char buf[1 << 16];
    int rc;
    do {
      zs.next_out = (Bytef*)buf;
      zs.avail_out = sizeof(buf);
      rc = inflate(&zs, Z_NO_FLUSH);
      out.append(buf, sizeof(buf) - zs.avail_out);
    } while (rc == Z_OK);
    inflateEnd(&zs);
    return out;
  }
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("cannot open " + path);
  std::string out;
  char buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof(buf), f)) > 0) out.append(buf, n);
  fclose(f);
  return out;
}

void write_file(const std::string& path, const std::string& data, bool gzip) {
  if (gzip || ends_with(path, ".gz")) {
    gzFile g = gzopen(path.c_str(), "wb");
    if (!g) throw std::runtime_error("cannot write " + path);
    gzwrite(g, data.data(), (unsigned)data.size());
    gzclose(g);
    return;
  }
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("cannot write " + path);
  fwrite(data.data(), 1, data.size(), f);
  fclose(f);
}

std::vector<std::string> list_dir(const std::string& dir, const std::string& hadoop_home) {
  std::vector<std::string> out;
  if (dir.rfind("hdfs://", 0) == 0 || !hadoop_home.empty()) {
    std::string ls = popen_read(hadoop_bin(hadoop_home) + " fs -ls '" + dir + "'");
    size_t p = 0;
    while (p < ls.size()) {
      size_t e = ls.find('\n', p);
      if (e == std::string::npos) e = ls.size();
      std::string line = ls.substr(p, e - p);
      size_t sp = line.rfind(' ');
      if (!line.empty() && line[0] != 'F' && sp != std::string::npos) {
        std::string f = line.substr(sp + 1);
        size_t sl = f.rfind('/');
        out.push_back(sl == std::string::npos ? f : f.substr(sl + 1));
      }
      p = e + 1;
    }
    return out;
  }
  DIR* d = opendir(dir.empty() ? "." : dir.c_str());
  if (!d) return out;
  while (dirent* ent = readdir(d)) {
    std::string n = ent->d_name;
    if (n != "." && n != "..") out.push_back(n);
  }
  closedir(d);
  std::sort(out.begin(), out.end());
  return out;
}

std::string recordio_pack(const std::vector<std::string>& records) {
  std::string out;
  for (const auto& r : records) {
    uint32_t hdr[2] = {kRecordIOMagic, (uint32_t)r.size()};
    out.append((const char*)hdr, 8);
    out.append(r);
    out.append((4 - r.size() % 4) % 4, '\0');
  }
  return out;
}

std::vector<std::string> recordio_unpack(const std::string& data) {
  std::vector<std::string> out;
  size_t p = 0;
  while (p + 8 <= data.size()) {
    uint32_t hdr[2];
    std::memcpy(hdr, data.data() + p, 8);
    if (hdr[0] != kRecordIOMagic) throw std::runtime_error("recordio: bad magic");
    p += 8;
    if (p + hdr[1] > data.size()) throw std::runtime_error("recordio: truncated record");
    out.emplace_back(data.data() + p, hdr[1]);
    p += hdr[1] + (4 - hdr[1] % 4) % 4;
  }
  return out;
}

}  // namespace pscore
