// Host-side race / memory-error test for the native runtime (no GPU involved).
//
// The reference's race-detection story is building with -fsanitize (its
// Makefile/CMake `-fsanitize=address` knobs) and running the multi-threaded
// control plane under it. Here the same native sources that make up `_pscore`
// (runtime.cc, textproto.cc, data.cc, hashing.cc) are compiled WITHOUT the
// pybind layer (PSAMD_CORE_STANDALONE) into one binary and driven from many
// threads: tests/test_native_sanitizers.py builds it with -fsanitize=thread and
// with -fsanitize=address,undefined and requires a clean exit.
//
//   - Van: two loopback endpoints, 4 sender threads per side + concurrent
//     receivers; every multi-frame message is checked byte for byte.
//   - TaskTracker: concurrent start/finish with waiters blocked on timestamps.
//   - textproto: parse -> print -> parse round trip from several threads.
//   - data: multi-threaded LIBSVM/CRITEO buffer parsing vs single-threaded.
//   - crc32c: known-answer vector, concurrent use.
#define PSAMD_CORE_STANDALONE 1
#include "runtime.cc"
#include "textproto.cc"
#include "data.cc"
#include "hashing.cc"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <thread>

using namespace pscore;

static int g_fail = 0;
#define CHECK(cond)                                                          \
  do {                                                                       \
    if (!(cond)) {                                                           \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_fail;                                                              \
    }                                                                        \
  } while (0)

static std::string payload(int sender, int i, int frame) {
  std::string s = std::to_string(sender) + ":" + std::to_string(i) + ":" + std::to_string(frame) + ":";
  s.append((size_t)((i * 37 + frame * 11) % 2000), (char)('a' + (i + frame) % 26));
  return s;
}

static void test_van() {
  constexpr int kThreads = 4, kMsgs = 300;
  Van a("A"), b("B");
  int pa = a.bind("127.0.0.1", 0), pb = b.bind("127.0.0.1", 0);
  CHECK(pa > 0 && pb > 0);
  a.connect("B", "127.0.0.1", pb);
  b.connect("A", "127.0.0.1", pa);

  auto receiver = [&](Van* v, const char* from, std::atomic<int>* got) {
    Received r;
    while (got->load() < kThreads * kMsgs) {
      if (!v->recv(&r, 5.0)) { CHECK(false && "recv timeout"); return; }
      CHECK(r.sender == from);
      CHECK(r.frames.size() == 3);
      if (r.frames.size() != 3) continue;
      int s = 0, i = 0;
      CHECK(std::sscanf(r.frames[0].c_str(), "%d:%d:", &s, &i) == 2);
      for (int f = 0; f < 3; ++f) CHECK(r.frames[f] == payload(s, i, f));
      got->fetch_add(1);
    }
  };
  std::atomic<int> got_a{0}, got_b{0};
  std::thread ra(receiver, &a, "B", &got_a), rb(receiver, &b, "A", &got_b);
  std::vector<std::thread> senders;
  for (int t = 0; t < kThreads; ++t) {
    for (int side = 0; side < 2; ++side) {
      senders.emplace_back([&, t, side] {
        Van& v = side ? b : a;
        const char* to = side ? "A" : "B";
        for (int i = 0; i < kMsgs; ++i) {
          std::string f0 = payload(t, i, 0), f1 = payload(t, i, 1), f2 = payload(t, i, 2);
          std::vector<std::pair<const char*, size_t>> frames = {
              {f0.data(), f0.size()}, {f1.data(), f1.size()}, {f2.data(), f2.size()}};
          CHECK(v.send(to, frames) > 0);
        }
      });
    }
  }
  for (auto& s : senders) s.join();
  ra.join();
  rb.join();
  CHECK(got_a.load() == kThreads * kMsgs);
  CHECK(got_b.load() == kThreads * kMsgs);
  // local short-circuit queue + stop() racing a blocked receiver
  std::thread blocked([&] { Received r; a.recv(&r, -1); });
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  a.stop();
  blocked.join();
  b.stop();
}

static void test_tracker() {
  TaskTracker tr;
  constexpr int kN = 2000, kThreads = 4;
  std::vector<std::thread> th;
  std::atomic<int> waited{0};
  for (int w = 0; w < 2; ++w)
    th.emplace_back([&, w] {
      for (int t = w; t < kN; t += 97) {
        if (tr.wait(t, 10.0)) waited.fetch_add(1);
      }
    });
  for (int k = 0; k < kThreads; ++k)
    th.emplace_back([&, k] {
      for (int t = k; t < kN; t += kThreads) {
        tr.start(t);
        tr.finish(t);
      }
    });
  for (auto& t : th) t.join();
  CHECK(tr.all_finished(0, kN - 1));
  CHECK(waited.load() > 0);
  tr.clear_below(kN / 2);
  CHECK(tr.has_finished(kN - 1));
}

static void test_textproto() {
  const std::string src =
      "app_name: \"ctr\" # comment\n"
      "linear_method { loss { type: LOGIT } penalty { type: L1 lambda: 1 lambda: .1 }\n"
      "  darlin { max_block_delay: 4 [PS.LM.delta_init_value]: 1e-2 }\n"
      "  training_data < format: TEXT text: LIBSVM file: 'a' \"b\\n\" > }\n";
  std::vector<std::thread> th;
  for (int k = 0; k < 4; ++k)
    th.emplace_back([&] {
      for (int i = 0; i < 50; ++i) {
        TPMessage m = parse_textproto(src);
        std::string p = print_textproto(m);
        CHECK(print_textproto(parse_textproto(p)) == p);
      }
    });
  for (auto& t : th) t.join();
  bool threw = false;
  try { parse_textproto("a { b: 1"); } catch (const TextProtoError&) { threw = true; }
  CHECK(threw);
}

static void test_data() {
  std::string text;
  for (int r = 0; r < 5000; ++r) {
    text += (r % 3 ? "1" : "-1");
    for (int j = 0; j < 1 + r % 13; ++j)
      text += " " + std::to_string((uint64_t)r * 7919u + (uint64_t)j * 104729u) + ":" +
              std::to_string(0.5 + j);
    text += "\n";
  }
  ParseOptions o1;
  o1.format = TextFormat::LIBSVM;
  ParseOptions o8 = o1;
  o8.nthreads = 8;
  ParsedBatch s = parse_buffer(text.data(), text.size(), o1);
  ParsedBatch p = parse_buffer(text.data(), text.size(), o8);
  CHECK(s.rows() == 5000 && p.rows() == 5000);
  CHECK(s.keys == p.keys && s.vals == p.vals && s.row_ptr == p.row_ptr && s.labels == p.labels);
  CHECK(!p.binary);
  std::string rec = recordio_pack({"x", "yy", std::string(1000, 'z')});
  auto recs = recordio_unpack(rec);
  CHECK(recs.size() == 3 && recs[2].size() == 1000);
}

static void test_crc() {
  const char* v = "123456789";
  CHECK(crc32c(v, 9) == 0xE3069283u);
  std::vector<std::thread> th;
  std::string big(1 << 16, 'q');
  uint32_t want = crc32c(big.data(), big.size());
  for (int k = 0; k < 4; ++k)
    th.emplace_back([&] {
      for (int i = 0; i < 20; ++i) CHECK(crc32c(big.data(), big.size()) == want);
    });
  for (auto& t : th) t.join();
}

int main() {
  const std::pair<const char*, void (*)()> tests[] = {
      {"crc", test_crc}, {"textproto", test_textproto}, {"data", test_data},
      {"tracker", test_tracker}, {"van", test_van}};
  for (auto& t : tests) {
    std::fprintf(stderr, "[run] %s\n", t.first);
    t.second();
  }
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("core_sanitize_test OK\n");
  return 0;
}
