// Host runtime: TCP transport ("Van"), TaskTracker, local-machine helpers.
//
// Reference Van (src/system/van.cc:20-233) binds one ZeroMQ ROUTER socket and
// opens one DEALER per peer; a message is multipart [Task proto][key][values...]
// and the receiver copies every frame. ZeroMQ is not available here, so this is a
// plain-socket equivalent: one listening socket, one outgoing connection per peer
// (lazily connected, identity handshake), one reader thread per incoming
// connection feeding a single receive queue. Frames are length prefixed and sent
// with writev straight from the caller's buffers (no staging copy).
//
// TaskTracker (src/system/task_tracker.h:11-55): thread-safe set of finished
// timestamps with blocking wait — the primitive behind every consistency model.
#include <arpa/inet.h>
#include <ifaddrs.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#ifndef PSAMD_CORE_STANDALONE  // sanitizer test builds (tests/native) include this file
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#endif
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#ifndef PSAMD_CORE_STANDALONE
#include "module_parts.h"

namespace py = pybind11;
#endif

namespace pscore {

namespace {
constexpr uint32_t kMagic = 0x50535631;  // "PSV1"

bool write_all(int fd, const struct iovec* iov, int n) {
  std::vector<struct iovec> v(iov, iov + n);
  size_t i = 0;
  while (i < v.size()) {
    const int cnt = (int)std::min<size_t>(v.size() - i, 512);
    ssize_t w = ::writev(fd, &v[i], cnt);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    size_t left = (size_t)w;
    while (i < v.size() && left >= v[i].iov_len) {
      left -= v[i].iov_len;
      ++i;
    }
    if (i < v.size() && left) {
      v[i].iov_base = (char*)v[i].iov_base + left;
      v[i].iov_len -= left;
    }
  }
  return true;
}

bool read_all(int fd, void* buf, size_t n) {
  char* p = (char*)buf;
  while (n) {
    ssize_t r = ::recv(fd, p, n, 0);
    if (r == 0) return false;
    if (r < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += r;
    n -= (size_t)r;
  }
  return true;
}

int tcp_connect(const std::string& host, int port, int retries) {
  for (int attempt = 0; attempt <= retries; ++attempt) {
    struct addrinfo hints {}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) == 0 && res) {
      int fd = ::socket(res->ai_family, res->ai_socktype, res->ai_protocol);
      if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
        freeaddrinfo(res);
        int one = 1;
        setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        return fd;
      }
      if (fd >= 0) ::close(fd);
      freeaddrinfo(res);
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(50 + 50 * std::min(attempt, 20)));
  }
  return -1;
}
}  // namespace

struct Received {
  std::string sender;
  std::vector<std::string> frames;
};

class Van {
 public:
  explicit Van(std::string my_id) : my_id_(std::move(my_id)) {}
  ~Van() { stop(); }

  int bind(const std::string& host, int port) {
    listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    if (listen_fd_ < 0) throw std::runtime_error("socket failed");
    int one = 1;
    setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in addr{};
    addr.sin_family = AF_INET;
    addr.sin_port = htons((uint16_t)port);
    addr.sin_addr.s_addr = host.empty() || host == "*" ? INADDR_ANY : inet_addr(host.c_str());
    if (::bind(listen_fd_, (sockaddr*)&addr, sizeof(addr)) != 0)
      throw std::runtime_error("bind failed on port " + std::to_string(port) + ": " + strerror(errno));
    if (::listen(listen_fd_, 256) != 0) throw std::runtime_error("listen failed");
    socklen_t len = sizeof(addr);
    getsockname(listen_fd_, (sockaddr*)&addr, &len);
    port_ = ntohs(addr.sin_port);
    running_ = true;
    accept_thread_ = std::thread([this] { accept_loop(); });
    return port_;
  }

  void connect(const std::string& node_id, const std::string& host, int port) {
    std::lock_guard<std::mutex> lk(peers_mu_);
    if (peers_.count(node_id)) return;
    int fd = tcp_connect(host, port, 100);
    if (fd < 0) throw std::runtime_error("cannot connect to " + node_id + " at " + host + ":" +
                                         std::to_string(port));
    uint32_t hdr[2] = {kMagic, (uint32_t)my_id_.size()};
    struct iovec iov[2] = {{hdr, 8}, {(void*)my_id_.data(), my_id_.size()}};
    if (!write_all(fd, iov, 2)) throw std::runtime_error("handshake failed");
    auto p = std::make_shared<Peer>();
    p->fd = fd;
    p->local = host == "127.0.0.1" || host == "localhost";
    peers_[node_id] = p;
  }

  bool connected(const std::string& node_id) {
    std::lock_guard<std::mutex> lk(peers_mu_);
    return peers_.count(node_id) > 0;
  }

  void disconnect(const std::string& node_id) {
    std::shared_ptr<Peer> p;
    {
      std::lock_guard<std::mutex> lk(peers_mu_);
      auto it = peers_.find(node_id);
      if (it == peers_.end()) return;
      p = it->second;
      peers_.erase(it);
    }
    std::lock_guard<std::mutex> lk(p->mu);
    ::shutdown(p->fd, SHUT_RDWR);
    ::close(p->fd);
  }

  // frames given as (ptr, len) views; the caller keeps them alive for the call.
  int64_t send(const std::string& node_id, const std::vector<std::pair<const char*, size_t>>& frames) {
    std::shared_ptr<Peer> p;
    {
      std::lock_guard<std::mutex> lk(peers_mu_);
      auto it = peers_.find(node_id);
      if (it == peers_.end()) throw std::runtime_error("not connected to " + node_id);
      p = it->second;
    }
    std::vector<uint64_t> lens(frames.size() + 1);
    lens[0] = ((uint64_t)kMagic << 32) | (uint64_t)frames.size();
    int64_t total = 0;
    for (size_t i = 0; i < frames.size(); ++i) {
      lens[i + 1] = frames[i].second;
      total += (int64_t)frames[i].second;
    }
    std::vector<struct iovec> iov;
    iov.push_back({lens.data(), lens.size() * sizeof(uint64_t)});
    for (auto& f : frames)
      if (f.second) iov.push_back({(void*)f.first, f.second});
    {
      std::lock_guard<std::mutex> lk(p->mu);
      if (!write_all(p->fd, iov.data(), (int)iov.size()))
        throw std::runtime_error("send to " + node_id + " failed");
    }
    total += (int64_t)(lens.size() * 8);
    (p->local ? sent_local_ : sent_remote_) += total;
    return total;
  }

  bool recv(Received* out, double timeout) {
    std::unique_lock<std::mutex> lk(q_mu_);
    auto pred = [this] { return !q_.empty() || !running_; };
    if (timeout < 0) {
      q_cv_.wait(lk, pred);
    } else if (!q_cv_.wait_for(lk, std::chrono::duration<double>(timeout), pred)) {
      return false;
    }
    if (q_.empty()) return false;
    *out = std::move(q_.front());
    q_.pop_front();
    return true;
  }

  // Inject a message into the local receive queue (local replies, loopback).
  void push_local(Received&& r) {
    {
      std::lock_guard<std::mutex> lk(q_mu_);
      q_.push_back(std::move(r));
    }
    q_cv_.notify_one();
  }

  void stop() {
    if (!running_.exchange(false)) return;
    if (listen_fd_ >= 0) {
      ::shutdown(listen_fd_, SHUT_RDWR);
      ::close(listen_fd_);
    }
    {
      std::lock_guard<std::mutex> lk(peers_mu_);
      for (auto& [id, p] : peers_) {
        ::shutdown(p->fd, SHUT_RDWR);
        ::close(p->fd);
      }
      peers_.clear();
    }
    {
      std::lock_guard<std::mutex> lk(conn_mu_);
      for (int fd : conns_) ::shutdown(fd, SHUT_RDWR);
    }
    q_cv_.notify_all();
    if (accept_thread_.joinable()) accept_thread_.join();
    for (auto& t : readers_)
      if (t.joinable()) t.join();
    std::lock_guard<std::mutex> lk(conn_mu_);
    for (int fd : conns_) ::close(fd);
    conns_.clear();
  }

  int port() const { return port_; }
  std::map<std::string, int64_t> stats() const {
    return {{"sent_local", sent_local_.load()}, {"sent_remote", sent_remote_.load()},
            {"recv_local", recv_local_.load()}, {"recv_remote", recv_remote_.load()}};
  }

 private:
  struct Peer {
    int fd = -1;
    bool local = false;
    std::mutex mu;
  };

  void accept_loop() {
    while (running_) {
      sockaddr_in cli{};
      socklen_t len = sizeof(cli);
      int fd = ::accept(listen_fd_, (sockaddr*)&cli, &len);
      if (fd < 0) {
        if (!running_) break;
        if (errno == EINTR) continue;
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
        continue;
      }
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      const bool local = cli.sin_addr.s_addr == htonl(INADDR_LOOPBACK);
      std::lock_guard<std::mutex> lk(conn_mu_);
      conns_.push_back(fd);
      readers_.emplace_back([this, fd, local] { read_loop(fd, local); });
    }
  }

  void read_loop(int fd, bool local) {
    uint32_t hdr[2];
    if (!read_all(fd, hdr, 8) || hdr[0] != kMagic || hdr[1] > 4096) return;
    std::string sender(hdr[1], '\0');
    if (!read_all(fd, sender.data(), hdr[1])) return;
    while (running_) {
      uint64_t h;
      if (!read_all(fd, &h, 8)) break;
      if ((h >> 32) != kMagic) break;
      const uint64_t n = h & 0xffffffffu;
      std::vector<uint64_t> lens(n);
      if (n && !read_all(fd, lens.data(), n * 8)) break;
      Received r;
      r.sender = sender;
      r.frames.resize(n);
      int64_t total = 8 + 8 * (int64_t)n;
      bool ok = true;
      for (uint64_t i = 0; i < n; ++i) {
        r.frames[i].resize(lens[i]);
        if (lens[i] && !read_all(fd, r.frames[i].data(), lens[i])) { ok = false; break; }
        total += (int64_t)lens[i];
      }
      if (!ok) break;
      (local ? recv_local_ : recv_remote_) += total;
      push_local(std::move(r));
    }
  }

  std::string my_id_;
  int listen_fd_ = -1, port_ = 0;
  std::atomic<bool> running_{false};
  std::thread accept_thread_;
  std::vector<std::thread> readers_;
  std::mutex conn_mu_;
  std::vector<int> conns_;
  std::mutex peers_mu_;
  std::unordered_map<std::string, std::shared_ptr<Peer>> peers_;
  std::mutex q_mu_;
  std::condition_variable q_cv_;
  std::deque<Received> q_;
  std::atomic<int64_t> sent_local_{0}, sent_remote_{0}, recv_local_{0}, recv_remote_{0};
};

class TaskTracker {
 public:
  void start(int t) {
    std::lock_guard<std::mutex> lk(mu_);
    done_.emplace(t, false);
  }
  void finish(int t) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      done_[t] = true;
    }
    cv_.notify_all();
  }
  bool has_finished(int t) {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = done_.find(t);
    return it != done_.end() && it->second;
  }
  bool wait(int t, double timeout) {
    std::unique_lock<std::mutex> lk(mu_);
    auto pred = [&] {
      auto it = done_.find(t);
      return it != done_.end() && it->second;
    };
    if (timeout < 0) {
      cv_.wait(lk, pred);
      return true;
    }
    return cv_.wait_for(lk, std::chrono::duration<double>(timeout), pred);
  }
  // all timestamps in [lo, hi] finished?
  bool all_finished(int lo, int hi) {
    std::lock_guard<std::mutex> lk(mu_);
    for (int t = lo; t <= hi; ++t) {
      auto it = done_.find(t);
      if (it == done_.end() || !it->second) return false;
    }
    return true;
  }
  void clear_below(int t) {
    std::lock_guard<std::mutex> lk(mu_);
    done_.erase(done_.begin(), done_.lower_bound(t));
  }
  size_t size() {
    std::lock_guard<std::mutex> lk(mu_);
    return done_.size();
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::map<int, bool> done_;
};

std::string interface_ip(const std::string& iface) {
  struct ifaddrs* ifa = nullptr;
  if (getifaddrs(&ifa) != 0) return "";
  std::string out;
  for (auto* p = ifa; p; p = p->ifa_next) {
    if (!p->ifa_addr || p->ifa_addr->sa_family != AF_INET) continue;
    char buf[INET_ADDRSTRLEN];
    inet_ntop(AF_INET, &((sockaddr_in*)p->ifa_addr)->sin_addr, buf, sizeof(buf));
    const std::string ip = buf;
    if (!iface.empty() ? iface == p->ifa_name : ip.rfind("127.", 0) != 0) {
      out = ip;
      break;
    }
  }
  freeifaddrs(ifa);
  return out;
}

int free_port() {
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  addr.sin_port = 0;
  ::bind(fd, (sockaddr*)&addr, sizeof(addr));
  socklen_t len = sizeof(addr);
  getsockname(fd, (sockaddr*)&addr, &len);
  const int p = ntohs(addr.sin_port);
  ::close(fd);
  return p;
}

#ifndef PSAMD_CORE_STANDALONE
void register_runtime(py::module_& m) {
  py::class_<Van>(m, "Van")
      .def(py::init<std::string>())
      .def("bind", &Van::bind, py::arg("host") = "*", py::arg("port") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("connect", &Van::connect, py::call_guard<py::gil_scoped_release>())
      .def("connected", &Van::connected)
      .def("disconnect", &Van::disconnect, py::call_guard<py::gil_scoped_release>())
      .def("send", [](Van& v, const std::string& node, const py::list& frames) {
        std::vector<py::buffer_info> infos;
        std::vector<std::pair<const char*, size_t>> views;
        infos.reserve(frames.size());
        for (auto f : frames) {
          if (py::isinstance<py::bytes>(f)) {
            char* p;
            Py_ssize_t n;
            PyBytes_AsStringAndSize(f.ptr(), &p, &n);
            views.emplace_back(p, (size_t)n);
          } else {
            infos.push_back(py::reinterpret_borrow<py::buffer>(f).request());
            auto& bi = infos.back();
            views.emplace_back((const char*)bi.ptr, (size_t)(bi.size * bi.itemsize));
          }
        }
        py::gil_scoped_release rel;
        return v.send(node, views);
      })
      .def("recv", [](Van& v, double timeout) -> py::object {
        Received r;
        bool ok;
        {
          py::gil_scoped_release rel;
          ok = v.recv(&r, timeout);
        }
        if (!ok) return py::none();
        py::list frames;
        for (auto& f : r.frames) frames.append(py::bytes(f));
        return py::make_tuple(r.sender, frames);
      }, py::arg("timeout") = -1.0)
      .def("push_local", [](Van& v, const std::string& sender, const std::vector<py::bytes>& frames) {
        Received r;
        r.sender = sender;
        for (auto& f : frames) r.frames.emplace_back(f);
        v.push_local(std::move(r));
      })
      .def("stop", &Van::stop, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("port", &Van::port)
      .def("stats", &Van::stats);

  py::class_<TaskTracker>(m, "TaskTracker")
      .def(py::init<>())
      .def("start", &TaskTracker::start)
      .def("finish", &TaskTracker::finish)
      .def("has_finished", &TaskTracker::has_finished)
      .def("wait", &TaskTracker::wait, py::arg("t"), py::arg("timeout") = -1.0,
           py::call_guard<py::gil_scoped_release>())
      .def("all_finished", &TaskTracker::all_finished)
      .def("clear_below", &TaskTracker::clear_below)
      .def("__len__", &TaskTracker::size);

  m.def("interface_ip", &interface_ip, py::arg("interface") = "");
  m.def("free_port", &free_port);
}

#endif  // PSAMD_CORE_STANDALONE

}  // namespace pscore
