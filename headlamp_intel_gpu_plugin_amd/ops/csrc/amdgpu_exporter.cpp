// amdgpu-exporter — minimal native Prometheus exporter for MI355X nodes.
//
// Serves the probe's exporter-format metrics (probe_core.h: power, power cap,
// GFX / HBM-controller activity, HBM used / total, temperatures, clocks, xGMI
// link hops) over HTTP so Prometheus can scrape one instance per GPU node
// (DaemonSet), and the plugin's Metrics page reads them with the same queries
// it uses for the AMD Device Metrics Exporter (src/api/metrics.js SERIES).
//
//   amdgpu-exporter [--port 9400] [--bind 0.0.0.0] [--hostname NAME]
//                   [--device N [--gpu-label L]] [--no-topology] [--sysfs-only] [--once]
//
// --hostname defaults to $NODE_NAME (set from the downward API in a
// DaemonSet), then gethostname(). --once prints one scrape and exits (used by
// tests and for debugging). Endpoints: GET /metrics, GET /healthz.
//
// --sysfs-only never starts the HIP runtime: devices come from the DRM cards
// in sysfs and xGMI links from the KFD topology where it is readable
// (probe_core.h), so the exporter needs no device node and runs unprivileged
// with /sys mounted read-only (deploy/exporter/daemonset.yaml).
//
// Serving: the accept loop hands connections to a few worker threads through
// a bounded queue (full → the connection is closed at once). Each connection
// has ONE deadline for the whole request (kRequestDeadlineMs, enforced with
// poll() on every read) and a send timeout, so a client that trickles bytes
// or stops reading holds one worker for at most a few seconds and never the
// /healthz probe or the Prometheus scrape behind it. SIGINT / SIGTERM stop
// the loop and the workers cleanly.

#include <arpa/inet.h>
#include <netinet/in.h>
#include <poll.h>
#include <signal.h>
#include <sys/socket.h>
#include <sys/time.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "probe_core.h"

namespace {

std::atomic<bool> g_stop{false};

constexpr int kRequestDeadlineMs = 3000;  // whole request: headers in, response out
constexpr int kWorkers = 4;
constexpr size_t kMaxQueued = 64;

void on_signal(int) { g_stop.store(true); }

struct Args {
  int port = 9400;
  std::string bind = "0.0.0.0";
  amdprobe::RenderOptions render;
  bool once = false;
};

bool parse_args(int argc, char** argv, Args* a) {
  const char* env = std::getenv("NODE_NAME");
  if (env && *env) {
    a->render.hostname = env;
  } else {
    char host[256] = {0};
    if (gethostname(host, sizeof(host) - 1) == 0) a->render.hostname = host;
  }
  for (int i = 1; i < argc; ++i) {
    std::string k = argv[i];
    auto next = [&](const char* what) -> const char* {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "missing value for %s\n", what);
        return nullptr;
      }
      return argv[++i];
    };
    if (k == "--port") {
      const char* v = next("--port");
      if (!v) return false;
      a->port = std::atoi(v);
    } else if (k == "--bind") {
      const char* v = next("--bind");
      if (!v) return false;
      a->bind = v;
    } else if (k == "--hostname") {
      const char* v = next("--hostname");
      if (!v) return false;
      a->render.hostname = v;
    } else if (k == "--device") {
      const char* v = next("--device");
      if (!v) return false;
      a->render.only_device = std::atoi(v);
    } else if (k == "--gpu-label") {
      const char* v = next("--gpu-label");
      if (!v) return false;
      a->render.gpu_label = v;
    } else if (k == "--no-topology") {
      a->render.topology = false;
    } else if (k == "--sysfs-only") {
      a->render.sysfs_only = true;
    } else if (k == "--once") {
      a->once = true;
    } else if (k == "--help" || k == "-h") {
      std::printf("usage: amdgpu-exporter [--port 9400] [--bind ADDR] [--hostname NAME] [--device N [--gpu-label L]] "
                  "[--no-topology] [--sysfs-only] [--once]\n");
      std::exit(0);
    } else {
      std::fprintf(stderr, "unknown argument %s\n", k.c_str());
      return false;
    }
  }
  if (a->port < 0 || a->port > 65535) {
    std::fprintf(stderr, "bad port %d\n", a->port);
    return false;
  }
  return true;
}

void send_all(int fd, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    ssize_t n = send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
    if (n <= 0) return;
    off += static_cast<size_t>(n);
  }
}

void respond(int fd, int code, const char* reason, const std::string& type, const std::string& body) {
  std::string h = "HTTP/1.1 " + std::to_string(code) + " " + reason + "\r\nContent-Type: " + type +
                  "\r\nContent-Length: " + std::to_string(body.size()) + "\r\nConnection: close\r\n\r\n";
  send_all(fd, h + body);
}

using Clock = std::chrono::steady_clock;

int remaining_ms(Clock::time_point deadline) {
  const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - Clock::now()).count();
  return left > 0 ? static_cast<int>(left) : 0;
}

void handle(int fd, const Args& a) {
  const Clock::time_point deadline = Clock::now() + std::chrono::milliseconds(kRequestDeadlineMs);
  // A peer that stops reading cannot hold the worker past the deadline either.
  timeval stv{kRequestDeadlineMs / 1000, 0};
  setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &stv, sizeof(stv));
  std::string req;
  char buf[2048];
  while (req.find("\r\n\r\n") == std::string::npos && req.size() < 16384) {
    // One deadline for the whole header, however slowly the bytes arrive.
    pollfd p{fd, POLLIN, 0};
    const int wait = remaining_ms(deadline);
    if (wait <= 0 || poll(&p, 1, wait) <= 0) return;
    ssize_t n = recv(fd, buf, sizeof(buf), 0);
    if (n <= 0) return;
    req.append(buf, static_cast<size_t>(n));
  }
  const size_t sp1 = req.find(' ');
  const size_t sp2 = sp1 == std::string::npos ? std::string::npos : req.find(' ', sp1 + 1);
  if (sp2 == std::string::npos) {
    respond(fd, 400, "Bad Request", "text/plain", "bad request\n");
    return;
  }
  const std::string method = req.substr(0, sp1);
  std::string path = req.substr(sp1 + 1, sp2 - sp1 - 1);
  const size_t q = path.find('?');
  if (q != std::string::npos) path.resize(q);
  if (method != "GET") {
    respond(fd, 405, "Method Not Allowed", "text/plain", "GET only\n");
  } else if (path == "/metrics") {
    std::string body;
    {
      // The probe keeps process-wide state (error text, HIP handles): one
      // scrape renders at a time; /healthz never waits for it.
      static std::mutex render_mu;
      std::lock_guard<std::mutex> lk(render_mu);
      body = amdprobe::render(a.render);
    }
    respond(fd, 200, "OK", "text/plain; version=0.0.4", body);
  } else if (path == "/healthz") {
    respond(fd, 200, "OK", "text/plain", "ok\n");
  } else {
    respond(fd, 404, "Not Found", "text/plain", "not found\n");
  }
}

// Accepted connections waiting for a worker.
class ConnQueue {
 public:
  bool push(int fd) {
    std::lock_guard<std::mutex> lk(mu_);
    if (q_.size() >= kMaxQueued) return false;
    q_.push_back(fd);
    cv_.notify_one();
    return true;
  }
  // Next connection, or -1 once stopped.
  int pop() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return stopped_ || !q_.empty(); });
    if (q_.empty()) return -1;
    const int fd = q_.front();
    q_.pop_front();
    return fd;
  }
  void stop() {
    std::lock_guard<std::mutex> lk(mu_);
    stopped_ = true;
    cv_.notify_all();
  }
  void drain() {
    std::lock_guard<std::mutex> lk(mu_);
    for (int fd : q_) close(fd);
    q_.clear();
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<int> q_;
  bool stopped_ = false;
};

}  // namespace

int main(int argc, char** argv) {
  Args a;
  if (!parse_args(argc, argv, &a)) return 2;
  if (a.render.sysfs_only) {
    std::fprintf(stderr, "amdgpu-exporter: sysfs-only (no HIP runtime)\n");
  } else if (!amdprobe::init_hip()) {
    // No device is not fatal: the exporter still answers (with no GPU series),
    // which is what the plugin's "No AMD GPU Metrics" state expects.
    std::fprintf(stderr, "amdgpu-exporter: %s\n", amdprobe::g_error.c_str());
  }
  if (a.once) {
    std::fputs(amdprobe::render(a.render).c_str(), stdout);
    return 0;
  }
  signal(SIGINT, on_signal);
  signal(SIGTERM, on_signal);
  int srv = socket(AF_INET, SOCK_STREAM, 0);
  if (srv < 0) {
    std::perror("socket");
    return 1;
  }
  int one = 1;
  setsockopt(srv, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons(static_cast<uint16_t>(a.port));
  if (inet_pton(AF_INET, a.bind.c_str(), &addr.sin_addr) != 1) {
    std::fprintf(stderr, "bad bind address %s\n", a.bind.c_str());
    return 2;
  }
  if (bind(srv, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) < 0 || listen(srv, 16) < 0) {
    std::perror("bind/listen");
    return 1;
  }
  socklen_t len = sizeof(addr);
  getsockname(srv, reinterpret_cast<sockaddr*>(&addr), &len);
  const int gpus = a.render.sysfs_only ? static_cast<int>(amdprobe::sysfs_gpu_bdfs().size()) : amdprobe::g_count;
  std::printf("amdgpu-exporter listening on %s:%d (%d GPU%s, hostname %s%s)\n", a.bind.c_str(), ntohs(addr.sin_port),
              gpus, gpus == 1 ? "" : "s", a.render.hostname.c_str(), a.render.sysfs_only ? ", sysfs-only" : "");
  std::fflush(stdout);
  ConnQueue queue;
  std::vector<std::thread> workers;
  for (int i = 0; i < kWorkers; ++i) {
    workers.emplace_back([&] {
      for (int fd = queue.pop(); fd >= 0; fd = queue.pop()) {
        handle(fd, a);
        close(fd);
      }
    });
  }
  // Wake accept() periodically so a signal ends the loop promptly.
  timeval tv{1, 0};
  setsockopt(srv, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  while (!g_stop.load()) {
    int fd = accept(srv, nullptr, nullptr);
    if (fd < 0) {
      if (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR) continue;
      std::perror("accept");
      break;
    }
    if (!queue.push(fd)) close(fd);  // overloaded: shed the connection
  }
  queue.stop();
  for (auto& w : workers) w.join();
  queue.drain();
  close(srv);
  return 0;
}
