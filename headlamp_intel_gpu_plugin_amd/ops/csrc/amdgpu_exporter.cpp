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
// Serving: one thread multiplexes the listening socket and every connection
// with poll() over non-blocking sockets. Each connection has ONE deadline for
// the whole request (kRequestDeadlineMs: headers in, response out); a peer
// that trickles bytes or stops reading only holds its own socket until then,
// never a thread, so no number of slow peers below kMaxConns delays /healthz
// or a Prometheus scrape. At kMaxConns (or near the descriptor limit) the
// oldest connection still sending its request is dropped for the new one. A /metrics render is shared by requests
// arriving within kRenderCacheMs. SIGINT / SIGTERM end the loop.

#include <arpa/inet.h>
#include <netinet/in.h>
#include <poll.h>
#include <signal.h>
#include <sys/resource.h>
#include <sys/socket.h>
#include <sys/time.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <string>
#include <vector>

#include "probe_core.h"

namespace {

std::atomic<bool> g_stop{false};

constexpr int kRequestDeadlineMs = 3000;  // whole request: headers in, response out
constexpr size_t kMaxConns = 512;         // open connections (each is a socket, not a thread)
constexpr size_t kMaxHeader = 16384;
constexpr int kRenderCacheMs = 250;       // /metrics requests this close together share one render

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

using Clock = std::chrono::steady_clock;

int remaining_ms(Clock::time_point deadline, Clock::time_point now) {
  const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - now).count();
  return left > 0 ? static_cast<int>(left) : 0;
}

std::string response(int code, const char* reason, const std::string& type, const std::string& body) {
  return "HTTP/1.1 " + std::to_string(code) + " " + reason + "\r\nContent-Type: " + type +
         "\r\nContent-Length: " + std::to_string(body.size()) + "\r\nConnection: close\r\n\r\n" + body;
}

// /metrics body, re-rendered at most every kRenderCacheMs.
const std::string& metrics_body(const Args& a, Clock::time_point now) {
  static std::string body;
  static Clock::time_point at;
  static bool have = false;
  if (!have || now - at >= std::chrono::milliseconds(kRenderCacheMs)) {
    body = amdprobe::render(a.render);
    at = Clock::now();
    have = true;
  }
  return body;
}

// The response to a complete request header.
std::string answer(const std::string& req, const Args& a, Clock::time_point now) {
  const size_t sp1 = req.find(' ');
  const size_t sp2 = sp1 == std::string::npos ? std::string::npos : req.find(' ', sp1 + 1);
  if (sp2 == std::string::npos) return response(400, "Bad Request", "text/plain", "bad request\n");
  const std::string method = req.substr(0, sp1);
  std::string path = req.substr(sp1 + 1, sp2 - sp1 - 1);
  const size_t q = path.find('?');
  if (q != std::string::npos) path.resize(q);
  if (method != "GET") return response(405, "Method Not Allowed", "text/plain", "GET only\n");
  if (path == "/metrics") return response(200, "OK", "text/plain; version=0.0.4", metrics_body(a, now));
  if (path == "/healthz") return response(200, "OK", "text/plain", "ok\n");
  return response(404, "Not Found", "text/plain", "not found\n");
}

struct Conn {
  int fd;
  Clock::time_point accepted;
  Clock::time_point deadline;
  std::string in;
  std::string out;
  size_t off = 0;
  bool writing = false;
  bool eof = false;  // the peer shut its write side (recv returned 0)
};

// Read what is there; false when the read failed. A peer that sends its
// request and then half-closes (`nc -N`, some HTTP/1.0 probes) sets `eof`:
// what was read so far is still answered if it is a complete request.
bool read_some(Conn& c) {
  char buf[4096];
  for (;;) {
    const ssize_t n = recv(c.fd, buf, sizeof(buf), 0);
    if (n > 0) {
      c.in.append(buf, static_cast<size_t>(n));
      if (c.in.size() >= kMaxHeader) return true;
      continue;
    }
    if (n == 0) {
      c.eof = true;
      return true;
    }
    return errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR;
  }
}

// Send what the socket takes; true when the whole response is out.
bool write_some(Conn& c, bool* failed) {
  while (c.off < c.out.size()) {
    const ssize_t n = send(c.fd, c.out.data() + c.off, c.out.size() - c.off, MSG_NOSIGNAL);
    if (n > 0) {
      c.off += static_cast<size_t>(n);
      continue;
    }
    if (n < 0 && (errno == EAGAIN || errno == EWOULDBLOCK || errno == EINTR)) return false;
    *failed = true;
    return false;
  }
  return true;
}

// Advance one connection; false when it is finished (to be closed).
bool step(Conn& c, short revents, const Args& a, Clock::time_point now) {
  if (!c.writing) {
    if (revents & (POLLIN | POLLHUP | POLLERR)) {
      if (!read_some(c)) return false;
    }
    const bool complete = c.in.find("\r\n\r\n") != std::string::npos;
    if (complete || c.in.size() >= kMaxHeader) {
      c.out = complete ? answer(c.in, a, now) : response(431, "Request Header Fields Too Large", "text/plain", "header too large\n");
      c.writing = true;
    } else if (c.eof) {
      return false;  // closed before a whole request arrived: nothing to answer
    }
  } else if (revents & (POLLERR | POLLHUP | POLLNVAL)) {
    return false;
  }
  if (c.writing) {
    bool failed = false;
    if (write_some(c, &failed) || failed) return false;  // all sent (Connection: close) or peer gone
  }
  return now < c.deadline;
}

}  // namespace

int main(int argc, char** argv) {
  Args a;
  if (!parse_args(argc, argv, &a)) return 2;
  if (a.render.sysfs_only) {
    std::fprintf(stderr, "amdgpu-exporter: sysfs-only (no HIP runtime)\n");
  } else if (!amdprobe::init_hip()) {
    // No device is not fatal: the exporter still answers (with no GPU series),
    // which is what the plugin's "No AMD GPU Metrics" state expects.
    std::fprintf(stderr, "amdgpu-exporter: %s\n", amdprobe::last_error().c_str());
  }
  if (a.once) {
    std::fputs(amdprobe::render(a.render).c_str(), stdout);
    return 0;
  }
  signal(SIGINT, on_signal);
  signal(SIGTERM, on_signal);
  int srv = socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
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
  if (bind(srv, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) < 0 || listen(srv, 128) < 0) {
    std::perror("bind/listen");
    return 1;
  }
  socklen_t len = sizeof(addr);
  getsockname(srv, reinterpret_cast<sockaddr*>(&addr), &len);
  const int gpus = a.render.sysfs_only ? static_cast<int>(amdprobe::sysfs_gpu_bdfs().size()) : amdprobe::g_count;
  std::printf("amdgpu-exporter listening on %s:%d (%d GPU%s, hostname %s%s)\n", a.bind.c_str(), ntohs(addr.sin_port),
              gpus, gpus == 1 ? "" : "s", a.render.hostname.c_str(), a.render.sysfs_only ? ", sysfs-only" : "");
  std::fflush(stdout);
  // Stay below the descriptor limit: an accept() failing with EMFILE would
  // leave the listen socket readable and spin poll() until a peer closes.
  size_t max_conns = kMaxConns;
  rlimit nofile{};
  if (getrlimit(RLIMIT_NOFILE, &nofile) == 0 && nofile.rlim_cur != RLIM_INFINITY) {
    const rlim_t spare = 16;  // stdio, the listen socket, sysfs files opened while rendering
    max_conns = nofile.rlim_cur > spare + 1 ? std::min<size_t>(kMaxConns, nofile.rlim_cur - spare) : 1;
  }
  std::vector<Conn> conns;
  std::vector<pollfd> pfds;
  while (!g_stop.load()) {
    Clock::time_point now = Clock::now();
    pfds.clear();
    pfds.push_back(pollfd{srv, POLLIN, 0});
    int wait = 1000;  // wake at least once a second so a signal ends the loop promptly
    for (const Conn& c : conns) {
      pfds.push_back(pollfd{c.fd, static_cast<short>(c.writing ? POLLOUT : POLLIN), 0});
      wait = std::min(wait, remaining_ms(c.deadline, now));
    }
    const int r = poll(pfds.data(), pfds.size(), wait);
    if (r < 0) {
      if (errno == EINTR) continue;
      std::perror("poll");
      break;
    }
    now = Clock::now();
    for (size_t i = 0; i < conns.size(); ++i) {
      if (!step(conns[i], pfds[i + 1].revents, a, now)) {
        close(conns[i].fd);
        conns[i].fd = -1;
      }
    }
    conns.erase(std::remove_if(conns.begin(), conns.end(), [](const Conn& c) { return c.fd < 0; }), conns.end());
    if (pfds[0].revents & POLLIN) {
      for (;;) {
        const int fd = accept4(srv, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
        if (fd < 0) break;  // EAGAIN: nothing more to accept (or a transient error)
        if (conns.size() >= max_conns) {
          // Full: drop the oldest connection still sending its request (a
          // slow peer, most likely) rather than the new one.
          auto victim = conns.end();
          for (auto it = conns.begin(); it != conns.end(); ++it) {
            if (!it->writing && (victim == conns.end() || it->accepted < victim->accepted)) victim = it;
          }
          if (victim == conns.end()) {
            close(fd);
            continue;
          }
          close(victim->fd);
          conns.erase(victim);
        }
        Conn c;
        c.fd = fd;
        c.accepted = now;
        c.deadline = now + std::chrono::milliseconds(kRequestDeadlineMs);
        conns.push_back(std::move(c));
        // Most requests arrive with the connection: answer them in this pass.
        if (!step(conns.back(), POLLIN, a, now)) {
          close(conns.back().fd);
          conns.pop_back();
        }
      }
    }
  }
  for (const Conn& c : conns) close(c.fd);
  close(srv);
  return 0;
}
