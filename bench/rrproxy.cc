// hola_rrproxy — round-robin L4 (TCP) front for N hola replicas on one node: the role of the
// Kubernetes `LoadBalancer` Service (pom.xml:77-80) in the scale-out configs.
//
// Each accepted client connection is bound to the next *healthy* backend (round-robin).
// Health = GET /api/health answered 200 (the readiness probe of pom.xml:90-94), checked
// every --health-ms by a background thread; unhealthy replicas are skipped until they pass
// again. Bytes are relayed with recv/send through a small per-direction buffer.
#include <errno.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "client/url.h"
#include "core/affinity.h"
#include "core/net.h"

using namespace hola;

namespace {

struct Backend {
  std::string host;
  int port;
  sockaddr_storage addr;
  socklen_t len;
  std::atomic<bool> healthy{true};
  std::atomic<uint64_t> picked{0};
};

std::vector<std::unique_ptr<Backend>> g_backends;
std::atomic<uint64_t> g_rr{0};
std::atomic<bool> g_stop{false};

Backend* pick() {
  size_t n = g_backends.size();
  for (size_t k = 0; k < n; ++k) {
    Backend* b = g_backends[g_rr.fetch_add(1, std::memory_order_relaxed) % n].get();
    if (b->healthy.load(std::memory_order_relaxed)) return b;
  }
  return nullptr;
}

// One direction of a session: bytes read from `from` waiting to be written to `to`.
struct Dir {
  char buf[16384];
  size_t len = 0, off = 0;
};

struct Session;
struct Ev {
  Session* s;
  bool client;  // event on the client socket
};

struct Session {
  int cfd = -1, bfd = -1;
  Dir c2b, b2c;
  bool closing = false;
  Ev ec{this, true}, eb{this, false};
  uint32_t cint = EPOLLIN | EPOLLRDHUP, bint = EPOLLIN | EPOLLRDHUP;
};

// Plain recv/send relay: for the small request/response messages of this service it costs
// two syscalls per hop, less than splice(2) through a pipe (four).
// Returns false when the session must close.
bool pump(int epfd, Session* s, bool from_client) {
  int from = from_client ? s->cfd : s->bfd, to = from_client ? s->bfd : s->cfd;
  Dir& d = from_client ? s->c2b : s->b2c;
  for (;;) {
    if (d.off < d.len) {
      ssize_t m = ::send(to, d.buf + d.off, d.len - d.off, MSG_NOSIGNAL);
      if (m < 0) {
        if (errno == EAGAIN) {
          // destination full: stop reading `from`, wait for `to` to drain
          uint32_t& fi = from_client ? s->cint : s->bint;
          uint32_t& ti = from_client ? s->bint : s->cint;
          epoll_event ev{};
          fi = EPOLLRDHUP;
          ev.events = fi;
          ev.data.ptr = from_client ? &s->ec : &s->eb;
          epoll_ctl(epfd, EPOLL_CTL_MOD, from, &ev);
          ti |= EPOLLOUT;
          ev.events = ti;
          ev.data.ptr = from_client ? &s->eb : &s->ec;
          epoll_ctl(epfd, EPOLL_CTL_MOD, to, &ev);
          return true;
        }
        return false;
      }
      d.off += size_t(m);
      continue;
    }
    d.off = d.len = 0;
    ssize_t n = ::recv(from, d.buf, sizeof d.buf, 0);
    if (n == 0) return false;
    if (n < 0) return errno == EAGAIN || errno == EINTR;
    d.len = size_t(n);
  }
}

// `fd` became writable: flush what was waiting for it and resume reading the other side.
bool drained(int epfd, Session* s, bool client_writable) {
  bool from_client = !client_writable;  // data flowing *to* the writable socket
  Dir& d = from_client ? s->c2b : s->b2c;
  int to = client_writable ? s->cfd : s->bfd, from = client_writable ? s->bfd : s->cfd;
  while (d.off < d.len) {
    ssize_t m = ::send(to, d.buf + d.off, d.len - d.off, MSG_NOSIGNAL);
    if (m < 0) return errno == EAGAIN;
    d.off += size_t(m);
  }
  d.off = d.len = 0;
  uint32_t& ti = client_writable ? s->cint : s->bint;
  uint32_t& fi = client_writable ? s->bint : s->cint;
  epoll_event ev{};
  ti &= ~uint32_t(EPOLLOUT);
  ev.events = ti;
  ev.data.ptr = client_writable ? &s->ec : &s->eb;
  epoll_ctl(epfd, EPOLL_CTL_MOD, to, &ev);
  fi = EPOLLIN | EPOLLRDHUP | (fi & EPOLLOUT);
  ev.events = fi;
  ev.data.ptr = client_writable ? &s->eb : &s->ec;
  epoll_ctl(epfd, EPOLL_CTL_MOD, from, &ev);
  return pump(epfd, s, from_client);
}

void close_session(int epfd, Session* s) {
  epoll_ctl(epfd, EPOLL_CTL_DEL, s->cfd, nullptr);
  epoll_ctl(epfd, EPOLL_CTL_DEL, s->bfd, nullptr);
  ::close(s->cfd);
  ::close(s->bfd);
}

void worker(int lfd, int cpu) {
  if (cpu >= 0) pin_current_thread(cpu);
  int epfd = epoll_create1(EPOLL_CLOEXEC);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.ptr = nullptr;
  epoll_ctl(epfd, EPOLL_CTL_ADD, lfd, &ev);
  epoll_event evs[256];
  std::vector<Session*> dead;
  while (!g_stop.load()) {
    int n = epoll_wait(epfd, evs, 256, 200);
    for (int i = 0; i < n; ++i) {
      if (!evs[i].data.ptr) {
        for (;;) {
          int c = accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
          if (c < 0) break;
          set_nodelay(c);
          Backend* b = pick();
          if (!b) {
            ::close(c);
            continue;
          }
          b->picked.fetch_add(1, std::memory_order_relaxed);
          int bfd = connect_blocking(b->addr, b->len, 1000);
          if (bfd < 0) {
            b->healthy.store(false);
            ::close(c);
            continue;
          }
          set_nonblocking(bfd, true);
          auto* s = new Session();
          s->cfd = c;
          s->bfd = bfd;
          ev.events = s->cint;
          ev.data.ptr = &s->ec;
          epoll_ctl(epfd, EPOLL_CTL_ADD, c, &ev);
          ev.events = s->bint;
          ev.data.ptr = &s->eb;
          epoll_ctl(epfd, EPOLL_CTL_ADD, bfd, &ev);
        }
        continue;
      }
      Ev* e = static_cast<Ev*>(evs[i].data.ptr);
      Session* s = e->s;
      if (s->closing) continue;
      bool ok = true;
      uint32_t evm = evs[i].events;
      if (evm & EPOLLOUT) ok = drained(epfd, s, e->client);
      if (ok && (evm & (EPOLLIN | EPOLLRDHUP | EPOLLHUP))) ok = pump(epfd, s, e->client);
      if (!ok || (evm & EPOLLERR)) {
        s->closing = true;
        close_session(epfd, s);
        dead.push_back(s);  // the peer's event may still be in this batch: free afterwards
      }
    }
    for (Session* s : dead) delete s;
    dead.clear();
  }
}

void health_loop(int interval_ms) {
  while (!g_stop.load()) {
    for (auto& b : g_backends) {
      client::Url u;
      u.host = b->host;
      u.port = b->port;
      int fd = -1;
      client::BlockingResponse r;
      bool ok = client::blocking_request(u, &fd, "GET", "/api/health", "", "", 1000, &r) && r.status == 200;
      if (fd >= 0) ::close(fd);
      bool was = b->healthy.exchange(ok);
      if (was != ok) fprintf(stderr, "rrproxy: backend %s:%d is %s\n", b->host.c_str(), b->port, ok ? "UP" : "DOWN");
    }
    for (int w = 0; w < interval_ms && !g_stop.load(); w += 20) std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

}  // namespace

int main(int argc, char** argv) {
  int port = 8080, threads = 1, health_ms = 500;
  std::string backends, cpu_list, host = "0.0.0.0", port_file;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) exit(2);
      return argv[++i];
    };
    if (a == "--port") port = atoi(val().c_str());
    else if (a == "--host") host = val();
    else if (a == "--backends") backends = val();
    else if (a == "--threads") threads = atoi(val().c_str());
    else if (a == "--cpu-list") cpu_list = val();
    else if (a == "--health-ms") health_ms = atoi(val().c_str());
    else if (a == "--port-file") port_file = val();
    else {
      fprintf(stderr, "usage: hola_rrproxy --backends h:p,h:p.. [--port N] [--threads N] [--cpu-list L] [--health-ms N]\n");
      return 2;
    }
  }
  signal(SIGPIPE, SIG_IGN);
  size_t i = 0;
  while (i < backends.size()) {
    size_t j = backends.find(',', i);
    if (j == std::string::npos) j = backends.size();
    std::string t = backends.substr(i, j - i);
    i = j + 1;
    size_t colon = t.rfind(':');
    if (colon == std::string::npos) return 2;
    auto b = std::make_unique<Backend>();
    b->host = t.substr(0, colon);
    b->port = atoi(t.substr(colon + 1).c_str());
    std::string err;
    if (!resolve_host(b->host, b->port, &b->addr, &b->len, &err)) {
      fprintf(stderr, "rrproxy: %s\n", err.c_str());
      return 2;
    }
    g_backends.push_back(std::move(b));
  }
  if (g_backends.empty()) {
    fprintf(stderr, "rrproxy: --backends required\n");
    return 2;
  }
  std::vector<int> cpus;
  if (!cpu_list.empty()) parse_cpu_list(cpu_list, &cpus);
  ListenOptions lo;
  lo.host = host;
  lo.port = port;
  lo.reuseport = true;
  std::vector<int> lfds;
  std::string err;
  for (int t = 0; t < threads; ++t) {
    int fd = listen_tcp(lo, &err);
    if (fd < 0) {
      fprintf(stderr, "rrproxy: %s\n", err.c_str());
      return 1;
    }
    if (t == 0) lo.port = bound_port(fd);
    lfds.push_back(fd);
  }
  if (!port_file.empty()) {
    FILE* f = fopen((port_file + ".tmp").c_str(), "w");
    fprintf(f, "%d\n", lo.port);
    fclose(f);
    rename((port_file + ".tmp").c_str(), port_file.c_str());
  }
  fprintf(stderr, "rrproxy: listening on %s:%d -> %zu backends\n", host.c_str(), lo.port, g_backends.size());
  sigset_t sigs;
  sigemptyset(&sigs);
  sigaddset(&sigs, SIGTERM);
  sigaddset(&sigs, SIGINT);
  pthread_sigmask(SIG_BLOCK, &sigs, nullptr);
  std::thread hc(health_loop, health_ms);
  std::vector<std::thread> ws;
  for (int t = 0; t < threads; ++t) ws.emplace_back(worker, lfds[size_t(t)], cpus.empty() ? -1 : cpus[size_t(t) % cpus.size()]);
  int sig;
  sigwait(&sigs, &sig);
  g_stop.store(true);
  for (auto& w : ws) w.join();
  hc.join();
  for (auto& b : g_backends) fprintf(stderr, "rrproxy: %s:%d picked %llu\n", b->host.c_str(), b->port, (unsigned long long)b->picked.load());
  return 0;
}
