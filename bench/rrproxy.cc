// hola_rrproxy — round-robin L4 (TCP) front for N hola replicas on one node: the role of the
// Kubernetes `LoadBalancer` Service (pom.xml:77-80) in the scale-out configs.
//
// Each accepted client connection is bound to the next *healthy* backend (round-robin).
// Health = GET /api/health answered 200 (the readiness probe of pom.xml:90-94), checked
// every --health-ms by a background thread; unhealthy replicas are skipped until they pass
// again, and a backend that refuses a connect is marked down at once and the next one tried.
//
// Data path: one pinned EventLoop (src/core/loop.h, the server's own loop) per proxy thread.
// Both sockets of a session live on one loop, registered once, edge-triggered, for
// IN|OUT|RDHUP: no epoll_ctl per message. A read that comes back short has drained the
// socket (no extra EAGAIN read); a send that would block parks the bytes until the OUT edge
// and stops reading the other side until they are gone (backpressure). Accepted sockets are
// handed to a loop in the client's L3 domain (SO_INCOMING_CPU), as the server does. A FIN
// is passed on as a half-close; sessions silent for --idle-timeout-ms are closed.
//
// Service mode (`python -m hola_amd apply`, the local manifest executor): --endpoints-file F
// takes the backend set from F (one host:port per line), re-read whenever it changes; the
// executor writes the Ready pods there, the role of the Endpoints object that kube-proxy
// follows. After applying a file whose first line is `# gen N`, the proxy writes N to
// F.applied, so the writer knows when new connections follow the new set. --health-ms 0 turns the proxy's own probing off (kube-proxy does not probe), and
// --no-failover makes a connection to a backend that refuses fail as it does through
// kube-proxy's DNAT rules, instead of being retried on the next backend. Sessions keep their
// backend when it leaves the set (conntrack keeps established flows).
//
// Topology hints: a backend given as `host:port@cpus` (e.g. 127.0.0.1:18400@16-17) says where
// its workers run. A proxy thread then deals its sessions round-robin over the healthy
// backends that share its L3 domain, and over all of them only when none does (Kubernetes'
// topology-aware routing, with the L3 as the zone): a session's client, proxy thread and
// server then stay in one cache domain. Without hints every thread deals over every backend.
#include <errno.h>
#include <sys/stat.h>
#include <signal.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "client/url.h"
#include "core/build_info.h"
#include "core/isa.h"
#include "core/affinity.h"
#include "core/loop.h"
#include "core/net.h"

using namespace hola;

namespace {

struct Backend {
  std::string host;
  int port;
  sockaddr_storage addr;
  socklen_t len;
  // L3 domains of its workers (topology hint); empty = unknown. Written and read only by the
  // thread that parses backend lists (under g_backends_mu); proxy threads read the copy in the
  // published BackendSet, which never changes once published.
  std::vector<int> hint;
  std::atomic<bool> healthy{true};
  std::atomic<uint64_t> picked{0};
};

// Every backend ever named, never freed (sessions and the current set point into it).
std::vector<std::unique_ptr<Backend>> g_backends;
std::mutex g_backends_mu;  // guards g_backends growth (the endpoints reloader)
// The set new connections are dealt over. Replaced whole on an endpoints change; an old set
// is kept (a few pointers) because a loop thread may still be reading it.
struct BackendSet {
  std::vector<Backend*> list;
  std::vector<std::vector<int>> l3;  // list[i]'s topology hint, copied at publish
};
std::atomic<const BackendSet*> g_set{nullptr};
std::vector<std::unique_ptr<BackendSet>> g_sets;  // owner of every set published
std::atomic<uint64_t> g_rr{0};
std::atomic<bool> g_stop{false};
bool g_failover = true;

// Why sessions ended other than by both sides' FIN, reported at exit: a client that sees a
// reset can then be matched to its cause (the backend's side, its own side, or a connect).
struct CloseStats {
  std::atomic<uint64_t> sessions{0}, client_err{0}, backend_err{0}, connect_fail{0};
  std::atomic<int> client_errno{0}, backend_errno{0}, connect_errno{0};
};
CloseStats g_close;

void note_connect_fail(int err) {
  g_close.connect_fail.fetch_add(1, std::memory_order_relaxed);
  g_close.connect_errno.store(err, std::memory_order_relaxed);
}

const BackendSet& current_set() { return *g_set.load(std::memory_order_acquire); }

// `l3` = the calling proxy thread's L3 domain (-1: unknown); `rr` = its own round-robin
// counter for the backends of that domain.
Backend* pick(int l3 = -1, uint64_t* rr = nullptr) {
  const BackendSet& set = current_set();
  const size_t n = set.list.size();
  if (l3 >= 0 && rr) {
    // topology hints: the healthy backends in this thread's L3, round-robin
    for (size_t k = 0; k < n; ++k) {
      const size_t i = (*rr)++ % n;
      Backend* b = set.list[i];
      const std::vector<int>& doms = set.l3[i];
      if (b->healthy.load(std::memory_order_relaxed) && std::find(doms.begin(), doms.end(), l3) != doms.end())
        return b;
    }
  }
  for (size_t k = 0; k < n; ++k) {
    Backend* b = set.list[g_rr.fetch_add(1, std::memory_order_relaxed) % n];
    if (b->healthy.load(std::memory_order_relaxed)) return b;
  }
  return nullptr;
}

Backend* backend_for(const std::string& host, int port) {
  std::lock_guard<std::mutex> g(g_backends_mu);
  for (auto& b : g_backends)
    if (b->host == host && b->port == port) return b.get();
  auto b = std::make_unique<Backend>();
  b->host = host;
  b->port = port;
  std::string err;
  if (!resolve_host(host, port, &b->addr, &b->len, &err)) {
    fprintf(stderr, "rrproxy: %s\n", err.c_str());
    return nullptr;
  }
  g_backends.push_back(std::move(b));
  return g_backends.back().get();
}

// "h:p,h:p" or one h:p per line (IPv6 as [addr]:port or addr:port split at the last colon).
bool parse_backends(const std::string& text, std::vector<Backend*>* out) {
  size_t i = 0;
  while (i < text.size()) {
    size_t j = text.find_first_of(",\n", i);
    if (j == std::string::npos) j = text.size();
    std::string t = text.substr(i, j - i);
    i = j + 1;
    while (!t.empty() && (t.back() == ' ' || t.back() == '\r')) t.pop_back();
    while (!t.empty() && t.front() == ' ') t.erase(0, 1);
    if (t.empty() || t[0] == '#') continue;
    std::vector<int> cpus;  // topology hint after '@'
    if (size_t at = t.find('@'); at != std::string::npos) {
      std::vector<int> tmp;
      std::string list = t.substr(at + 1);
      for (char& ch : list)
        if (ch == ';') ch = ',';  // "0-1;8" inside a comma-separated --backends
      if (!parse_cpu_list(list, &tmp)) return false;
      cpus = std::move(tmp);
      t.resize(at);
    }
    size_t colon = t.rfind(':');
    if (colon == std::string::npos) return false;
    std::string host = t.substr(0, colon);
    if (host.size() > 2 && host.front() == '[' && host.back() == ']') host = host.substr(1, host.size() - 2);
    Backend* b = backend_for(host, atoi(t.substr(colon + 1).c_str()));
    if (!b) return false;
    if (!cpus.empty()) {
      std::lock_guard<std::mutex> g(g_backends_mu);
      if (b->hint.empty()) {  // set once (a reload may name it again, with or without a hint)
        for (int c : cpus)
          if (int d = l3_domain_of(c); d >= 0 && std::find(b->hint.begin(), b->hint.end(), d) == b->hint.end())
            b->hint.push_back(d);
      }
    }
    if (std::find(out->begin(), out->end(), b) == out->end()) out->push_back(b);
  }
  return true;
}

void publish_set(std::vector<Backend*> list) {
  auto set = std::make_unique<BackendSet>();
  set->list = std::move(list);
  {
    // The hints as of now, copied: a later reload that adds a hint to a backend of this set
    // changes the Backend, never a set a proxy thread may be reading.
    std::lock_guard<std::mutex> g(g_backends_mu);
    for (Backend* b : set->list) set->l3.push_back(b->hint);
  }
  for (Backend* b : set->list) b->healthy.store(true);  // listed = Ready (the executor probed it)
  g_set.store(set.get(), std::memory_order_release);
  g_sets.push_back(std::move(set));
}

// Follows --endpoints-file. The writer replaces it with a rename, so a reader never sees half
// a file; the file is read again every pass and compared by content, because a replacement
// can keep the inode number (recycled), the size and the (coarse) mtime of the one before.
struct EndpointsFollower {
  std::string path, last;
  bool have = false;

  // Publishes the file's set if it changed; true once a set has been read.
  bool poll() {
    std::ifstream f(path);
    if (!f) return have;
    std::string text((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    std::vector<Backend*> list;
    if ((have && text == last) || !parse_backends(text, &list)) return have;
    publish_set(std::move(list));
    fprintf(stderr, "rrproxy: endpoints now %zu backends\n", current_set().list.size());
    last = std::move(text);
    have = true;
    unsigned long long gen = 0;
    if (sscanf(last.c_str(), "# gen %llu", &gen) == 1) {
      const std::string tmp = path + ".applied.tmp";
      if (FILE* out = fopen(tmp.c_str(), "w")) {
        fprintf(out, "%llu\n", gen);
        fclose(out);
        rename(tmp.c_str(), (path + ".applied").c_str());
      }
    }
    return true;
  }

  void loop() {
    while (!g_stop.load()) {
      poll();
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
  }
};

int socket_error(int fd) {
  int e = 0;
  socklen_t sl = sizeof e;
  if (getsockopt(fd, SOL_SOCKET, SO_ERROR, &e, &sl) != 0) e = errno;
  return e ? e : EIO;
}

void mark_down(Backend* b, int err) {
  if (b->healthy.exchange(false))
    fprintf(stderr, "rrproxy: backend %s:%d is DOWN (%s)\n", b->host.c_str(), b->port, strerror(err));
}

// Starts a non-blocking connect to a healthy backend, failing over (and marking refusers
// down) while connect() fails at once. The handshake may still be in progress: bytes sent
// before it completes wait for the socket's OUT edge, and a refusal reported then fails over
// from Session::on_event.
int connect_backend(Backend** chosen, bool* in_progress, int l3 = -1, uint64_t* rr = nullptr) {
  const size_t n = g_failover ? current_set().list.size() : 1;
  for (size_t tries = 0; tries < n; ++tries) {
    Backend* b = pick(l3, rr);
    if (!b) {
      note_connect_fail(EHOSTUNREACH);  // no healthy backend
      return -1;
    }
    int fd = connect_nonblocking(b->addr, b->len, in_progress);
    if (fd >= 0) {
      b->picked.fetch_add(1, std::memory_order_relaxed);
      *chosen = b;
      return fd;
    }
    note_connect_fail(errno);
    // Out of local fds, memory or ephemeral ports: the next backend would fail the same
    // way, and none of them is at fault.
    if (is_local_resource_error(errno)) return -1;
    if (!g_failover) return -1;  // kube-proxy: the client's connection fails with the backend's
    mark_down(b, errno);
  }
  return -1;
}

class ProxyLoop;

// One direction of a session: bytes read from one socket that the other has not taken yet.
struct Pipe {
  char buf[16384];
  size_t len = 0, off = 0;
  bool eof = false;   // the source sent its FIN
  bool shut = false;  // ... and it was passed on (shutdown(SHUT_WR) of the destination)
  bool hup = false;   // an edge carried RDHUP/HUP: read the source on to its EOF
  bool pending() const { return off < len; }
};

struct Session : EventLoop::Handler {
  struct Side : EventLoop::Handler {
    Session* s = nullptr;
    bool client = false;
    void on_event(uint32_t ev) override { s->on_event(client, ev); }
  };
  ProxyLoop* owner;
  int cfd, bfd;
  Side cside, bside;
  Pipe c2b, b2c;
  Backend* backend = nullptr;
  bool connecting = false;  // backend handshake not confirmed yet
  int failovers = 0;
  bool closed = false;
  int err = 0;              // the first hard socket error (errno), 0 = none
  bool err_client = false;  // ... and whether it was on the client's socket
  int64_t last_active_ms = 0;  // for the idle timeout
  Session *prev = nullptr, *next = nullptr;  // the owning loop's list of open sessions

  Session(ProxyLoop* o, int c, int b) : owner(o), cfd(c), bfd(b) {
    cside.s = bside.s = this;
    cside.client = true;
  }
  void on_event(uint32_t) override {}  // lifetime anchor for EventLoop::retire
  void on_event(bool client_side, uint32_t ev);
  bool flush(Pipe& p, int to);
  bool pump(bool from_client);
  void close();
  bool backend_connected(uint32_t ev);
  void note_err(bool on_client, int e) {
    if (err == 0 && e != 0) {
      err = e;
      err_client = on_client;
    }
  }
};

class ProxyLoop {
 public:
  ProxyLoop(int index, int cpu, int busy_poll_us, int busy_poll_pause, int idle_timeout_ms)
      : index_(index), cpu_(cpu), idle_timeout_ms_(idle_timeout_ms), l3_(cpu >= 0 ? l3_domain_of(cpu) : -1) {
    loop_.set_busy_poll_us(busy_poll_us);
    loop_.set_busy_poll_pause(busy_poll_pause);
  }
  EventLoop& loop() { return loop_; }
  int cpu() const { return cpu_; }
  int l3() const { return l3_; }
  uint64_t* rr() { return &rr_; }
  int index() const { return index_; }
  std::atomic<int64_t>& sessions() { return sessions_; }

  void link(Session* s) {
    s->next = head_;
    if (head_) head_->prev = s;
    head_ = s;
  }
  void unlink(Session* s) {
    if (s->prev) s->prev->next = s->next;
    else head_ = s->next;
    if (s->next) s->next->prev = s->prev;
    s->prev = s->next = nullptr;
  }
  // After run() returned: closes what is still open (freed with the loop's retired handlers).
  void close_all();

  void adopt(int cfd) {
    loop_.post([this, cfd] { adopt_here(cfd); });
  }
  static constexpr uint32_t kEvents = EPOLLIN | EPOLLOUT | EPOLLRDHUP | EPOLLET;
  void adopt_here(int cfd) {
    Backend* b = nullptr;
    bool inprog = false;
    int bfd = connect_backend(&b, &inprog, l3_, &rr_);
    if (bfd < 0) {
      ::close(cfd);
      sessions_.fetch_sub(1, std::memory_order_relaxed);
      return;
    }
    auto* s = new Session(this, cfd, bfd);
    s->backend = b;
    s->connecting = inprog;
    s->last_active_ms = loop_.now_ms();
    link(s);
    loop_.add(bfd, kEvents, &s->bside);
    loop_.add(cfd, kEvents, &s->cside);
  }
  void run() {
    if (cpu_ >= 0) pin_current_thread(cpu_);
    if (idle_timeout_ms_ > 0) schedule_sweep();
    loop_.run();
  }
  // Closes sessions with no traffic in either direction for the idle timeout (an L4 front's
  // "timeout client/server"): e.g. a client that keeps a session open after the backend
  // closed its side.
  void schedule_sweep() {
    const int period = std::max(50, std::min(1000, idle_timeout_ms_ / 4));
    loop_.add_timer(period, [this] {
      const int64_t now = loop_.now_ms();
      for (Session* s = head_; s;) {
        Session* next = s->next;
        if (now - s->last_active_ms > idle_timeout_ms_) s->close();
        s = next;
      }
      schedule_sweep();
    });
  }

 private:
  EventLoop loop_;
  int index_, cpu_;
  int idle_timeout_ms_;
  int l3_;           // this thread's L3 domain (topology hints)
  uint64_t rr_ = 0;  // round-robin position over the backends of that domain
  std::atomic<int64_t> sessions_{0};
  Session* head_ = nullptr;
};

// Writes what `p` holds to `to`. False on a hard error; true otherwise (p may stay pending
// when `to` is full: the OUT edge resumes it).
bool Session::flush(Pipe& p, int to) {
  while (p.pending()) {
    ssize_t m = ::send(to, p.buf + p.off, p.len - p.off, MSG_NOSIGNAL);
    if (m < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN) return true;
      note_err(to == cfd, errno);
      return false;
    }
    p.off += size_t(m);
  }
  p.off = p.len = 0;
  return true;
}

// Moves bytes from one side to the other until the source is drained or the destination full.
// A FIN is passed on as a half-close once the bytes before it are delivered (a client may
// send its request and shut down its side, then read the response); the session ends when
// both directions are shut. Returns false when the session must close.
bool Session::pump(bool from_client) {
  Pipe& p = from_client ? c2b : b2c;
  const int from = from_client ? cfd : bfd, to = from_client ? bfd : cfd;
  for (;;) {
    if (!flush(p, to)) return false;
    if (p.pending()) return true;  // destination full: wait for its OUT edge
    if (p.eof) {
      if (!p.shut) {
        ::shutdown(to, SHUT_WR);
        p.shut = true;
      }
      return !(c2b.shut && b2c.shut);
    }
    ssize_t n = ::recv(from, p.buf, sizeof p.buf, 0);
    if (n == 0) {
      p.eof = true;
      continue;
    }
    if (n < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN) return true;
      note_err(from_client, errno);
      return false;
    }
    p.len = size_t(n);
    // A short read drained the source, unless this edge also carried its FIN: then read on
    // to the EOF (the edge will not come again).
    if (size_t(n) < sizeof p.buf && !p.hup) return flush(p, to);
  }
}

// First event on a backend socket whose connect was in progress: true once the handshake
// succeeded; on a refusal, marks the backend down and moves the session to the next one.
bool Session::backend_connected(uint32_t ev) {
  int soerr = 0;
  socklen_t sl = sizeof soerr;
  if (getsockopt(bfd, SOL_SOCKET, SO_ERROR, &soerr, &sl) != 0) soerr = errno;
  if (soerr == 0 && !(ev & (EPOLLERR | EPOLLHUP))) {
    connecting = false;
    return true;
  }
  note_connect_fail(soerr ? soerr : ECONNRESET);
  if (g_failover) mark_down(backend, soerr ? soerr : ECONNRESET);
  EventLoop& l = owner->loop();
  l.del(bfd);
  ::close(bfd);
  bfd = -1;
  if (!g_failover || ++failovers > int(current_set().list.size())) return false;
  bool inprog = false;
  bfd = connect_backend(&backend, &inprog, owner->l3(), owner->rr());
  if (bfd < 0) return false;
  connecting = inprog;
  l.add(bfd, ProxyLoop::kEvents, &bside);
  return !connecting;  // connected at once: carry on; else wait for the new socket's edge
}

void Session::on_event(bool client_side, uint32_t ev) {
  if (closed) return;
  last_active_ms = owner->loop().now_ms();
  if (connecting) {
    // The client is not read until the backend accepted, so a refusal can still fail over.
    if (client_side) {
      if (ev & (EPOLLRDHUP | EPOLLHUP)) c2b.hup = true;
      if (ev & EPOLLERR) {
        note_err(true, socket_error(cfd));
        close();
      }
      return;
    }
    if (!(ev & (EPOLLOUT | EPOLLERR | EPOLLHUP))) return;
    if (!backend_connected(ev)) {
      if (bfd < 0) close();
      return;  // closed, or waiting for the next backend's handshake
    }
    // What the client sent meanwhile, then anything the backend already sent.
    if (!pump(true) || ((ev & (EPOLLIN | EPOLLRDHUP)) && !pump(false))) close();
    return;
  }
  bool ok = !(ev & EPOLLERR);
  if (!ok) note_err(client_side, socket_error(client_side ? cfd : bfd));
  // Writable: deliver what was parked for this side, then read the other side again (it
  // was not read while the bytes waited).
  if (ok && (ev & EPOLLOUT)) {
    Pipe& into = client_side ? b2c : c2b;
    if (into.pending()) {
      ok = flush(into, client_side ? cfd : bfd);
      if (ok && !into.pending()) ok = pump(!client_side);
    }
  }
  if (ev & (EPOLLRDHUP | EPOLLHUP)) (client_side ? c2b : b2c).hup = true;
  if (ok && (ev & (EPOLLIN | EPOLLRDHUP | EPOLLHUP))) ok = pump(client_side);
  if (!ok) close();
}

void Session::close() {
  if (closed) return;
  closed = true;
  g_close.sessions.fetch_add(1, std::memory_order_relaxed);
  if (err) {
    (err_client ? g_close.client_err : g_close.backend_err).fetch_add(1, std::memory_order_relaxed);
    (err_client ? g_close.client_errno : g_close.backend_errno).store(err, std::memory_order_relaxed);
  }
  EventLoop& l = owner->loop();
  l.del(cfd);
  ::close(cfd);
  if (bfd >= 0) {
    l.del(bfd);
    ::close(bfd);
  }
  owner->sessions().fetch_sub(1, std::memory_order_relaxed);
  owner->unlink(this);
  l.retire(this);  // the other side's event may still be in this batch
}

void ProxyLoop::close_all() {
  while (head_) head_->close();
}

// Accepts on one listener (on loop 0) and deals each connection to a loop in the client's L3
// domain, least-loaded first, falling back to plain round-robin.
struct Acceptor : EventLoop::Handler {
  int fd = -1;
  std::vector<std::unique_ptr<ProxyLoop>>* loops = nullptr;
  bool steer = true;
  bool paused = false;  // accepts are paused at the fd limit (logged once per episode)
  uint64_t rr = 0;

  ProxyLoop* choose(int cfd) {
    auto& ls = *loops;
    ProxyLoop* best = nullptr;
    if (steer) {
      int cpu = -1;
      socklen_t len = sizeof cpu;
      if (getsockopt(cfd, SOL_SOCKET, SO_INCOMING_CPU, &cpu, &len) == 0 && cpu >= 0) {
        const int dom = l3_domain_of(cpu);
        for (auto& l : ls) {
          if (l->cpu() < 0 || l3_domain_of(l->cpu()) != dom) continue;
          if (!best || l->sessions().load(std::memory_order_relaxed) < best->sessions().load(std::memory_order_relaxed))
            best = l.get();
        }
      }
    }
    if (!best) best = ls[rr++ % ls.size()].get();
    return best;
  }

  void on_event(uint32_t) override {
    for (int i = 0; i < 256; ++i) {
      int c = ::accept4(fd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
      if (c < 0) {
        if (errno == EINTR || errno == ECONNABORTED) continue;
        if (errno == EMFILE || errno == ENFILE) {
          // The listener is level-triggered: leaving it armed at the fd limit would spin
          // loop 0. Disarm it and retry in 50 ms (hola's server does the same).
          if (!paused) fprintf(stderr, "rrproxy: accept: %s (fd limit); pausing accepts\n", strerror(errno));
          paused = true;
          EventLoop& l = (*loops)[0]->loop();
          l.del(fd);
          l.add_timer(50, [this, &l] {
            if (!g_stop.load()) l.add(fd, EPOLLIN, this);
          });
        }
        return;
      }
      paused = false;
      set_nodelay(c);
      ProxyLoop* l = choose(c);
      l->sessions().fetch_add(1, std::memory_order_relaxed);
      if (l == (*loops)[0].get()) l->adopt_here(c);
      else l->adopt(c);
    }
  }
};

void health_loop(int interval_ms) {
  while (!g_stop.load()) {
    for (Backend* b : current_set().list) {
      client::Url u;
      u.host = b->host;
      u.port = b->port;
      int fd = -1;
      client::BlockingResponse r;
      errno = 0;
      bool ok = client::blocking_request(u, &fd, "GET", "/api/health", "", "", 1000, &r) && r.status == 200;
      const int err = errno;
      if (fd >= 0) ::close(fd);
      if (!ok && is_local_resource_error(err)) continue;  // local, not the backend
      bool was = b->healthy.exchange(ok);
      if (was != ok) fprintf(stderr, "rrproxy: backend %s:%d is %s\n", b->host.c_str(), b->port, ok ? "UP" : "DOWN");
    }
    for (int w = 0; w < interval_ms && !g_stop.load(); w += 20) std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

}  // namespace

int main(int argc, char** argv) {
  int port = 8080, threads = 1, health_ms = 500, busy_poll_us = 0, busy_poll_pause = 0, idle_timeout_ms = 60000;
  bool steer = true;
  std::string backends, cpu_list, host = "0.0.0.0", port_file, endpoints_file;
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
    else if (a == "--busy-poll-us") busy_poll_us = atoi(val().c_str());
    else if (a == "--busy-poll-pause") busy_poll_pause = atoi(val().c_str());
    else if (a == "--no-steer") steer = false;
    else if (a == "--idle-timeout-ms") idle_timeout_ms = atoi(val().c_str());
    else if (a == "--endpoints-file") endpoints_file = val();
    else if (a == "--no-failover") g_failover = false;
    else if (a == "--version") {
      printf("hola_rrproxy %s (revision %s, %s)\n", hola::build_info::version(), hola::build_info::revision(),
             hola::isa::build_level());
      return 0;
    }
    else {
      fprintf(stderr,
              "usage: hola_rrproxy --backends h:p,h:p.. [--port N] [--host H] [--threads N] [--cpu-list L]\n"
              "                    [--health-ms N] [--busy-poll-us N [--busy-poll-pause P]] [--no-steer] [--port-file F]\n"
              "                    [--idle-timeout-ms N (default 60000, 0 = never)]\n"
              "                    [--endpoints-file F (backend set re-read on change)] [--no-failover]\n"
              "                    (a backend h:p@CPUS names its workers' CPUs: each proxy thread prefers\n"
              "                     the backends in its own L3; ';' separates CPU ranges inside --backends)\n"
              "                    (--health-ms 0: no probing of backends)\n");
      return 2;
    }
  }
  signal(SIGPIPE, SIG_IGN);
  std::vector<Backend*> initial;
  if (!parse_backends(backends, &initial)) return 2;
  if (initial.empty() && endpoints_file.empty()) {
    fprintf(stderr, "rrproxy: --backends or --endpoints-file required\n");
    return 2;
  }
  publish_set(std::move(initial));
  // Read the endpoints before listening (and before the port file says so): a client that
  // connects in between would otherwise meet an empty set and be reset.
  EndpointsFollower follower;
  follower.path = endpoints_file;
  if (!endpoints_file.empty() && !follower.poll())
    fprintf(stderr, "rrproxy: no endpoints in %s yet: connections are closed at once until there are\n",
            endpoints_file.c_str());
  if (threads < 1) threads = 1;
  std::vector<int> cpus;
  if (!cpu_list.empty() && !parse_cpu_list(cpu_list, &cpus)) {
    fprintf(stderr, "rrproxy: bad --cpu-list\n");
    return 2;
  }
  ListenOptions lo;
  lo.host = host;
  lo.port = port;
  std::string err;
  Acceptor acc;
  acc.fd = listen_tcp(lo, &err);
  if (acc.fd < 0) {
    fprintf(stderr, "rrproxy: %s\n", err.c_str());
    return 1;
  }
  lo.port = bound_port(acc.fd);
  if (!port_file.empty()) {
    FILE* f = fopen((port_file + ".tmp").c_str(), "w");
    if (!f) return 1;
    fprintf(f, "%d\n", lo.port);
    fclose(f);
    rename((port_file + ".tmp").c_str(), port_file.c_str());
  }
  fprintf(stderr, "rrproxy: listening on %s:%d -> %zu backends, %d threads\n", host.c_str(), lo.port,
          current_set().list.size(), threads);

  std::vector<std::unique_ptr<ProxyLoop>> loops;
  for (int t = 0; t < threads; ++t)
    loops.push_back(std::make_unique<ProxyLoop>(t, cpus.empty() ? -1 : cpus[size_t(t) % cpus.size()], busy_poll_us,
                                                busy_poll_pause, idle_timeout_ms));
  acc.loops = &loops;
  acc.steer = steer && !cpus.empty();
  loops[0]->loop().add(acc.fd, EPOLLIN, &acc);

  sigset_t sigs;
  sigemptyset(&sigs);
  sigaddset(&sigs, SIGTERM);
  sigaddset(&sigs, SIGINT);
  pthread_sigmask(SIG_BLOCK, &sigs, nullptr);
  std::thread hc;
  if (health_ms > 0) hc = std::thread(health_loop, health_ms);
  std::thread ep;
  if (!endpoints_file.empty()) ep = std::thread([&follower] { follower.loop(); });
  std::vector<std::thread> ws;
  for (auto& l : loops) ws.emplace_back([p = l.get()] { p->run(); });
  int sig;
  sigwait(&sigs, &sig);
  g_stop.store(true);
  for (auto& l : loops) l->loop().stop();
  for (auto& w : ws) w.join();
  if (hc.joinable()) hc.join();
  if (ep.joinable()) ep.join();
  for (auto& l : loops) l->close_all();
  ::close(acc.fd);
  for (auto& b : g_backends)
    fprintf(stderr, "rrproxy: %s:%d picked %llu\n", b->host.c_str(), b->port, (unsigned long long)b->picked.load());
  auto why = [](const std::atomic<uint64_t>& n, const std::atomic<int>& e) {
    return n.load() ? strerror(e.load()) : "-";
  };
  fprintf(stderr,
          "rrproxy: sessions closed %llu; on an error: client side %llu (last %s), backend side %llu (last %s); "
          "backend connects failed %llu (last %s)\n",
          (unsigned long long)g_close.sessions.load(), (unsigned long long)g_close.client_err.load(),
          why(g_close.client_err, g_close.client_errno), (unsigned long long)g_close.backend_err.load(),
          why(g_close.backend_err, g_close.backend_errno), (unsigned long long)g_close.connect_fail.load(),
          why(g_close.connect_fail, g_close.connect_errno));
  return 0;
}
