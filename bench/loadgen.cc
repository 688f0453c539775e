// hola_loadgen — wrk-style closed-loop HTTP/1.1 load generator.
//
// C keep-alive connections spread over T pinned threads; each connection keeps exactly
// one request in flight (no pipelining, like wrk's default) and records send->last-byte
// latency in a log-linear histogram. `--pipeline P` sends P requests back to back in one
// write and waits for all P responses (wrk's pipeline.lua, the TechEmpower "plaintext"
// setup); each response's latency is counted from the batch's send. Connections are dealt round-robin over --targets
// (client-side round-robin across replicas, BASELINE.json config 4).
//
// Modes:
//   --duration S [--warmup S]   timed run, prints one JSON line (rps, p50/p90/p99/p99.9)
//   --duration S --rate R       open loop at R req/s total (wrk2-style): latency counted from
//                               each request's intended send time (no coordinated omission)
//   --control                   stdin protocol used by bench.py:
//        run <R>     every connection completes exactly R requests; replies
//                    {"elapsed_ns":..,"requests":..,"errors":..}
//        runfor <MS> [<WARM_MS>]
//                    every connection sends back to back for WARM_MS + MS milliseconds, then
//                    finishes the request it has in flight; only responses after the first
//                    WARM_MS count (requests, errors, latency, bodies), and elapsed_ns covers
//                    that part: warm-up and measurement are one continuous run, where a
//                    series of `run`s leaves every connection idle between them
//        stats       {"count":..,"p50_ns":..,...,"hist":"bin:count,..."} (since last reset)
//        reset       clears the histogram
//        quit
//
// Response bodies are verified against --expect-body (one per target in --targets order, or
// one for all) and/or, with --verify-body, against the first 2xx body each thread sees from
// each target; a mismatch counts as an error (and in "body_mismatch"), so a server that
// answers fast with the wrong bytes cannot inflate req/s. --alt-body B names an accepted
// second answer (e.g. the chaining endpoint's Hystrix fallback body): a response equal to it
// is counted in "body_alt" instead of as a mismatch, so a run reports how many of each came.
//
// Service mode (`--endpoints-file F`): the load generator addresses a Kubernetes Service (the
// --targets / URL address, used in the Host header) and each new connection is DNATed at
// connect time to one of the Service's current endpoints, read from F (the file the local
// manifest executor publishes, `ip:port` per line, re-read when it changes). That is what
// kube-proxy's iptables/IPVS modes do in the client's kernel: an established connection keeps
// its pod whatever the endpoints do later, a new one (after `Connection: close`) goes to a
// current endpoint, and there is no failover: a connection refused by a pod that stopped
// listening counts as an error. Endpoints are taken in round-robin order (IPVS `rr`).
//
// wrk-style invocation: `hola_loadgen -t8 -c64 -d30s [--latency] http://host:port/path`
// takes the target from the URL, accepts wrk's duration suffixes (s/m/h) and prints a
// wrk-like text summary (`--json` keeps the JSON line).
#include <errno.h>
#include <netinet/in.h>
#include <pthread.h>
#include <sys/epoll.h>
#include <sys/prctl.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/syscall.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "core/build_info.h"
#include "core/isa.h"
#include "core/cpuprof.h"
#include "core/histogram.h"
#include "core/affinity.h"
#include "core/clock.h"
#include "core/net.h"
#include "core/perfcount.h"
#include "core/scan.h"

using namespace hola;
using hola::Histogram;

namespace {

struct Target {
  std::string host;
  int port;
  sockaddr_storage addr;
  socklen_t len;
};

struct Options {
  std::vector<Target> targets;
  int connections = 64;
  int threads = 1;
  std::vector<int> cpus;
  std::string path = "/api/hola";
  std::string method = "GET";
  double duration_s = 0, warmup_s = 0;
  bool control = false;
  int target_offset = 0;
  std::vector<std::string> extra_headers;
  int busy_poll_us = 0;
  int busy_poll_pause = 0;  // PAUSE instructions between empty polls
  // Edge-triggered connection sockets: a response (<4 KiB) arrives in one read, so a short
  // read drains the socket and no re-poll of level-triggered items is needed.
  bool edge_triggered = true;
  double rate = 0;  // --rate: open-loop total req/s (wrk2-style, latency from intended time)
  bool rx_timestamps = false;  // --rate: kernel receive timestamps (set with --rate)
  int sched_slice_us = 0;  // each thread asks for this scheduler time slice (0 = the kernel's)
  int spin_us = 0;  // --rate: spin instead of sleeping when the next send is this close (burns CPU)
  // control: a run of R requests per connection is R x connections requests drawn from one
  // shared budget (connections that answer faster do more, so no thread idles at the end of
  // a run waiting for a slower one); --per-conn-quota gives each connection exactly R.
  bool per_conn_quota = false;
  int pipeline = 1;  // requests per batch (closed loop only)
  std::vector<std::string> expect_bodies;  // --expect-body: per target, or one for all
  std::vector<std::string> alt_bodies;     // --alt-body: accepted alternatives (counted apart)
  bool verify_body = false;                // --verify-body: learn the first 2xx body per target
  std::vector<int> conn_targets;           // --conn-targets: target index of connection i (cycled)
  std::string endpoints_file;              // --endpoints-file: Service mode (connect-time DNAT)
};

struct Conn {
  int fd = -1;
  int target = 0;
  std::string req;   // one batch: `pipeline` copies of the request
  char buf[16384];  // holds a whole batch of responses
  size_t have = 0;
  int inflight = 0;  // responses still due for the batch in flight
  int64_t t0 = 0;
  int64_t quota = 0;  // remaining requests in control mode
  bool busy = false;
  int64_t next_due = 0;   // --rate: intended send time of the next request
  int64_t intended = 0;   // --rate: intended send time of the in-flight request
  int64_t free_at = 0;    // --rate: when its last response completed (free to send again)
};

// The scheduler's run_delay of one of this process's threads (ns it spent runnable, waiting
// for a CPU another task held); 0 when schedstats are unavailable.
uint64_t run_delay_ns(int tid) {
  if (tid <= 0) return 0;
  char path[64];
  snprintf(path, sizeof path, "/proc/self/task/%d/schedstat", tid);
  FILE* f = fopen(path, "r");
  if (!f) return 0;
  unsigned long long on_cpu = 0, delay = 0;
  const int got = fscanf(f, "%llu %llu", &on_cpu, &delay);
  fclose(f);
  return got == 2 ? uint64_t(delay) : 0;
}

// A counter one polling thread raises and the control thread reads or zeroes between runs.
struct Stat {
  std::atomic<uint64_t> v{0};
  operator uint64_t() const { return v.load(std::memory_order_relaxed); }
  Stat& operator=(uint64_t x) {
    v.store(x, std::memory_order_relaxed);
    return *this;
  }
  void operator++() { v.fetch_add(1, std::memory_order_relaxed); }
  void operator+=(uint64_t d) { v.fetch_add(d, std::memory_order_relaxed); }
  void raise(uint64_t x) {
    if (x > v.load(std::memory_order_relaxed)) v.store(x, std::memory_order_relaxed);
  }
};

struct ThreadState {
  int index = 0;
  int epfd = -1;
  int wakefd = -1;
  std::vector<int> conn_ids;  // connection i goes to target (i + offset) % targets
  std::vector<std::unique_ptr<Conn>> conns;
  Histogram hist;
  // --rate: service time of each response, from its send() to its arrival in this host's
  // kernel (receive timestamp): what the server and the network took, with none of this
  // generator's own delays (a late send, a late read) in it
  Histogram svc;
  std::mutex hist_mu;
  uint64_t completed = 0, errors = 0, non2xx = 0, reconnects = 0, bytes = 0;
  uint64_t body_checked = 0, body_mismatch = 0, body_alt = 0;
  // Where the thread's time goes (since the last reset; read between runs): polls that found
  // work at once / after spinning / spins that ran out, waits that could block, CPU spent in
  // empty polls, gaps between polls (event handling + descheduling) past 100 us / 1 ms /
  // 10 ms and the longest, and (open loop) the latest a scheduled send went out.
  // These are read ("stats") and zeroed ("reset") by the control thread while the thread may
  // still be polling, so each is a relaxed atomic: counts are exact, a maximum raised in the
  // same instant as a reset may survive it.
  Stat poll_hits, spin_hits, spin_misses, blocking_waits, idle_spin_ns;
  // send_late: a scheduled request sent late although its connection was free at the due
  // time (this generator's own delay); behind: late because the connection was still waiting
  // for the server's previous response (the server's delay, passed on)
  Stat gaps_over[3], gap_max_ns, send_late_max_ns, behind_max_ns, sends_late_1ms;
  // the thread's own user-space instructions and cycles (hardware counters, where allowed),
  // counted from the last reset
  ThreadCounters pmu;
  Stat pmu_ins0, pmu_cyc0;
  // time the thread was runnable but waiting for its CPU (the scheduler's run_delay: another
  // task held the CPU), counted from the last reset
  std::atomic<int> tid{0};
  Stat run_delay0, run_delay_last;
  void sched_reset() { run_delay0 = run_delay_ns(tid.load(std::memory_order_relaxed)); }
  void pmu_reset() {
    uint64_t i = 0, c = 0;
    if (!pmu.read(&i, &c)) return;
    pmu_ins0 = i;
    pmu_cyc0 = c;
  }
  void note_gap(int64_t ns) {
    if (ns <= 100000) return;
    ++gaps_over[0];
    if (ns > 1000000) ++gaps_over[1];
    if (ns > 10000000) ++gaps_over[2];
    gap_max_ns.raise(uint64_t(ns));
  }
  std::vector<std::string> expected;  // per target: the body every response must carry
  std::vector<bool> have_expected;
  std::atomic<int64_t> run_quota{0};  // control: batches per connection for the next run
  std::atomic<uint64_t> run_gen{0};
  std::atomic<uint64_t> done_gen{0};
  std::atomic<uint64_t> done_requests{0}, done_errors{0};
  bool recording = true;
};

std::atomic<bool> g_stop{false};
std::atomic<int64_t> g_budget{0};  // control, shared mode: requests left in this run
// control `runfor` with a warm-up: responses that arrive before this time (mono ns) are not
// counted (0 = count all)
std::atomic<int64_t> g_count_from{0};
int g_donefd = -1;  // EFD_SEMAPHORE: one count per thread finishing a control run
std::atomic<bool> g_connect_failed{false};
char g_connect_error[256];

void signal_done() {
  uint64_t one = 1;
  ssize_t w = ::write(g_donefd, &one, sizeof one);
  (void)w;
}

// Service mode: the endpoints of the Service as last published, and every endpoint ever seen
// (its index is the connection's `target`, so bodies are checked per pod).
struct Dnat {
  std::mutex mu;
  std::string path;
  std::string text;  // the file as last read
  std::vector<Target> all;
  std::map<std::string, int> ids;
  std::vector<int> current;
  uint64_t rr = 0;

  // Read at every new connection and compared by content: a replacement (by rename) can keep
  // the inode number, the size and the coarse mtime of the file before it.
  void reload_locked() {
    std::ifstream f(path);
    if (!f) {
      current.clear();
      text.clear();
      return;
    }
    std::string now((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    if (now == text) return;
    text = now;
    std::vector<int> next;
    size_t at = 0;
    while (at < now.size()) {
      size_t eol = now.find('\n', at);
      if (eol == std::string::npos) eol = now.size();
      std::string line = now.substr(at, eol - at);
      at = eol + 1;
      while (!line.empty() && isspace((unsigned char)line.back())) line.pop_back();
      if (line.empty() || line[0] == '#') continue;
      auto it = ids.find(line);
      if (it == ids.end()) {
        const size_t colon = line.rfind(':');
        if (colon == std::string::npos) continue;
        Target t;
        t.host = line.substr(0, colon);
        if (t.host.size() > 2 && t.host.front() == '[') t.host = t.host.substr(1, t.host.size() - 2);
        t.port = atoi(line.c_str() + colon + 1);
        if (!resolve_host(t.host, t.port, &t.addr, &t.len, nullptr)) continue;
        it = ids.emplace(line, int(all.size())).first;
        all.push_back(t);
      }
      next.push_back(it->second);
    }
    current.swap(next);
  }
  // The next endpoint for a new connection; false when the Service has none.
  bool pick(Target* out, int* id) {
    std::lock_guard<std::mutex> g(mu);
    reload_locked();
    if (current.empty()) return false;
    *id = current[rr++ % current.size()];
    *out = all[size_t(*id)];
    return true;
  }
  size_t seen() {
    std::lock_guard<std::mutex> g(mu);
    return all.size();
  }
};
Dnat g_dnat;

bool connect_once(Conn* c, const Options& o) {
  Target picked;
  const Target* tp = nullptr;
  if (!o.endpoints_file.empty()) {
    int id = 0;
    if (!g_dnat.pick(&picked, &id)) {
      errno = EHOSTUNREACH;  // a Service without endpoints (kube-proxy rejects it)
      return false;
    }
    c->target = id;
    tp = &picked;
  } else {
    tp = &o.targets[size_t(c->target)];
  }
  const Target& t = *tp;
  c->fd = connect_blocking(t.addr, t.len, 1000);
  if (c->fd < 0) return false;
  set_nonblocking(c->fd, true);
  set_nodelay(c->fd);
  if (o.rx_timestamps) {
    // the kernel stamps each segment as it arrives: a response's arrival is then known even
    // when this thread reads it late (the service time below)
    const int one = 1;
    setsockopt(c->fd, SOL_SOCKET, SO_TIMESTAMPNS, &one, sizeof one);
  }
  c->have = 0;
  c->busy = false;
  return true;
}

// Reconnect after a failure: like a client-side load balancer, fail over to the next
// target when the current one refuses, retrying for up to ~5 s (a replica restart). In
// Service mode every attempt is DNATed afresh, and each failed one is a client-visible
// connection error (`*failed`): there is no failover below the Service.
bool connect_conn(Conn* c, const Options& o, uint64_t* failed = nullptr) {
  const int n = int(o.targets.size());
  const bool dnat = !o.endpoints_file.empty();
  for (int attempt = 0; attempt < 100; ++attempt) {
    if (connect_once(c, o)) return true;
    if (dnat) {
      if (failed && errno != EHOSTUNREACH) ++*failed;
      usleep(errno == EHOSTUNREACH ? 50000 : 1000);
      continue;
    }
    c->target = (c->target + 1) % n;
    if ((attempt + 1) % n == 0) usleep(50000);
  }
  return false;
}

bool send_req(Conn* c, int depth) {
  c->t0 = mono_ns();
  c->busy = true;
  c->have = 0;
  c->inflight = depth;
  size_t off = 0;
  while (off < c->req.size()) {
    ssize_t w = ::send(c->fd, c->req.data() + off, c->req.size() - off, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN) continue;  // tiny request; socket buffer is never full here
      return false;
    }
    off += size_t(w);
  }
  return true;
}

// Returns 1 when a full response starts at buf[from] (its size in *used), 0 if more is
// needed, -1 on malformed input.
// Case-insensitive prefix test against a lower-case literal (letters, digits, '-', ':'; all
// fixed by OR 0x20), eight bytes at a time: the per-byte loop was most of this load
// generator's own instructions per response (profiles/round4/11_instr).
template <size_t N>
inline bool iprefix(const char* p, size_t n, const char (&lower)[N]) {
  constexpr size_t k = N - 1;
  if (n < k) return false;
  auto word = [](const char* q, size_t m) {
    uint64_t w = 0;
    memcpy(&w, q, m);
    return w;
  };
  constexpr uint64_t kFold = 0x2020202020202020ull;
  if constexpr (k <= 8) {
    const uint64_t mask = k == 8 ? kFold : kFold & ((uint64_t(1) << (8 * k)) - 1);
    return (word(p, k) | mask) == word(lower, k);
  } else {
    for (size_t off = 0; off + 8 < k; off += 8)
      if ((word(p + off, 8) | kFold) != word(lower + off, 8)) return false;
    return (word(p + k - 8, 8) | kFold) == word(lower + k - 8, 8);
  }
}

// Returns 1 when a full response starts at buf[from] (its size in *used), 0 if more is
// needed, -1 on malformed input. One pass over the head's lines: the status line, then
// Content-Length and Connection, up to the empty line.
int response_complete(Conn* c, size_t from, int* status, bool* close, size_t* used, size_t* body_at) {
  const char* s = c->buf + from;
  const size_t n = c->have - from;
  auto incomplete = [&] { return (from == 0 && c->have >= sizeof c->buf) ? -1 : 0; };  // head > buf
  const char* nl = hola::find_newline(s, n);
  if (!nl) return incomplete();
  if (nl - s < 12 || memcmp(s, "HTTP/", 5) != 0) return -1;
  *status = (s[9] - '0') * 100 + (s[10] - '0') * 10 + (s[11] - '0');
  *close = false;
  size_t cl = 0, p = size_t(nl - s) + 1;
  for (;;) {
    const char* line = s + p;
    const char* e = hola::find_newline(line, n - p);
    if (!e) return incomplete();
    size_t len = size_t(e - line);
    p += len + 1;
    if (len && line[len - 1] == '\r') --len;
    if (len == 0) break;  // end of head
    if ((line[0] | 0x20) != 'c') continue;
    if (iprefix(line, len, "content-length:")) {
      size_t i = 15;
      while (i < len && line[i] == ' ') ++i;
      for (; i < len && line[i] >= '0' && line[i] <= '9'; ++i) cl = cl * 10 + size_t(line[i] - '0');
    } else if (iprefix(line, len, "connection:")) {
      size_t i = 11;
      while (i < len && line[i] == ' ') ++i;
      *close = iprefix(line + i, len - i, "close");
    }
  }
  if (p + cl > sizeof c->buf) return -1;
  *used = p + cl;
  *body_at = from + p;
  return n >= *used ? 1 : 0;
}

void thread_main(ThreadState* ts, const Options* o) {
  if (!o->cpus.empty()) pin_current_thread(o->cpus[size_t(ts->index) % o->cpus.size()]);
  {
    char name[16];
    snprintf(name, sizeof name, "hola-lg%d", ts->index);
    pthread_setname_np(pthread_self(), name);
  }
  hola::cpuprof::register_thread();
  ts->tid.store(int(syscall(SYS_gettid)), std::memory_order_relaxed);
  if (o->sched_slice_us > 0 && hola::set_current_thread_slice_us(o->sched_slice_us) < 0)
    fprintf(stderr, "loadgen: could not set a %d us time slice\n", o->sched_slice_us);
  ts->sched_reset();
  if (ts->pmu.open()) ts->pmu_reset();
  // Connections (and their receive buffers) are built here, after pinning, so their pages
  // are first touched on this thread's NUMA node: on a 2-socket node a thread may drive a
  // replica on the other socket from main()'s.
  for (int i : ts->conn_ids) {
    auto c = std::make_unique<Conn>();
    c->target = o->conn_targets.empty() ? (i + o->target_offset) % int(o->targets.size())
                                        : o->conn_targets[size_t(i) % o->conn_targets.size()];
    const Target& t = o->targets[size_t(c->target)];  // Service mode: the Service's address
    const bool v6 = t.host.find(':') != std::string::npos;  // RFC 3986 IP-literal in Host
    c->req = o->method + " " + o->path + " HTTP/1.1\r\nHost: " + (v6 ? "[" + t.host + "]" : t.host) + ":" +
             std::to_string(t.port) + "\r\n";
    for (auto& h : o->extra_headers) c->req += h + "\r\n";
    c->req += "\r\n";
    const std::string one = c->req;
    for (int k = 1; k < o->pipeline; ++k) c->req += one;
    ts->conns.push_back(std::move(c));
  }
  const bool verify = o->verify_body || !o->expect_bodies.empty();
  ts->expected.assign(o->targets.size(), std::string());
  ts->have_expected.assign(o->targets.size(), false);
  for (size_t k = 0; k < o->targets.size(); ++k) {
    const size_t e = o->expect_bodies.size() == 1 ? 0 : k;
    if (e >= o->expect_bodies.size()) continue;  // learned with --verify-body, or unchecked
    ts->expected[k] = o->expect_bodies[e];
    ts->have_expected[k] = true;
  }
  const bool dnat = !o->endpoints_file.empty();
  for (auto& c : ts->conns) {
    if (!(dnat ? connect_conn(c.get(), *o) : connect_once(c.get(), *o))) {
      const Target& t = o->targets[dnat ? 0 : size_t(c->target)];
      if (!g_connect_failed.exchange(true))
        snprintf(g_connect_error, sizeof g_connect_error, "connect %s:%d failed: %s", t.host.c_str(), t.port,
                 strerror(errno));
      signal_done();
      return;
    }
  }
  signal_done();
  epoll_event ev{};
  const uint32_t conn_events = EPOLLIN | (o->edge_triggered ? uint32_t(EPOLLET) : 0u);
  for (auto& c : ts->conns) {
    ev.events = conn_events;
    ev.data.ptr = c.get();
    epoll_ctl(ts->epfd, EPOLL_CTL_ADD, c->fd, &ev);
  }
  ev.events = EPOLLIN;
  ev.data.ptr = nullptr;
  epoll_ctl(ts->epfd, EPOLL_CTL_ADD, ts->wakefd, &ev);

  const bool control = o->control;
  uint64_t seen_gen = 0;
  int64_t outstanding = 0;  // control: connections with quota left
  uint64_t run_requests = 0, run_errors = 0;
  // Shared-budget claims are taken in batches so threads rarely touch the global counter.
  constexpr int64_t kClaimBatch = 32;
  int64_t local_claims = 0;
  const bool shared = control && !o->per_conn_quota;
  auto claim = [&]() -> bool {
    if (local_claims > 0) {
      --local_claims;
      return true;
    }
    int64_t before = g_budget.fetch_sub(kClaimBatch, std::memory_order_relaxed);
    if (before <= 0) return false;
    local_claims = std::min(kClaimBatch, before) - 1;
    return true;
  };
  int64_t warm_end = o->duration_s > 0 ? mono_ns() + int64_t(o->warmup_s * 1e9) : 0;
  int64_t end = o->duration_s > 0 ? warm_end + int64_t(o->duration_s * 1e9) : 0;
  ts->recording = !(o->warmup_s > 0);

  auto start_all = [&]() {
    for (auto& c : ts->conns) {
      if (c->busy || c->quota <= 0) continue;
      if (!send_req(c.get(), o->pipeline)) ++ts->errors;
    }
  };
  // --rate (open loop): connection k of this thread sends every `interval` ns on a fixed
  // schedule; latency is measured from the *intended* send time, so a stalled server is
  // charged for the requests it delayed (no coordinated omission).
  const bool rate_mode = !control && o->rate > 0;
  const int64_t interval = rate_mode ? int64_t(double(o->connections) * 1e9 / o->rate) : 0;
  if (rate_mode) {
    prctl(PR_SET_TIMERSLACK, 1UL, 0, 0, 0);  // precise wake-ups for the send schedule
    int64_t t0 = mono_ns();
    size_t k = 0;
    for (auto& c : ts->conns) {
      c->quota = INT64_MAX;
      c->next_due = t0 + interval * int64_t(k++) / int64_t(ts->conns.size());
    }
  } else if (!control) {
    for (auto& c : ts->conns) c->quota = INT64_MAX;
    start_all();
  }
  auto send_due = [&](int64_t now) -> int64_t {  // returns ns until the next due send
    int64_t wait = INT64_MAX;
    for (auto& c : ts->conns) {
      if (c->busy) continue;
      if (c->next_due <= now) {
        // late by the time since it was both due and free: the generator's own delay
        const int64_t own = now - std::max(c->next_due, c->free_at);
        ts->send_late_max_ns.raise(uint64_t(own));
        if (own > 1000000) ++ts->sends_late_1ms;
        if (c->free_at > c->next_due) ts->behind_max_ns.raise(uint64_t(c->free_at - c->next_due));
        c->intended = c->next_due;
        c->next_due += interval;
        if (!send_req(c.get(), o->pipeline)) ++ts->errors;
      } else {
        wait = std::min(wait, c->next_due - now);
      }
    }
    return wait;
  };

  epoll_event evs[256];
  int64_t pass_at = mono_ns();  // when the last pass's events began to be handled
  while (!g_stop.load(std::memory_order_relaxed)) {
    int n = 0;
    if (o->busy_poll_us > 0) {
      const int64_t spin0 = mono_ns(), until = spin0 + int64_t(o->busy_poll_us) * 1000;
      ts->note_gap(spin0 - pass_at);
      int64_t t = spin0;
      bool spun = false;
      for (;;) {
        n = epoll_wait(ts->epfd, evs, 256, 0);
        if (n != 0) break;
        spun = true;
        const int64_t prev = t;
        t = mono_ns();
        ts->note_gap(t - prev);  // descheduled while spinning
        if (t >= until) break;
        for (int k = 0; k < o->busy_poll_pause; ++k) __builtin_ia32_pause();
      }
      if (spun) ts->idle_spin_ns += uint64_t(t - spin0);
      if (n > 0) {
        if (spun) ++ts->spin_hits;
        else ++ts->poll_hits;
      }
      else ++ts->spin_misses;
    } else {
      ts->note_gap(mono_ns() - pass_at);
    }
    if (n == 0) {
      if (rate_mode) {
        int64_t wait = send_due(mono_ns());
        if (wait <= int64_t(o->spin_us) * 1000) {
          // The next send is close: poll instead of sleeping, so the schedule is kept to
          // within a few microseconds (a timer sleep + wake-up costs more than the gap).
          n = epoll_wait(ts->epfd, evs, 256, 0);
        } else {
          wait -= int64_t(o->spin_us) * 1000;  // wake early, then spin the rest
          if (wait > 5000000) wait = 5000000;
          timespec tmo{0, long(wait)};
          n = epoll_pwait2(ts->epfd, evs, 256, &tmo, nullptr);
          ++ts->blocking_waits;
        }
      } else {
        n = epoll_wait(ts->epfd, evs, 256, control ? -1 : 5);
        ++ts->blocking_waits;
      }
    }
    int64_t now = mono_ns();
    pass_at = now;
    if (!control) {
      if (!ts->recording && now >= warm_end) {
        std::lock_guard<std::mutex> g(ts->hist_mu);
        ts->hist.reset();
        ts->svc.reset();
        ts->completed = 0;
        ts->recording = true;
        // the time accounting covers the measured part too
        ts->pmu_reset();
        ts->sched_reset();
        for (Stat* x : {&ts->poll_hits, &ts->spin_hits, &ts->spin_misses, &ts->blocking_waits, &ts->idle_spin_ns,
                        &ts->gaps_over[0], &ts->gaps_over[1], &ts->gaps_over[2], &ts->gap_max_ns,
                        &ts->send_late_max_ns, &ts->behind_max_ns, &ts->sends_late_1ms})
          *x = 0;
      }
      if (now >= end) break;
    }
    for (int i = 0; i < n; ++i) {
      Conn* c = static_cast<Conn*>(evs[i].data.ptr);
      if (!c) {  // control wake-up
        uint64_t v;
        while (::read(ts->wakefd, &v, sizeof v) > 0) {
        }
        uint64_t g = ts->run_gen.load();
        if (g != seen_gen) {
          seen_gen = g;
          int64_t q = ts->run_quota.load();
          outstanding = 0;
          run_requests = run_errors = 0;
          local_claims = 0;
          for (auto& cc : ts->conns) {
            cc->quota = shared ? (claim() ? 1 : 0) : q;  // shared: 1 = holds a claimed request
            if (cc->quota > 0) ++outstanding;
          }
          if (outstanding == 0) {
            ts->done_requests.store(0);
            ts->done_errors.store(0);
            ts->done_gen.store(seen_gen);
            signal_done();
          }
          start_all();
        }
        continue;
      }
      ssize_t r;
      int64_t rx_kernel = 0;  // CLOCK_MONOTONIC ns of the data's arrival (0 = unknown)
      if (o->rx_timestamps) {
        iovec iov{c->buf + c->have, sizeof c->buf - c->have};
        alignas(cmsghdr) char cbuf[CMSG_SPACE(sizeof(timespec))];
        msghdr mh{};
        mh.msg_iov = &iov;
        mh.msg_iovlen = 1;
        mh.msg_control = cbuf;
        mh.msg_controllen = sizeof cbuf;
        r = ::recvmsg(c->fd, &mh, 0);
        if (r > 0)
          for (cmsghdr* cm = CMSG_FIRSTHDR(&mh); cm; cm = CMSG_NXTHDR(&mh, cm))
            if (cm->cmsg_level == SOL_SOCKET && cm->cmsg_type == SCM_TIMESTAMPNS) {
              timespec rx;
              memcpy(&rx, CMSG_DATA(cm), sizeof rx);
              // realtime -> monotonic with the two clocks' offset as of now (a slew since the
              // arrival, microseconds ago, is negligible)
              timespec rt, mt;
              clock_gettime(CLOCK_REALTIME, &rt);
              clock_gettime(CLOCK_MONOTONIC, &mt);
              const int64_t off = (int64_t(rt.tv_sec) - int64_t(mt.tv_sec)) * 1000000000 + (rt.tv_nsec - mt.tv_nsec);
              rx_kernel = int64_t(rx.tv_sec) * 1000000000 + rx.tv_nsec - off;
            }
      } else {
        r = ::recv(c->fd, c->buf + c->have, sizeof c->buf - c->have, 0);
      }
      if (r <= 0) {
        if (r < 0 && (errno == EAGAIN || errno == EINTR)) continue;
        // peer closed: reconnect and retry
        epoll_ctl(ts->epfd, EPOLL_CTL_DEL, c->fd, nullptr);
        ::close(c->fd);
        ++ts->errors;
        ++run_errors;
        ++ts->reconnects;
        if (!connect_conn(c, *o, &ts->errors)) {
          g_stop.store(true);
          signal_done();
          break;
        }
        ev.events = conn_events;
        ev.data.ptr = c;
        epoll_ctl(ts->epfd, EPOLL_CTL_ADD, c->fd, &ev);
        if (c->quota > 0 && !send_req(c, o->pipeline)) ++ts->errors;
        continue;
      }
      c->have += size_t(r);
      bool close = false;
      const int64_t now_rx = mono_ns();
      // a `runfor` warm-up: the responses go uncounted, the connections stay busy
      const bool live = !control || now_rx >= g_count_from.load(std::memory_order_relaxed);
      const bool rec = ts->recording && live;
      if (rec) ts->bytes += uint64_t(r);
      size_t at = 0;  // responses are consumed in place; what is left moves down once
      for (;;) {  // every complete response in the buffer (several when pipelining)
        int status = 0;
        size_t used = 0, body_at = 0;
        int rc = response_complete(c, at, &status, &close, &used, &body_at);
        if (rc == 0) break;
        if (rc < 0) {
          ++ts->errors;
          ++run_errors;
          close = true;
          break;
        }
        int64_t lat = now_rx - (rate_mode ? c->intended : c->t0);
        // (the histogram is only read between control runs / after the run: no lock)
        if (rec) {
          ts->hist.add(uint64_t(lat));
          ++ts->completed;
          if (rx_kernel > c->t0) ts->svc.add(uint64_t(rx_kernel - c->t0));
        }
        if (status < 200 || status > 299) {
          if (live) ++ts->non2xx;
        } else if (verify) {
          const size_t t = size_t(c->target);
          if (t >= ts->expected.size()) {  // Service mode: an endpoint first seen since start-up
            ts->expected.resize(t + 1);
            ts->have_expected.resize(t + 1, false);
            if (o->expect_bodies.size() == 1)
              for (size_t k = 0; k <= t; ++k)
                if (!ts->have_expected[k]) {
                  ts->expected[k] = o->expect_bodies[0];
                  ts->have_expected[k] = true;
                }
          }
          const size_t blen = at + used - body_at;
          if (!ts->have_expected[t]) {
            ts->expected[t].assign(c->buf + body_at, blen);
            ts->have_expected[t] = true;
          } else if (blen != ts->expected[t].size() || memcmp(c->buf + body_at, ts->expected[t].data(), blen) != 0) {
            bool alt = false;
            for (const auto& b : o->alt_bodies)
              if (blen == b.size() && memcmp(c->buf + body_at, b.data(), blen) == 0) alt = true;
            if (alt) {
              if (rec) ++ts->body_alt;
            } else {
              if (rec) ++ts->body_mismatch;
              if (live) {
                ++ts->errors;
                ++run_errors;
              }
            }
          }
          if (rec) ++ts->body_checked;
        }
        if (live) ++run_requests;
        --c->inflight;
        at += used;
        if (close || c->inflight <= 0) break;
      }
      if (at) {
        c->have -= at;
        if (c->have) memmove(c->buf, c->buf + at, c->have);
      }
      if (!close && c->inflight > 0) continue;  // the rest of the batch is still due
      c->busy = false;
      // free since the response arrived (its kernel timestamp when known): a late read is
      // this generator's delay, not the server's
      c->free_at = rx_kernel > 0 && rx_kernel <= now_rx ? rx_kernel : now_rx;
      if (close) {
        epoll_ctl(ts->epfd, EPOLL_CTL_DEL, c->fd, nullptr);
        ::close(c->fd);
        ++ts->reconnects;
        if (!connect_conn(c, *o, &ts->errors)) {
          g_stop.store(true);
          signal_done();
          break;
        }
        ev.events = conn_events;
        ev.data.ptr = c;
        epoll_ctl(ts->epfd, EPOLL_CTL_ADD, c->fd, &ev);
      }
      if (control) {
        if (shared) c->quota = claim() ? 1 : 0;
        else --c->quota;
        if (c->quota <= 0) {
          if (--outstanding == 0) {
            ts->done_requests.store(run_requests);
            ts->done_errors.store(run_errors);
            ts->done_gen.store(seen_gen);
            signal_done();
          }
          continue;
        }
      }
      if (rate_mode) continue;  // the schedule decides when this connection sends next
      if (!send_req(c, o->pipeline)) ++ts->errors;
    }
    if (rate_mode) send_due(mono_ns());
  }
  // the thread's /proc entry goes with it; stats read after the join use this
  ts->run_delay_last = run_delay_ns(ts->tid.load(std::memory_order_relaxed));
}

bool parse_targets(const std::string& s, std::vector<Target>* out) {
  size_t i = 0;
  while (i < s.size()) {
    size_t j = s.find(',', i);
    if (j == std::string::npos) j = s.size();
    std::string t = s.substr(i, j - i);
    i = j + 1;
    size_t colon = t.rfind(':');
    if (colon == std::string::npos) return false;
    Target tg;
    tg.host = t.substr(0, colon);
    tg.port = atoi(t.substr(colon + 1).c_str());
    std::string err;
    if (!resolve_host(tg.host, tg.port, &tg.addr, &tg.len, &err)) {
      fprintf(stderr, "loadgen: %s\n", err.c_str());
      return false;
    }
    out->push_back(tg);
  }
  return !out->empty();
}

std::string stats_json(std::vector<std::unique_ptr<ThreadState>>& ts, bool with_hist) {
  Histogram h, svc;
  uint64_t errors = 0, non2xx = 0, reconnects = 0, checked = 0, mismatch = 0, alt = 0;
  uint64_t poll_hits = 0, spin_hits = 0, spin_misses = 0, sleeps = 0, idle_ns = 0, gmax = 0, late = 0, behind = 0,
           late_1ms = 0;
  uint64_t over[3] = {}, u_ins = 0, u_cyc = 0, rdelay = 0, rdelay_max = 0;
  bool pmu = false;
  for (auto& t : ts) {
    uint64_t a = 0, b = 0;
    if (t->pmu.read(&a, &b)) {
      pmu = true;
      u_ins += a - t->pmu_ins0;
      u_cyc += b - t->pmu_cyc0;
    }
    if (const int tid = t->tid.load(std::memory_order_relaxed); tid > 0) {
      uint64_t now_rd = run_delay_ns(tid);
      if (!now_rd) now_rd = t->run_delay_last;
      const uint64_t base = t->run_delay0;
      const uint64_t d = now_rd > base ? now_rd - base : 0;
      rdelay += d;
      rdelay_max = std::max(rdelay_max, d);
    }
    std::lock_guard<std::mutex> g(t->hist_mu);
    h.merge(t->hist);
    svc.merge(t->svc);
    errors += t->errors;
    non2xx += t->non2xx;
    reconnects += t->reconnects;
    checked += t->body_checked;
    mismatch += t->body_mismatch;
    alt += t->body_alt;
    poll_hits += t->poll_hits;
    spin_hits += t->spin_hits;
    spin_misses += t->spin_misses;
    sleeps += t->blocking_waits;
    idle_ns += t->idle_spin_ns;
    gmax = std::max<uint64_t>(gmax, t->gap_max_ns);
    late = std::max<uint64_t>(late, t->send_late_max_ns);
    behind = std::max<uint64_t>(behind, t->behind_max_ns);
    late_1ms += t->sends_late_1ms;
    for (int k = 0; k < 3; ++k) over[k] += t->gaps_over[k];
  }
  char buf[704];
  snprintf(buf, sizeof buf,
           "{\"count\":%llu,\"mean_ns\":%.0f,\"p50_ns\":%llu,\"p90_ns\":%llu,\"p99_ns\":%llu,\"p999_ns\":%llu,"
           "\"max_ns\":%llu,\"errors\":%llu,\"non2xx\":%llu,\"reconnects\":%llu,\"body_checked\":%llu,"
           "\"body_mismatch\":%llu,\"body_alt\":%llu",
           (unsigned long long)h.count(), h.mean(), (unsigned long long)h.percentile(50),
           (unsigned long long)h.percentile(90), (unsigned long long)h.percentile(99),
           (unsigned long long)h.percentile(99.9), (unsigned long long)h.max(), (unsigned long long)errors,
           (unsigned long long)non2xx, (unsigned long long)reconnects, (unsigned long long)checked,
           (unsigned long long)mismatch, (unsigned long long)alt);
  std::string s = buf;
  snprintf(buf, sizeof buf,
           ",\"poll_hits\":%llu,\"spin_hits\":%llu,\"spin_misses\":%llu,\"blocking_waits\":%llu,"
           "\"idle_spin_ns\":%llu,\"gaps_over_100us\":%llu,\"gaps_over_1ms\":%llu,\"gaps_over_10ms\":%llu,"
           "\"gap_max_ns\":%llu,\"send_late_max_ns\":%llu,\"sends_late_1ms\":%llu,\"behind_max_ns\":%llu,"
           "\"run_delay_ns\":%llu,\"run_delay_max_thread_ns\":%llu",
           (unsigned long long)poll_hits, (unsigned long long)spin_hits, (unsigned long long)spin_misses,
           (unsigned long long)sleeps, (unsigned long long)idle_ns, (unsigned long long)over[0],
           (unsigned long long)over[1], (unsigned long long)over[2], (unsigned long long)gmax,
           (unsigned long long)late, (unsigned long long)late_1ms, (unsigned long long)behind,
           (unsigned long long)rdelay, (unsigned long long)rdelay_max);
  s += buf;
  if (svc.count()) {
    snprintf(buf, sizeof buf,
             ",\"service_count\":%llu,\"service_p50_ns\":%llu,\"service_p99_ns\":%llu,\"service_p999_ns\":%llu,"
             "\"service_max_ns\":%llu",
             (unsigned long long)svc.count(), (unsigned long long)svc.percentile(50),
             (unsigned long long)svc.percentile(99), (unsigned long long)svc.percentile(99.9),
             (unsigned long long)svc.max());
    s += buf;
  }
  if (pmu) {
    snprintf(buf, sizeof buf, ",\"user_instructions\":%llu,\"user_cycles\":%llu", (unsigned long long)u_ins,
             (unsigned long long)u_cyc);
    s += buf;
  }
  if (with_hist) s += ",\"hist\":\"" + h.encode() + "\"";
  return s + "}";
}

// wrk's duration syntax: "30", "30s", "2m", "1h".
double parse_duration(const std::string& v) {
  char* end = nullptr;
  double x = strtod(v.c_str(), &end);
  if (end && *end == 'm') x *= 60;
  else if (end && *end == 'h') x *= 3600;
  return x;
}

// "http://host:port/path" (host may be a bracketed IPv6 literal) -> "host:port", "/path".
bool parse_url_arg(const std::string& url, std::string* target, std::string* path) {
  if (url.rfind("http://", 0) != 0) return false;
  std::string rest = url.substr(7);
  size_t slash = rest.find('/');
  std::string hostport = rest.substr(0, slash);
  *path = slash == std::string::npos ? "/" : rest.substr(slash);
  std::string host = hostport, port = "80";
  if (!hostport.empty() && hostport[0] == '[') {
    size_t rb = hostport.find(']');
    if (rb == std::string::npos) return false;
    host = hostport.substr(1, rb - 1);
    if (rb + 1 < hostport.size() && hostport[rb + 1] == ':') port = hostport.substr(rb + 2);
  } else if (size_t colon = hostport.rfind(':'); colon != std::string::npos) {
    host = hostport.substr(0, colon);
    port = hostport.substr(colon + 1);
  }
  *target = host + ":" + port;
  return !host.empty();
}

// --expect-body text with \n \r \t \\ escapes.
std::string unescape(const std::string& s) {
  std::string o;
  for (size_t i = 0; i < s.size(); ++i) {
    if (s[i] != '\\' || i + 1 == s.size()) {
      o += s[i];
      continue;
    }
    char n = s[++i];
    o += n == 'n' ? '\n' : n == 'r' ? '\r' : n == 't' ? '\t' : n;
  }
  return o;
}

std::string human_ns(double ns) {
  char b[32];
  if (ns < 1e3) snprintf(b, sizeof b, "%.0fns", ns);
  else if (ns < 1e6) snprintf(b, sizeof b, "%.2fus", ns / 1e3);
  else if (ns < 1e9) snprintf(b, sizeof b, "%.2fms", ns / 1e6);
  else snprintf(b, sizeof b, "%.2fs", ns / 1e9);
  return b;
}

std::string human_bytes(double b) {
  const char* u[] = {"B", "KB", "MB", "GB", "TB"};
  int k = 0;
  while (b >= 1024 && k < 4) {
    b /= 1024;
    ++k;
  }
  char s[32];
  snprintf(s, sizeof s, "%.2f%s", b, u[k]);
  return s;
}

}  // namespace

int main(int argc, char** argv) {
  Options o;
  std::string targets = "127.0.0.1:8080", cpu_list, url, cpu_profile;
  bool json = false, latency = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) {
        fprintf(stderr, "loadgen: %s needs a value\n", a.c_str());
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--targets") targets = val();
    else if (a == "--connections" || a == "-c") o.connections = atoi(val().c_str());
    else if (a == "--threads" || a == "-t") o.threads = atoi(val().c_str());
    else if (a == "--cpu-list") cpu_list = val();
    else if (a == "--path") o.path = val();
    else if (a == "--method") o.method = val();
    else if (a == "--duration" || a == "-d") o.duration_s = parse_duration(val());
    else if (a.size() > 2 && (a.rfind("-d", 0) == 0 || a.rfind("-c", 0) == 0 || a.rfind("-t", 0) == 0) &&
             (isdigit((unsigned char)a[2]))) {  // wrk's glued short options: -d30s -c64 -t8
      if (a[1] == 'd') o.duration_s = parse_duration(a.substr(2));
      else if (a[1] == 'c') o.connections = atoi(a.c_str() + 2);
      else o.threads = atoi(a.c_str() + 2);
    }
    else if (a == "--latency") latency = true;
    else if (a == "--json") json = true;
    else if (a == "--version") {
      printf("hola_loadgen %s (revision %s, %s)\n", hola::build_info::version(), hola::build_info::revision(),
             hola::isa::build_level());
      return 0;
    }
    else if (a.rfind("http://", 0) == 0) url = a;
    else if (a == "--warmup") o.warmup_s = atof(val().c_str());
    else if (a == "--control") o.control = true;
    else if (a == "--target-offset") o.target_offset = atoi(val().c_str());
    else if (a == "--header" || a == "-H") o.extra_headers.push_back(val());
    else if (a == "--busy-poll-us") o.busy_poll_us = atoi(val().c_str());
    else if (a == "--busy-poll-pause") o.busy_poll_pause = atoi(val().c_str());
    else if (a == "--epoll-lt") o.edge_triggered = false;
    else if (a == "--rate" || a == "-R") {
      o.rate = atof(val().c_str());
      o.rx_timestamps = o.rate > 0;
    }
    else if (a == "--spin-us") o.spin_us = atoi(val().c_str());
    else if (a == "--sched-slice-us") o.sched_slice_us = atoi(val().c_str());
    else if (a == "--per-conn-quota") o.per_conn_quota = true;
    else if (a == "--pipeline") o.pipeline = atoi(val().c_str());
    else if (a == "--expect-body") o.expect_bodies.push_back(unescape(val()));
    else if (a == "--alt-body") o.alt_bodies.push_back(unescape(val()));
    else if (a == "--verify-body") o.verify_body = true;
    else if (a == "--cpu-profile") cpu_profile = val();
    else if (a == "--endpoints-file") o.endpoints_file = val();
    else if (a == "--conn-targets") {
      if (!parse_cpu_list(val(), &o.conn_targets)) {  // same "0,1,1,0" / "0-3" syntax
        fprintf(stderr, "loadgen: bad --conn-targets\n");
        return 2;
      }
    }
    else {
      fprintf(stderr,
              "usage: hola_loadgen --targets h:p[,h:p..] -c CONNS -t THREADS [--cpu-list L] [--path P]\n"
              "                    (--duration S [--warmup S] [--rate R [--spin-us N]] | --control [--per-conn-quota])\n"
              "                    [--sched-slice-us N]  (each thread asks the scheduler for an N us slice)\n"
              "                    [--target-offset K] [--busy-poll-us N [--busy-poll-pause P]] [--epoll-lt] [-H 'Name: v']\n"
              "                    [--pipeline P] [--expect-body B]... [--alt-body B]... [--verify-body] [--conn-targets i,j,..]\n"
              "                    [--cpu-profile FILE]  (sampled call stacks, bench/cpuprof_report.py --threads hola-lg)\n"
              "                    [--endpoints-file F]  (Service mode: --targets is the Service, F its endpoints)\n"
              "       hola_loadgen -t T -c C -d 30s [--latency] [--json] [-H 'Name: v'] http://host:port/path   (wrk style)\n");
      return 2;
    }
  }
  if (!url.empty()) {
    if (!parse_url_arg(url, &targets, &o.path)) {
      fprintf(stderr, "loadgen: bad URL %s\n", url.c_str());
      return 2;
    }
  }
  const bool wrk_text = !url.empty() && !json && !o.control;
  if (!parse_targets(targets, &o.targets)) return 2;
  if (!o.endpoints_file.empty()) {
    if (o.targets.size() != 1 || !o.conn_targets.empty() || o.expect_bodies.size() > 1) {
      fprintf(stderr, "loadgen: --endpoints-file takes one Service address, one --expect-body at most\n");
      return 2;
    }
    g_dnat.path = o.endpoints_file;
  }
  for (int t : o.conn_targets)
    if (t < 0 || size_t(t) >= o.targets.size()) {
      fprintf(stderr, "loadgen: --conn-targets index %d out of range\n", t);
      return 2;
    }
  if (!cpu_list.empty() && !parse_cpu_list(cpu_list, &o.cpus)) {
    fprintf(stderr, "loadgen: bad --cpu-list\n");
    return 2;
  }
  if (o.threads < 1) o.threads = 1;
  if (o.connections < o.threads) o.connections = o.threads;
  if (o.pipeline < 1 || o.pipeline > 64 || (o.pipeline > 1 && o.rate > 0)) {
    fprintf(stderr, "loadgen: --pipeline takes 1..64 and is closed-loop only\n");
    return 2;
  }
  if (!o.control && o.duration_s <= 0) o.duration_s = 10;
  signal(SIGPIPE, SIG_IGN);
  if (!o.control) {
    // SIGINT/SIGTERM end a timed run early: the summary covers the time actually run (a
    // harness can run the load "until the rollout is over").
    struct sigaction sa {};
    sa.sa_handler = [](int) { g_stop.store(true, std::memory_order_relaxed); };
    sigaction(SIGINT, &sa, nullptr);
    sigaction(SIGTERM, &sa, nullptr);
  }
  if (!cpu_profile.empty() && !hola::cpuprof::start(cpu_profile)) {
    fprintf(stderr, "loadgen: cannot start the CPU profiler\n");
    return 2;
  }
  g_donefd = eventfd(0, EFD_SEMAPHORE | EFD_CLOEXEC);

  std::vector<std::unique_ptr<ThreadState>> ts;
  for (int t = 0; t < o.threads; ++t) {
    auto s = std::make_unique<ThreadState>();
    s->index = t;
    s->epfd = epoll_create1(EPOLL_CLOEXEC);
    s->wakefd = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    ts.push_back(std::move(s));
  }
  for (int i = 0; i < o.connections; ++i) ts[size_t(i % o.threads)]->conn_ids.push_back(i);
  std::vector<std::thread> th;
  for (auto& s : ts) th.emplace_back(thread_main, s.get(), &o);
  // Each thread connects its own connections from its pinned CPU (as wrk does), so the
  // server sees every connection's packets arrive on the CPU that will drive it.
  for (size_t k = 0; k < ts.size(); ++k) {
    uint64_t v;
    while (::read(g_donefd, &v, sizeof v) < 0 && errno == EINTR) {
    }
  }
  if (g_connect_failed.load()) {
    fprintf(stderr, "loadgen: %s\n", g_connect_error);
    _exit(1);
  }

  if (!o.control) {
    const int64_t t_start = mono_ns();
    for (auto& t : th) t.join();
    if (!cpu_profile.empty()) hola::cpuprof::write();
    std::string s = stats_json(ts, false);
    uint64_t completed = 0;
    for (auto& t : ts) completed += t->completed;
    if (g_stop.load()) {  // stopped by a signal: the measured part is what ran after the warm-up
      const double ran = double(mono_ns() - t_start) / 1e9 - o.warmup_s;
      o.duration_s = std::max(1e-3, std::min(o.duration_s, ran));
    }
    double rps = double(completed) / o.duration_s;
    if (wrk_text) {
      Histogram h;
      uint64_t errors = 0, non2xx = 0, bytes = 0;
      for (auto& t : ts) {
        h.merge(t->hist);
        errors += t->errors;
        non2xx += t->non2xx;
        bytes += t->bytes;
      }
      printf("Running %.0fs test @ %s\n  %d threads and %d connections\n", o.duration_s, url.c_str(), o.threads,
             o.connections);
      printf("  Latency   avg %s, max %s\n", human_ns(h.mean()).c_str(), human_ns(double(h.max())).c_str());
      if (latency) {
        printf("  Latency Distribution\n");
        for (double p : {50.0, 75.0, 90.0, 99.0, 99.9})
          printf("  %6.2f%%  %s\n", p, human_ns(double(h.percentile(p))).c_str());
      }
      printf("  %llu requests in %.2fs, %s read\n", (unsigned long long)completed, o.duration_s,
             human_bytes(double(bytes)).c_str());
      uint64_t mismatch = 0;
      for (auto& t : ts) mismatch += t->body_mismatch;
      if (errors) printf("  Socket errors: %llu\n", (unsigned long long)errors);
      if (mismatch) printf("  Body mismatches: %llu\n", (unsigned long long)mismatch);
      if (non2xx) printf("  Non-2xx or 3xx responses: %llu\n", (unsigned long long)non2xx);
      printf("Requests/sec: %12.2f\nTransfer/sec: %10s\n", rps, human_bytes(double(bytes) / o.duration_s).c_str());
      return 0;
    }
    printf("{\"mode\":\"%s\",\"duration_s\":%.3f,\"connections\":%d,\"threads\":%d,\"targets\":%zu,\"target_rate\":%.1f,\"rps\":%.1f,\"latency\":%s}\n",
           o.rate > 0 ? "open-loop" : "duration", o.duration_s, o.connections, o.threads,
           o.endpoints_file.empty() ? o.targets.size() : g_dnat.seen(), o.rate, rps, s.c_str());
    return 0;
  }

  // ---- control protocol ----
  printf("{\"ready\":true,\"connections\":%d,\"threads\":%d}\n", o.connections, o.threads);
  fflush(stdout);
  std::string line;
  uint64_t gen = 0;
  while (std::getline(std::cin, line)) {
    const bool run_for = line.rfind("runfor ", 0) == 0;
    if (run_for && o.per_conn_quota) {
      printf("{\"error\":\"runfor needs the shared budget (no --per-conn-quota)\"}\n");
      fflush(stdout);
    } else if (run_for || line.rfind("run ", 0) == 0) {
      const int64_t q = run_for ? INT64_MAX / 4 : atoll(line.c_str() + 4);
      int64_t for_ms = 0, warm_ms = 0;
      if (run_for) {
        long long a = 0, b = 0;
        const int got = sscanf(line.c_str() + 7, "%lld %lld", &a, &b);
        for_ms = a;
        warm_ms = got == 2 ? b : 0;
      }
      ++gen;
      const int64_t started = mono_ns();
      int64_t t0 = started + warm_ms * 1000000;  // start of the counted part
      g_count_from.store(warm_ms > 0 ? t0 : 0);
      // Budgets count batches: with --pipeline P, a claim is P requests. A timed run starts
      // with a budget no run can use up and has it taken away at the deadline: each thread then
      // finishes the requests it holds (at most a claim batch), and the run ends.
      const int64_t P = o.pipeline;
      g_budget.store(run_for ? INT64_MAX / 4 : (q * int64_t(o.connections) + P - 1) / P);
      for (auto& t : ts) {
        t->run_quota.store(std::max<int64_t>(1, (q + P - 1) / P));
        t->run_gen.store(gen);
        uint64_t one = 1;
        ssize_t w = ::write(t->wakefd, &one, sizeof one);
        (void)w;
      }
      if (run_for) {
        const int64_t deadline = t0 + for_ms * 1000000;  // after the warm-up
        for (int64_t now = mono_ns(); now < deadline && !g_stop.load(); now = mono_ns()) {
          const int64_t left = deadline - now;
          struct timespec d {left / 1000000000, left % 1000000000};
          nanosleep(&d, nullptr);
        }
        g_budget.store(INT64_MIN / 4);
      }
      uint64_t reqs = 0, errs = 0;
      for (size_t k = 0; k < ts.size(); ++k) {
        uint64_t v;
        while (::read(g_donefd, &v, sizeof v) < 0 && errno == EINTR) {
        }
        if (g_stop.load()) {
          printf("{\"error\":\"connection failure\"}\n");
          fflush(stdout);
          _exit(1);
        }
      }
      for (auto& t : ts) {
        reqs += t->done_requests.load();
        errs += t->done_errors.load();
      }
      g_count_from.store(0);
      int64_t el = mono_ns() - t0;
      printf("{\"elapsed_ns\":%lld,\"requests\":%llu,\"errors\":%llu}\n", (long long)el, (unsigned long long)reqs,
             (unsigned long long)errs);
      fflush(stdout);
    } else if (line == "stats") {
      printf("%s\n", stats_json(ts, true).c_str());
      fflush(stdout);
    } else if (line == "reset") {
      for (auto& t : ts) {
        std::lock_guard<std::mutex> g(t->hist_mu);
        t->hist.reset();
        t->svc.reset();
        t->errors = t->non2xx = t->reconnects = t->body_checked = t->body_mismatch = t->body_alt = 0;
        t->pmu_reset();
        t->sched_reset();
        for (Stat* x : {&t->poll_hits, &t->spin_hits, &t->spin_misses, &t->blocking_waits, &t->idle_spin_ns,
                        &t->gaps_over[0], &t->gaps_over[1], &t->gaps_over[2], &t->gap_max_ns,
                        &t->send_late_max_ns, &t->behind_max_ns, &t->sends_late_1ms})
          *x = 0;
      }
      printf("{\"reset\":true}\n");
      fflush(stdout);
    } else if (line == "quit") {
      break;
    }
  }
  g_stop.store(true);
  for (auto& t : ts) {
    uint64_t one = 1;
    ssize_t w = ::write(t->wakefd, &one, sizeof one);
    (void)w;
  }
  for (auto& t : th) t.join();
  if (!cpu_profile.empty()) hola::cpuprof::write();
  return 0;
}
