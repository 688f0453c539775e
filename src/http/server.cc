#include "http/server.h"

#include <errno.h>
#include <netinet/in.h>
#include <pthread.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>

#include "core/affinity.h"
#include "core/clock.h"
#include "core/cpuprof.h"
#include "core/log.h"
#include "core/net.h"

namespace hola::http {

namespace {
constexpr size_t kMaxBufferedOutput = 1 << 20;  // stop reading while this much is unsent
constexpr int64_t kDrainIdleGraceMs = 100;       // see Server::shutdown
constexpr int64_t kAnswerGraceMs = 1000;          // ditto: the least time a worker gets to answer
constexpr int64_t kMaxBody = 1 << 20;           // request bodies are read and discarded

const char* reason_phrase(int status) {
  switch (status) {
    case 400: return "Bad Request";
    case 413: return "Request Entity Too Large";
    case 414: return "Request-URI Too Long";
    case 431: return "Request Header Fields Too Large";
    case 501: return "Not Implemented";
    case 505: return "HTTP Version Not Supported";
    default: return "Error";
  }
}
}  // namespace

std::string RequestHandler::error_response(int status) {
  std::string s = "HTTP/1.1 " + std::to_string(status) + " " + reason_phrase(status) +
                  "\r\nConnection: close\r\nContent-Length: 0\r\n\r\n";
  return s;
}

// ---------------------------------------------------------------- Connection

Connection::Connection(Worker* w, int fd, uint64_t id)
    : worker_(w), fd_(fd), id_(id), last_active_ms_(w->loop().now_ms()) {}

Connection::~Connection() {
  if (fd_ >= 0) ::close(fd_);
}

uint64_t Connection::state_bits(uint32_t iterations) const {
  const uint64_t flags = uint64_t(parked_) | uint64_t(close_after_flush_) << 1 | uint64_t(reading_) << 2 |
                         uint64_t(want_write_) << 3 | uint64_t(streaming_) << 4 | uint64_t(closed_) << 5 |
                         uint64_t(in_process_) << 6 | uint64_t(read_pending_) << 7;
  return flags | uint64_t(std::min<size_t>(in_.size(), 0xFFFFFF)) << 8 |
         uint64_t(std::min<size_t>(unsent(), 0xFFFFFF)) << 32 | uint64_t(std::min<uint32_t>(iterations, 255)) << 56;
}

std::string Connection::describe_state(uint64_t s) {
  static const char* const names[] = {"parked", "close_after_flush", "reading", "want_write",
                                      "streaming", "closed", "in_process", "read_pending"};
  std::string out = "{";
  for (int b = 0; b < 8; ++b)
    if (s >> b & 1) out += std::string(out.size() > 1 ? "," : "") + names[b];
  out += "} in=" + std::to_string(s >> 8 & 0xFFFFFF) + " unsent=" + std::to_string(s >> 32 & 0xFFFFFF) +
         " read_iterations=" + std::to_string(s >> 56);
  return out;
}

void Connection::on_event(uint32_t ev) {
  worker_->loop().note(kConnectionHandler, id_, state_bits(0));
  if (closed_) return;
  if (ev & EPOLLERR) {
    close();
    return;
  }
  if (ev & EPOLLOUT) {
    on_writable();
    if (closed_) return;
  }
  if (ev & (EPOLLIN | EPOLLHUP | EPOLLRDHUP)) on_readable((ev & (EPOLLHUP | EPOLLRDHUP)) != 0);
}

void Connection::on_readable(bool peer_closed) {
  WorkerStats& st = worker_->stats();
  last_active_ms_ = worker_->loop().now_ms();
  // Sockets are edge-triggered by default (ServerOptions::edge_triggered): a read that fills
  // the buffer may have left data behind, so read again; a short read drained the socket.
  // This saves the re-poll of every level-triggered ready item on the next epoll_wait. When
  // the peer has shut down its side, its FIN may sit behind the data of this same edge: read
  // on to the EOF, answer what was read, then close.
  if (streaming_) {
    char buf[4096];
    for (;;) {
      ssize_t n = ::recv(fd_, buf, sizeof buf, 0);
      if (n < 0 && errno == EINTR) continue;
      if (n == 0 || (n < 0 && errno != EAGAIN)) close();
      if (n < ssize_t(sizeof buf)) return;
    }
  }
  if (parked_) {
    read_pending_ = true;
    peer_closed_pending_ |= peer_closed;
    return;
  }
  StageProfile* prof = worker_->profile();
  bool more = false;
  uint32_t iterations = 0;
  while (!parked_ && reading_ && !streaming_ && !closed_) {
    if (++iterations > 1) worker_->loop().note_state(state_bits(iterations));
    int64_t t0 = prof ? mono_ns() : 0;
    if (in_.empty()) {
      char* buf = worker_->scratch();
      const size_t cap = worker_->scratch_size();
      ssize_t n = ::recv(fd_, buf, cap, 0);
      if (prof && n > 0) prof->recv.add(uint64_t(mono_ns() - t0));
      if (n <= 0) {
        if (n < 0 && errno == EINTR) continue;
        if (n == 0 || errno != EAGAIN) {
          flush();
          close();
        }
        break;
      }
      WorkerStats::bump(st.bytes_in, uint64_t(n));
      more = size_t(n) == cap || peer_closed;
      size_t consumed = 0;
      if (!process(buf, size_t(n), &consumed)) return;
      if (consumed < size_t(n)) in_.assign(buf + consumed, size_t(n) - consumed);
    } else {
      size_t old = in_.size();
      size_t chunk = worker_->server().options().read_chunk;
      in_.resize(old + chunk);
      ssize_t n = ::recv(fd_, &in_[old], chunk, 0);
      if (n <= 0) {
        in_.resize(old);
        if (n < 0 && errno == EINTR) continue;
        if (n == 0 || errno != EAGAIN) {
          flush();
          close();
        }
        break;
      }
      WorkerStats::bump(st.bytes_in, uint64_t(n));
      in_.resize(old + size_t(n));
      more = size_t(n) == chunk || peer_closed;
      size_t consumed = 0;
      std::string buf;
      buf.swap(in_);  // handlers may park: leftovers are re-stored below
      if (!process(buf.data(), buf.size(), &consumed)) return;
      if (consumed < buf.size()) in_.assign(buf, consumed, std::string::npos);
    }
    if (!more) break;
  }
  if (parked_ && more) {
    // parked with input possibly still in the socket: no new edge will announce it
    read_pending_ = true;
    peer_closed_pending_ |= peer_closed;
  }
  if (!closed_) flush();
}

bool Connection::process(const char* data, size_t len, size_t* consumed) {
  WorkerStats& st = worker_->stats();
  RequestHandler& h = worker_->handler();
  in_process_ = true;
  size_t off = 0;
  uint64_t handled = 0;
  Request r;  // parse_request resets it for every request
  while (off < len && !parked_ && !streaming_ && !closed_ && !close_after_flush_) {
    int status = 400;
    StageProfile* prof = worker_->profile();
    int64_t tp = prof ? mono_ns() : 0;
    Parse p = parse_request(data + off, len - off, &r, &status);
    if (prof && p == Parse::kOk) prof->parse.add(uint64_t(mono_ns() - tp));
    if (p == Parse::kIncomplete) break;
    if (p == Parse::kError) {
      WorkerStats::bump(st.parse_errors);
      error_response(status);
      off = len;
      break;
    }
    size_t total = r.head_bytes;
    if (r.chunked) {
      size_t body = 0;
      Parse q = skip_chunked_body(data + off + total, len - off - total, &body);
      if (q == Parse::kIncomplete) {
        if (len - off > size_t(kMaxBody)) {
          error_response(413);
          off = len;
        }
        break;
      }
      if (q == Parse::kError) {
        WorkerStats::bump(st.parse_errors);
        error_response(400);
        off = len;
        break;
      }
      total += body;
    } else if (r.content_length > 0) {
      if (r.content_length > kMaxBody) {
        error_response(413);
        off = len;
        break;
      }
      if (len - off - total < size_t(r.content_length)) {
        // RFC 9110 §10.1.1: a client waiting on "Expect: 100-continue" gets the interim
        // response once, then sends the body.
        if (r.expect_continue && !continue_sent_) {
          static constexpr std::string_view k100 = "HTTP/1.1 100 Continue\r\n\r\n";
          out_.append(k100.data(), k100.size());
          continue_sent_ = true;
        }
        break;
      }
      continue_sent_ = false;
      total += size_t(r.content_length);
    }
    off += total;
    WorkerStats::bump(st.requests);
    ++handled;
    // Read before the handler chooses its Connection header: the flag only goes from false to
    // true, so when it is set here the handler sees it too and answers `Connection: close`.
    // Re-reading it after the handler would race with begin_termination() on another thread
    // and close a connection whose response had just announced keep-alive.
    const bool closing = worker_->server().closing();
    // a pending prepared response is copied before the next handler runs: that handler may
    // rebuild the prepared responses it points into (HolaApp::refresh)
    materialize();
    if (prof) {
      int64_t th = mono_ns();
      h.on_request(*this, r);
      prof->handle.add(uint64_t(mono_ns() - th));
    } else {
      h.on_request(*this, r);
    }
    if (closing) close_after_flush_ = true;
  }
  in_process_ = false;
  if (StageProfile* prof = worker_->profile(); prof && handled) prof->batch.add(handled);
  *consumed = off;
  if (closed_) return false;
  if (streaming_ || (parked_ && !worker_->server().options().edge_triggered)) update_interest();
  return true;
}

void Connection::error_response(int status) {
  std::string s = worker_->handler().error_response(status);
  send(s.data(), s.size());
  close_after_flush_ = true;
}

void Connection::send(const char* p, size_t n) {
  if (closed_) return;
  materialize();
  out_.append(p, n);
  if (!in_process_) flush();
}

void Connection::send_stable(std::string_view s) {
  if (closed_) return;
  if (out_off_ == out_.size() && !stable_) {
    out_.clear();
    out_off_ = 0;
    stable_ = s.data();
    stable_len_ = s.size();
  } else {
    materialize();
    out_.append(s.data(), s.size());
  }
  if (!in_process_) flush();
}

void Connection::complete(std::string_view response, bool keep_alive) {
  if (!closed_) {
    materialize();
    out_.append(response.data(), response.size());
  }
  complete_appended(keep_alive);
}

void Connection::complete_appended(bool keep_alive) {
  if (closed_) {
    parked_ = false;
    return;
  }
  parked_ = false;
  // keep_alive is what the response announced; the caller chose it with closing() (reading
  // the flag again here could close a connection whose response said keep-alive)
  if (!keep_alive) close_after_flush_ = true;
  if (in_process_) return;
  // Continue with pipelined requests that arrived while parked.
  if (!in_.empty() && !close_after_flush_) {
    std::string buf;
    buf.swap(in_);
    size_t consumed = 0;
    if (!process(buf.data(), buf.size(), &consumed)) return;
    if (consumed < buf.size()) in_.assign(buf, consumed, std::string::npos);
  }
  flush();
  if (closed_) return;
  if (!worker_->server().options().edge_triggered) {
    update_interest();  // level-triggered: input interest was dropped while parked
  } else if (read_pending_ && !parked_) {
    const bool pc = peer_closed_pending_;
    read_pending_ = peer_closed_pending_ = false;
    on_readable(pc);
  }
}

void Connection::start_streaming(std::function<void()> on_close) {
  streaming_ = true;
  on_close_ = std::move(on_close);
}

void Connection::flush() {
  WorkerStats& st = worker_->stats();
  StageProfile* prof = worker_->profile();
  while (stable_) {  // a prepared response, sent from where it lives (out_ is empty)
    int64_t ts = prof ? mono_ns() : 0;
    ssize_t w = ::send(fd_, stable_, stable_len_, MSG_NOSIGNAL);
    if (prof && w > 0) prof->send.add(uint64_t(mono_ns() - ts));
    if (w < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN) {
        materialize();  // the socket is full: the rest waits in out_ (handled below)
        break;
      }
      close();
      return;
    }
    WorkerStats::bump(st.bytes_out, uint64_t(w));
    sent_total_ += uint64_t(w);
    stable_ += w;
    stable_len_ -= size_t(w);
    if (!stable_len_) stable_ = nullptr;
  }
  while (out_off_ < out_.size()) {
    int64_t ts = prof ? mono_ns() : 0;
    ssize_t w = ::send(fd_, out_.data() + out_off_, out_.size() - out_off_, MSG_NOSIGNAL);
    if (prof && w > 0) prof->send.add(uint64_t(mono_ns() - ts));
    if (w < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN) {
        if (!want_write_) {
          want_write_ = true;
          if (out_.size() - out_off_ > kMaxBufferedOutput) reading_ = false;
          update_interest();
        }
        return;
      }
      close();
      return;
    }
    WorkerStats::bump(st.bytes_out, uint64_t(w));
    out_off_ += size_t(w);
    sent_total_ += uint64_t(w);
  }
  out_.clear();
  out_off_ = 0;
  if (want_write_ || !reading_) {
    want_write_ = false;
    reading_ = true;
    update_interest();
  }
  if (close_after_flush_ && !parked_) {
    ::shutdown(fd_, SHUT_WR);
    close();
  }
}

void Connection::on_writable() {
  // The slow path (the socket was full): progress here counts as activity for the idle sweep,
  // so only a peer that has stopped reading its responses is timed out.
  const uint64_t before = sent_total_;
  flush();
  if (sent_total_ != before) last_active_ms_ = worker_->loop().now_ms();
}

void Connection::update_interest() {
  if (closed_) return;
  uint32_t ev = worker_->server().options().edge_triggered ? uint32_t(EPOLLET) : 0u;
  if (streaming_) ev |= EPOLLIN | EPOLLRDHUP;
  // level-triggered input interest is dropped while a request is parked, edge-triggered
  // interest is kept (see read_pending_)
  else if (reading_ && (!parked_ || (ev & EPOLLET))) ev |= EPOLLIN | EPOLLRDHUP;
  if (want_write_) ev |= EPOLLOUT;
  worker_->loop().mod(fd_, ev, this);
}

void Connection::close() {
  if (closed_) return;
  closed_ = true;
  stable_ = nullptr;
  stable_len_ = 0;
  worker_->loop().del(fd_);
  ::close(fd_);
  fd_ = -1;
  WorkerStats::bump(worker_->stats().closed);
  worker_->on_connection_closed(this);
  if (on_close_) {
    auto f = std::move(on_close_);
    on_close_ = nullptr;
    f();
  }
  if (holds_ == 0) worker_->loop().retire(this);
}

void Connection::release() {
  if (--holds_ == 0 && closed_) worker_->loop().retire(this);
}

std::string Connection::peer() const {
  sockaddr_storage ss{};
  socklen_t len = sizeof ss;
  if (fd_ < 0 || getpeername(fd_, reinterpret_cast<sockaddr*>(&ss), &len) != 0) return "?";
  return sockaddr_to_string(ss);
}

// ---------------------------------------------------------------- Worker

Worker::Worker(Server* s, int index) : server_(s), index_(index) {
  // scratch_ is allocated by the worker thread itself once pinned (Server::start), so its
  // pages are first touched on the worker's own NUMA node.
  if (s->options().profile) profile_ = std::make_unique<StageProfile>();
  memset(date_, ' ', sizeof date_);
  tick();
  loop_.set_tick([this] { tick(); });
  loop_.set_busy_poll_us(s->options().busy_poll_us);
  loop_.set_busy_poll_pause(s->options().busy_poll_pause);
  loop_.set_busy_poll_auto(s->options().busy_poll_auto);
}

Worker::~Worker() {
  while (conns_) conns_->close_silently();  // unlinks itself from conns_
}

RequestHandler& Worker::handler() { return server_->handler(); }

void Worker::tick() {
  // The Date header's second, re-read every 4 ms of the loop's own time (a busy loop runs
  // many passes per millisecond): the header is at most 4 ms late, and most passes read no
  // clock at all.
  const int64_t now = loop_.now_ms();
  if (now < next_date_check_ms_) return;
  next_date_check_ms_ = now + 4;
  int64_t s = wall_sec_coarse();
  if (s != date_sec_) {
    date_sec_ = s;
    format_http_date(s, date_);
    ++date_version_;
  }
}

void Worker::on_connection_closed(Connection* c) {
  --nconns_;
  server_->assigned_[size_t(index_)].fetch_sub(1, std::memory_order_relaxed);
  server_->open_.fetch_sub(1, std::memory_order_relaxed);
  if (c->prev_) c->prev_->next_ = c->next_;
  else conns_ = c->next_;
  if (c->next_) c->next_->prev_ = c->prev_;
  c->prev_ = c->next_ = nullptr;
}

void Worker::close_idle_connections(int64_t grace_ms) {
  const int64_t now = loop_.now_ms();
  for (Connection* c = conns_; c;) {
    Connection* next = c->next_;
    if (c->streaming() || (c->idle() && now - c->last_active_ms() >= grace_ms)) c->close();
    c = next;
  }
}

void Worker::sweep_idle() {
  const int64_t limit = server_->options().idle_timeout_ms;
  const int64_t now = loop_.now_ms();
  for (Connection* c = conns_; c;) {
    Connection* next = c->next_;
    // Includes connections holding a partial request (slow-loris): nothing arrived for the
    // whole timeout, so the request will not complete; and connections whose peer stopped
    // reading its responses: nothing was read or written for the whole timeout (the output
    // backlog stays bounded by kMaxBufferedOutput meanwhile). A parked request has its own
    // deadline (the Hystrix timeout), and SSE streams have theirs.
    if (!c->streaming() && !c->parked_ && now - c->last_active_ms() > limit) c->close();
    c = next;
  }
}

void Worker::adopt(int fd, int64_t accepted_ns) {
  loop_.post([this, fd, accepted_ns] { adopt_here(fd, accepted_ns); });
}

void Worker::adopt_here(int fd, int64_t accepted_ns) {
  if (profile_ && accepted_ns) profile_->accept.add(uint64_t(mono_ns() - accepted_ns));
  auto* c = new Connection(this, fd, (uint64_t(index_) << 48) | next_conn_id_++);
  const size_t maxc = server_->options().max_connections;
  if (maxc && server_->open_connections() >= maxc) {
    WorkerStats::bump(stats_.rejected);
    server_->assigned_[size_t(index_)].fetch_sub(1, std::memory_order_relaxed);
    delete c;  // over the limit: refuse by closing (the client sees a reset/EOF)
    return;
  }
  const uint32_t et = server_->options().edge_triggered ? uint32_t(EPOLLET) : 0u;
  if (server_->draining() || !loop_.add(fd, EPOLLIN | EPOLLRDHUP | et, c)) {
    server_->assigned_[size_t(index_)].fetch_sub(1, std::memory_order_relaxed);
    delete c;
    return;
  }
  ++nconns_;
  server_->open_.fetch_add(1, std::memory_order_relaxed);
  WorkerStats::bump(stats_.accepted);
  c->next_ = conns_;
  if (conns_) conns_->prev_ = c;
  conns_ = c;
}

// ---------------------------------------------------------------- Server

Server::Server(ServerOptions opts, RequestHandler* handler) : opts_(std::move(opts)), handler_(handler) {
  if (opts_.threads < 1) opts_.threads = 1;
  for (int i = 0; i < opts_.threads; ++i) workers_.push_back(std::make_unique<Worker>(this, i));
  assigned_.reset(new std::atomic<int32_t>[workers_.size()]);
  for (size_t i = 0; i < workers_.size(); ++i) assigned_[i].store(0);
  if (opts_.steer_l3 && !opts_.cpus.empty()) {
    for (size_t i = 0; i < workers_.size(); ++i) {
      int dom = l3_domain_of(opts_.cpus[i % opts_.cpus.size()]);
      if (dom < 0) {
        domain_workers_.clear();
        break;
      }
      auto it = std::find_if(domain_workers_.begin(), domain_workers_.end(),
                             [dom](const auto& p) { return p.first == dom; });
      if (it == domain_workers_.end()) domain_workers_.push_back({dom, {i}});
      else it->second.push_back(i);
    }
    // Workers pinned to a core whose SMT sibling may run a client thread: a connection from
    // that sibling is served on the same physical core (shared L1/L2 for both socket
    // buffers). Only cores holding exactly one worker qualify.
    for (size_t i = 0; i < workers_.size() && i < opts_.cpus.size(); ++i) {
      int core = core_of(opts_.cpus[i]);
      if (core < 0) continue;
      auto it = std::find_if(core_workers_.begin(), core_workers_.end(),
                             [core](const auto& p) { return p.first == core; });
      if (it == core_workers_.end()) core_workers_.push_back({core, i});
      else it->first = -1;  // two workers on one core: no single partner
    }
    core_workers_.erase(std::remove_if(core_workers_.begin(), core_workers_.end(),
                                       [](const auto& p) { return p.first < 0; }),
                        core_workers_.end());
    if (domain_workers_.size() <= 1) domain_workers_.clear();  // one domain: nothing to steer
    domain_rr_.reset(new std::atomic<uint32_t>[domain_workers_.size() + 1]);
    for (size_t i = 0; i <= domain_workers_.size(); ++i) domain_rr_[i].store(0);
  }
}

const char* Server::locality_name(int l) {
  static const char* const names[kNumLocality] = {"same_core", "same_l3", "same_socket", "cross_socket", "unknown"};
  return (l >= 0 && l < kNumLocality) ? names[l] : "?";
}

int Server::incoming_cpu(int fd) {
  int cpu = -1;
  socklen_t len = sizeof cpu;
  if (getsockopt(fd, SOL_SOCKET, SO_INCOMING_CPU, &cpu, &len) != 0) return -1;
  return cpu;
}

void Server::note_locality(int client_cpu, size_t worker) {
  int l = kUnknown;
  if (client_cpu >= 0 && !opts_.cpus.empty()) {
    const int wcpu = opts_.cpus[worker % opts_.cpus.size()];
    const int cc = core_of(client_cpu), wc = core_of(wcpu);
    const int cd = l3_domain_of(client_cpu), wd = l3_domain_of(wcpu);
    const int cp = package_of(client_cpu), wp = package_of(wcpu);
    if (client_cpu == wcpu || (cc >= 0 && cc == wc)) l = kSameCore;
    else if (cd >= 0 && cd == wd) l = kSameL3;
    else if (cp >= 0 && cp == wp) l = kSameSocket;
    else if (cp >= 0 && wp >= 0) l = kCrossSocket;
  }
  locality_[l].fetch_add(1, std::memory_order_relaxed);
}

Worker* Server::pick_worker(int fd) {
  const size_t n = workers_.size();
  size_t k = rr_.fetch_add(1, std::memory_order_relaxed) % n;
  // The CPU that processed this connection's latest packet: for loopback clients, the
  // client thread's own CPU. Serving it from the same L3 keeps both socket buffers in
  // one cache domain (cross-CCD hand-offs more than double the cost of send()).
  const int cpu = incoming_cpu(fd);
  if (!domain_workers_.empty() || !core_workers_.empty()) {
    if (cpu >= 0) {
      // Balance: a worker takes a steered connection unless it already holds twice its fair
      // share (+8). Comparing with the least loaded worker instead (+8) unsteered connections
      // whenever the clients of one L3 opened theirs before those of another, e.g. hola A's
      // pool to B warming up one L3 first: an eighth of A's connections to B then crossed
      // L3s for the whole run, +20 % CPU per chained request (profiles/round5/02_chain_modes).
      // Within an L3 the connections are dealt round-robin, so they stay even there.
      auto within_share = [&](size_t w) {
        int32_t small[256];
        std::vector<int32_t> big;  // more than 256 workers in one process: once per accept
        int32_t* counts = small;
        if (n > 256) {
          big.resize(n);
          counts = big.data();
        }
        for (size_t i = 0; i < n; ++i) counts[i] = assigned_[i].load(std::memory_order_relaxed);
        return steering_within_share(counts, n, w);
      };
      // Same physical core first (the client runs on this worker's SMT sibling).
      const int core = core_workers_.empty() ? -1 : core_of(cpu);
      for (const auto& [c, wi] : core_workers_) {
        if (c != core || opts_.cpus[wi] == cpu) continue;
        if (within_share(wi)) {
          assigned_[wi].fetch_add(1, std::memory_order_relaxed);
          steered_core_.fetch_add(1, std::memory_order_relaxed);
          note_locality(cpu, wi);
          return workers_[wi].get();
        }
        break;
      }
      int dom = domain_workers_.empty() ? -2 : l3_domain_of(cpu);
      for (size_t d = 0; d < domain_workers_.size(); ++d) {
        if (domain_workers_[d].first != dom) continue;
        const auto& ws = domain_workers_[d].second;
        size_t cand = ws[domain_rr_[d].fetch_add(1, std::memory_order_relaxed) % ws.size()];
        // Keep balance: do not pile onto a worker far beyond its share.
        if (within_share(cand)) {
          k = cand;
          steered_.fetch_add(1, std::memory_order_relaxed);
        } else {
          // Refused for balance: the least loaded worker. The round-robin index would alias
          // with the refusals' period (every third accept refused with three workers: the
          // same worker every time, the third idle).
          unsteered_.fetch_add(1, std::memory_order_relaxed);
          int32_t least = INT32_MAX;
          for (size_t i = 0; i < n; ++i)
            if (int32_t c = assigned_[i].load(std::memory_order_relaxed); c < least) {
              least = c;
              k = i;
            }
        }
        break;
      }
    }
  }
  assigned_[k].fetch_add(1, std::memory_order_relaxed);
  note_locality(cpu, k);
  return workers_[k].get();
}

Server::~Server() {
  for (auto& a : acceptors_)
    if (a->fd >= 0) ::close(a->fd);
  // Workers first, while the per-worker counters their connections update still exist.
  workers_.clear();
}

bool Server::bind(std::string* err) {
  ListenOptions lo;
  lo.host = opts_.host;
  lo.port = opts_.port;
  lo.backlog = opts_.backlog;
  lo.reuseport = opts_.reuseport_accept;
  size_t n = opts_.reuseport_accept ? workers_.size() : 1;
  for (size_t i = 0; i < n; ++i) {
    lo.incoming_cpu = -1;
    if (opts_.reuseport_accept && !opts_.cpus.empty() && opts_.reuseport_cpu != ServerOptions::ReuseportCpu::kNone) {
      const int cpu = opts_.cpus[i % opts_.cpus.size()];
      lo.incoming_cpu = opts_.reuseport_cpu == ServerOptions::ReuseportCpu::kSibling ? sibling_of(cpu) : cpu;
    }
    int fd = listen_tcp(lo, err);
    if (fd < 0) return false;
    if (i == 0) {
      port_ = bound_port(fd);
      lo.port = port_;  // with port 0, every reuseport listener must share the chosen port
    }
    auto a = std::make_unique<Acceptor>();
    a->server = this;
    a->worker = workers_[i].get();
    a->fd = fd;
    acceptors_.push_back(std::move(a));
  }
  return true;
}

void Server::Acceptor::on_event(uint32_t) {
  worker->loop().note(kAcceptorHandler, uint64_t(fd), 0);
  const bool prof = server->opts_.profile;
  for (int i = 0; i < 256; ++i) {
    const int64_t t0 = prof ? mono_ns() : 0;
    int c = ::accept4(fd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
    if (c < 0) {
      if (errno == EINTR || errno == ECONNABORTED) continue;
      if (errno == EMFILE || errno == ENFILE) {
        if (!paused) LOG_WARN("accept: %s (fd limit); pausing accepts", strerror(errno));
        paused = true;
        // back off for a moment; the listener stays level-triggered
        worker->loop().del(fd);
        int lfd = fd;
        Acceptor* self = this;
        worker->loop().add_timer(50, [self, lfd] {
          if (!self->server->draining()) self->worker->loop().add(lfd, EPOLLIN, self);
        });
      }
      return;
    }
    if (paused) {
      LOG_INFO("accept: resumed after the fd limit");
      paused = false;
    }
    if (server->opts_.reuseport_accept && !server->steering()) {
      // The kernel already spread connections over the workers' listeners.
      server->assigned_[size_t(worker->index())].fetch_add(1, std::memory_order_relaxed);
      server->note_locality(incoming_cpu(c), size_t(worker->index()));
      worker->adopt_here(c, t0);
    } else {
      // Round-robin accept, or reuseport with L3 steering: the kernel's hash ignores where
      // the client runs, so the connection may still move to a worker in the client's L3.
      Worker* w = server->pick_worker(c);
      if (w == worker) w->adopt_here(c, t0);
      else w->adopt(c, t0);
    }
  }
}

void Server::start() {
  for (auto& a : acceptors_) a->worker->loop().add(a->fd, EPOLLIN, a.get());
  for (auto& w : workers_) {
    Worker* wp = w.get();
    threads_.emplace_back([this, wp] {
      if (!opts_.cpus.empty()) {
        int cpu = opts_.cpus[size_t(wp->index()) % opts_.cpus.size()];
        if (!pin_current_thread(cpu)) LOG_WARN("worker %d: could not pin to cpu %d", wp->index(), cpu);
      }
      char name[16];
      snprintf(name, sizeof name, "hola-w%d", wp->index());
      pthread_setname_np(pthread_self(), name);
      if (opts_.perf_counters) wp->counters_.open();  // counts this thread only
      if (opts_.sched_slice_us > 0) {
        const long got = set_current_thread_slice_us(opts_.sched_slice_us);
        if (got < 0) LOG_WARN("worker %d: could not set a %d us time slice (errno %ld)", wp->index(), opts_.sched_slice_us, -got);
      }
      wp->slice_us_.store(current_thread_slice_us(), std::memory_order_relaxed);
      cpuprof::note_thread();  // stack bounds for a stall report's capture
      wp->tid_.store(cpuprof::current_tid());
      cpuprof::register_thread();
      wp->scratch_.assign(opts_.read_chunk, 0);
      handler_->on_worker_start(*wp);
      if (opts_.idle_timeout_ms > 0) {
        int period = std::max(50, std::min(1000, opts_.idle_timeout_ms / 4));
        auto sweep = std::make_shared<std::function<void()>>();
        Worker* w = wp;
        std::weak_ptr<std::function<void()>> weak = sweep;
        *sweep = [w, period, weak] {
          w->sweep_idle();
          if (auto f = weak.lock()) w->loop().add_timer(period, [f] { (*f)(); });
        };
        wp->sweep_ = sweep;
        wp->loop().add_timer(period, [sweep] { (*sweep)(); });
      }
      wp->loop().run();
      handler_->on_worker_stop(*wp);
      cpuprof::unregister_thread();
      wp->tid_.store(0);  // gone: no capture signal may be sent to this id any more
    });
  }
}

uint64_t Server::total_requests() const {
  uint64_t n = 0;
  for (auto& w : workers_) n += w->stats_.requests.load(std::memory_order_relaxed);
  return n;
}

namespace {
// A worker's answer to a task posted by shutdown(). Shared, so the task may still run after
// shutdown() stopped waiting for it (a worker that does not answer by the drain deadline is
// not waited for forever).
struct Answer {
  std::atomic<bool> done{false};
  std::atomic<size_t> open{0};
};

bool wait_answer(const Answer& a, std::chrono::steady_clock::time_point until) {
  while (!a.done.load()) {
    if (std::chrono::steady_clock::now() >= until) return false;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  return true;
}
}  // namespace

std::string Server::activity(size_t i) const {
  const Worker& w = *workers_[i];
  const EventLoop::Activity& a = w.loop().activity();
  const uint64_t passes = a.passes.load(std::memory_order_relaxed);
  const uint32_t phase = a.phase.load(std::memory_order_relaxed);
  const uint32_t kind = a.handler_kind.load(std::memory_order_relaxed);
  const uint64_t subject = a.subject.load(std::memory_order_relaxed);
  const uint64_t state = a.state.load(std::memory_order_relaxed);
  const int64_t pass_ns = a.pass_ns.load(std::memory_order_relaxed);
  char head[200];
  snprintf(head, sizeof head, "worker %zu: pass %llu, phase %s, pass began %.1f ms ago, last handler ", i,
           (unsigned long long)passes, EventLoop::phase_name(phase), pass_ns ? (mono_ns() - pass_ns) / 1e6 : -1.0);
  std::string out = head;
  char id[40];
  snprintf(id, sizeof id, "%llx", (unsigned long long)subject);
  if (kind == kConnectionHandler) out += std::string("connection ") + id + " " + Connection::describe_state(state);
  else if (kind == kAcceptorHandler) out += "acceptor fd " + std::to_string(subject);
  else if (kind == 0) out += "loop-internal " + std::to_string(subject) + "/" + std::to_string(state) + " (timer id or deferred round/size)";
  else out += "kind " + std::to_string(kind) + " subject " + id + " state " + std::to_string(state);
  return out;
}

std::string Server::stall_report(size_t i, bool with_stack) { return stall_reports({i}, with_stack)[0]; }

std::vector<std::string> Server::stall_reports(const std::vector<size_t>& which, bool with_stack) {
  // One 100 ms window for all of them (whether each loop's passes advance), then the stacks,
  // within an overall budget: the exit watchdog reports every worker and must finish well
  // before the kubelet's SIGKILL.
  std::vector<uint64_t> p0;
  for (size_t i : which) p0.push_back(workers_[i]->loop().activity().passes.load(std::memory_order_relaxed));
  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  const int64_t stacks_until = mono_ns() + int64_t(2000) * 1000000;
  std::vector<std::string> out;
  for (size_t k = 0; k < which.size(); ++k) {
    const size_t i = which[k];
    const EventLoop::Activity& a = workers_[i]->loop().activity();
    const uint64_t p1 = a.passes.load(std::memory_order_relaxed);
    const bool waiting = a.phase.load(std::memory_order_relaxed) == EventLoop::kWait;
    std::string r = activity(i) + (p1 != p0[k] ? "; passes advancing (" + std::to_string(p1 - p0[k]) + " in 100 ms)"
                                   : waiting  ? "; in epoll_wait, no pass over 100 ms"
                                              : "; passes NOT advancing over 100 ms");
    const int tid = workers_[i]->tid_.load();
    if (with_stack && tid == 0) r += "; thread exited";
    if (with_stack && tid > 0) {
      uintptr_t pcs[cpuprof::kMaxCaptureDepth];
      const int n = mono_ns() < stacks_until ? cpuprof::capture(tid, pcs, cpuprof::kMaxCaptureDepth) : -1;
      r += n > 0 ? "; stack" + cpuprof::describe_pcs(pcs, n)
                 : n == 0 ? "; stack: no answer to the capture signal" : "; stack: skipped (report budget spent)";
    }
    out.push_back(std::move(r));
  }
  return out;
}

void Server::shutdown(int drain_ms) {
  closing_.store(true);
  draining_.store(true);
  const auto start = std::chrono::steady_clock::now();
  const auto deadline = start + std::chrono::milliseconds(drain_ms);
  // A healthy loop answers a posted task within microseconds; even with a zero drain budget
  // each gets this long before it is given up on.
  const auto answer_by = std::max(deadline, start + std::chrono::milliseconds(kAnswerGraceMs));
  for (auto& a : acceptors_) {
    Acceptor* ap = a.get();
    auto ans = std::make_shared<Answer>();
    ap->worker->loop().post([ap, ans] {
      ap->worker->loop().del(ap->fd);
      ::close(ap->fd);
      ap->fd = -1;
      ans->done.store(true);
    });
    if (!wait_answer(*ans, answer_by)) LOG_WARN("drain: worker %d did not close its listener in time", ap->worker->index());
  }
  // Streaming connections close now, and kept-alive ones that have been idle for the grace
  // period; busy ones close after their current response (process() sets close_after_flush_
  // while closing). A connection active just before the drain is given until it has been
  // idle for the grace period to send one more request, answered with `Connection: close`:
  // a closed-loop client has its next request on the way within microseconds, and closing
  // under it would fail that request.
  const int64_t grace_ms = std::min<int64_t>(kDrainIdleGraceMs, drain_ms);
  for (;;) {
    size_t open = 0;
    bool answered = true;
    for (auto& w : workers_) {
      Worker* wp = w.get();
      auto ans = std::make_shared<Answer>();
      wp->loop().post([wp, ans, grace_ms] {
        wp->close_idle_connections(grace_ms);
        ans->open.store(wp->open_connections());
        ans->done.store(true);
      });
      if (!wait_answer(*ans, answer_by)) {
        // Where it is, straight to stderr too: the log writer is not needed to say it.
        const std::string why = stall_report(size_t(wp->index()), true);
        LOG_WARN("drain: worker %d did not answer by the drain deadline: %s", wp->index(), why.c_str());
        const std::string line = "hola: drain: worker did not answer: " + why + "\n";
        ssize_t wr = ::write(2, line.data(), line.size());
        (void)wr;
        answered = false;
        break;
      }
      open += ans->open.load();
    }
    if (!answered || open == 0 || std::chrono::steady_clock::now() >= deadline) break;
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
  }
  for (auto& w : workers_) w->loop().stop();
}

std::string Server::profile_json() const {
  if (!opts_.profile) return "{}";
  StageProfile all;
  for (auto& w : workers_) {
    const StageProfile* p = w->profile_.get();
    all.accept.merge(p->accept);
    all.recv.merge(p->recv);
    all.parse.merge(p->parse);
    all.handle.merge(p->handle);
    all.send.merge(p->send);
    all.batch.merge(p->batch);
  }
  auto one = [](const char* name, const Histogram& h) {
    char buf[256];
    snprintf(buf, sizeof buf, "\"%s\":{\"count\":%llu,\"mean\":%.1f,\"p50\":%llu,\"p99\":%llu,\"p999\":%llu,\"max\":%llu}",
             name, (unsigned long long)h.count(), h.mean(), (unsigned long long)h.percentile(50),
             (unsigned long long)h.percentile(99), (unsigned long long)h.percentile(99.9),
             (unsigned long long)h.max());
    return std::string(buf);
  };
  char steer[160];
  snprintf(steer, sizeof steer, "\"steering\":{\"same_core\":%llu,\"same_l3\":%llu,\"unsteered\":%llu},",
           (unsigned long long)steered_core_.load(), (unsigned long long)steered_.load(),
           (unsigned long long)unsteered_.load());
  std::string loc = "\"locality\":{";
  for (int l = 0; l < kNumLocality; ++l)
    loc += std::string(l ? "," : "") + "\"" + locality_name(l) + "\":" + std::to_string(locality(l));
  loc += "},";
  return "{\"unit\":\"ns (batch: requests per recv)\"," + std::string(steer) + loc + one("accept", all.accept) + "," + one("recv", all.recv) + "," + one("parse", all.parse) + "," +
         one("handle", all.handle) + "," + one("send", all.send) + "," + one("batch", all.batch) + "}";
}

void Server::join() {
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
}

}  // namespace hola::http
