#include "tracing/tracer.h"

#include <arpa/inet.h>
#include <pthread.h>
#include <poll.h>
#include <sys/eventfd.h>
#include <sys/random.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <type_traits>

#include "client/http_client.h"
#include "client/url.h"
#include "core/clock.h"
#include "core/cpuprof.h"
#include "core/log.h"
#include "http/parser.h"
#include "json/json.h"

namespace hola::tracing {

// ---------------------------------------------------------------- SpanRing

SpanRing::SpanRing(size_t cap) {
  size_t c = 1;
  while (c < cap) c <<= 1;
  static_assert(std::is_trivially_default_constructible_v<SpanRecord>);
  buf_.reset(new SpanRecord[c]);
  mask_ = c - 1;
}

bool SpanRing::push(const SpanRecord& r) {
  uint64_t t = tail_.load(std::memory_order_relaxed);
  if (t - head_.load(std::memory_order_acquire) > mask_) return false;
  buf_[t & mask_] = r;
  tail_.store(t + 1, std::memory_order_release);
  return true;
}

size_t SpanRing::drain(std::vector<SpanRecord>* out) {
  uint64_t h = head_.load(std::memory_order_relaxed);
  uint64_t t = tail_.load(std::memory_order_acquire);
  for (uint64_t i = h; i < t; ++i) out->push_back(buf_[i & mask_]);
  head_.store(t, std::memory_order_release);
  return size_t(t - h);
}

// ---------------------------------------------------------------- Tracer

Tracer::Tracer(TracerOptions o, int num_workers) : o_(std::move(o)) {
  stopfd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  for (int i = 0; i < num_workers + 1; ++i) {  // +1: slot for non-worker producers (tests)
    auto w = std::make_unique<WorkerState>();
    uint64_t seed[2] = {0, 0};
    if (getrandom(seed, sizeof seed, 0) != sizeof seed) {
      seed[0] = uint64_t(mono_ns()) ^ (uint64_t(i) << 32);
      seed[1] = uint64_t(wall_us()) * 0x9E3779B97F4A7C15ull;
    }
    w->s0 = seed[0] | 1;
    w->s1 = seed[1] | 2;
    ws_.push_back(std::move(w));
  }
  client::Url u;
  if (!o_.collector_url.empty()) {
    if (client::parse_url(o_.collector_url, &u)) {
      chost_ = u.host;
      cport_ = u.port;
      ctls_ = u.tls;
      cpath_ = u.base_path + (o_.v2 ? "api/v2/spans" : "api/v1/spans");
      collecting_ = true;
      caddr_ = std::make_unique<client::AddressCache>(chost_, cport_);
    } else {
      LOG_WARN("ZIPKIN_SERVER_URL '%s' is not an http:// or https:// URL; spans will be dropped",
               o_.collector_url.c_str());
    }
  }
  // Without a collector, spans are counted and dropped at the source: no rings.
  if (collecting_)
    for (auto& w : ws_) w->ring = std::make_unique<SpanRing>(o_.ring_capacity);
  budget_.store(o_.queue_spans ? int64_t(o_.queue_spans) : INT64_MAX);
}

bool Tracer::admit(int worker) {
  if (o_.queue_spans == 0) return true;
  // Read first: once the budget is spent, the line stays shared and the check costs a load.
  if (budget_.load(std::memory_order_relaxed) <= 0 || budget_.fetch_sub(1, std::memory_order_relaxed) <= 0) {
    auto& d = ws_[size_t(worker)]->over_budget;
    d.store(d.load(std::memory_order_relaxed) + 1, std::memory_order_relaxed);
    return false;
  }
  return true;
}

Tracer::~Tracer() {
  stop();
  if (stopfd_ >= 0) ::close(stopfd_);
}

uint64_t Tracer::next_id(int worker) {
  WorkerState& w = *ws_[size_t(worker)];
  uint64_t s1 = w.s0, s0 = w.s1;
  w.s0 = s0;
  s1 ^= s1 << 23;
  w.s1 = s1 ^ s0 ^ (s1 >> 17) ^ (s0 >> 26);
  uint64_t v = w.s1 + s0;
  return v ? v : 1;
}

ServerSpan Tracer::begin_server(int worker, const http::Request& r) {
  ServerSpan s;
  SpanContext in;
  Extract e = extract(r.b3_trace_id, r.b3_span_id, r.b3_parent_id, r.b3_sampled, r.b3_flags, r.b3_single, &in);
  if (e == Extract::kNotSampled) {
    s.ctx.sampled = false;
    return s;
  }
  if (e == Extract::kContext) {
    s.ctx = in;
    s.shared = true;
  } else {
    if (o_.sample_rate < 1.0) {
      double x = double(next_id(worker) >> 11) * (1.0 / 9007199254740992.0);
      if (x >= o_.sample_rate) {
        s.ctx.sampled = false;
        return s;
      }
    }
    uint64_t id = next_id(worker);
    s.ctx.trace_id = id;
    s.ctx.span_id = id;
    s.ctx.sampled = true;
  }
  if (!collecting_) {
    // No collector (ZIPKIN_SERVER_URL unset): ids still flow downstream via B3, but the span
    // is counted and dropped here rather than after a copy through the ring — the observable
    // result of Brave posting to an unreachable collector (ZipkinResource.java:37-38).
    auto& u = ws_[size_t(worker)]->unreported;
    u.store(u.load(std::memory_order_relaxed) + 1, std::memory_order_relaxed);
    return s;
  }
  if (!admit(worker)) return s;  // sampled (B3 flows on) but not exported this interval
  s.record = true;
  s.start_us = wall_us();
  s.method_len = uint8_t(r.method.size() < sizeof s.method ? r.method.size() : sizeof s.method);
  memcpy(s.method, r.method.data(), s.method_len);
  // http.url = request URL as the servlet container reconstructs it.
  size_t n = 0;
  auto app = [&](std::string_view v) {
    size_t k = v.size() < kMaxUrl - n ? v.size() : kMaxUrl - n;
    memcpy(s.url + n, v.data(), k);
    n += k;
  };
  app("http://");
  app(r.host.empty() ? std::string_view("localhost") : r.host);
  app(r.target);
  s.url_len = uint16_t(n);
  return s;
}

void Tracer::push(int worker, const SpanRecord& r) {
  WorkerState& w = *ws_[size_t(worker)];
  if (w.ring && w.ring->push(r)) w.recorded.store(w.recorded.load(std::memory_order_relaxed) + 1, std::memory_order_relaxed);
  else w.dropped.store(w.dropped.load(std::memory_order_relaxed) + 1, std::memory_order_relaxed);
}

void Tracer::end_server(int worker, const ServerSpan& s, int status) {
  if (!s.record) return;
  SpanRecord r;
  r.trace_hi = s.ctx.trace_hi;
  r.trace_id = s.ctx.trace_id;
  r.span_id = s.ctx.span_id;
  r.parent_id = s.ctx.parent_id;
  r.has_parent = s.ctx.has_parent;
  r.debug = s.ctx.debug;
  r.shared = s.shared;
  r.start_us = s.start_us;
  r.end_us = wall_us();
  r.kind = Kind::kServer;
  r.status = uint16_t(status);
  r.method_len = s.method_len;
  memcpy(r.method, s.method, sizeof r.method);
  r.url_len = s.url_len;
  memcpy(r.url, s.url, s.url_len);
  r.error_len = 0;
  push(worker, r);
}

SpanContext Tracer::new_child(int worker, const SpanContext& parent) {
  SpanContext c = parent;
  c.parent_id = parent.span_id;
  c.has_parent = true;
  c.span_id = next_id(worker);
  return c;
}

void Tracer::record_client(int worker, const SpanContext& ctx, int64_t start_us, int64_t end_us,
                           std::string_view url, int status, std::string_view error) {
  if (!ctx.sampled) return;
  if (!collecting_) {
    auto& u = ws_[size_t(worker)]->unreported;
    u.store(u.load(std::memory_order_relaxed) + 1, std::memory_order_relaxed);
    return;
  }
  if (!admit(worker)) return;
  SpanRecord r;
  r.trace_hi = ctx.trace_hi;
  r.trace_id = ctx.trace_id;
  r.span_id = ctx.span_id;
  r.parent_id = ctx.parent_id;
  r.has_parent = ctx.has_parent;
  r.debug = ctx.debug;
  r.shared = false;
  r.start_us = start_us;
  r.end_us = end_us;
  r.kind = Kind::kClient;
  r.status = uint16_t(status);
  r.method_len = 3;
  memcpy(r.method, "GET", 3);
  r.url_len = uint16_t(url.size() < kMaxUrl ? url.size() : kMaxUrl);
  memcpy(r.url, url.data(), r.url_len);
  r.error_len = uint16_t(error.size() < sizeof r.error ? error.size() : sizeof r.error);
  if (r.error_len) memcpy(r.error, error.data(), r.error_len);
  push(worker, r);
}

void Tracer::endpoint_json(std::string* out) const {
  char ip[INET_ADDRSTRLEN] = "127.0.0.1";
  in_addr a;
  a.s_addr = o_.ipv4;
  if (o_.ipv4) inet_ntop(AF_INET, &a, ip, sizeof ip);
  *out += "{\"serviceName\":";
  json::append_string(out, o_.service_name);
  *out += ",\"ipv4\":\"";
  *out += ip;
  *out += "\",\"port\":";
  *out += std::to_string(o_.port);
  *out += "}";
}

namespace {
std::string lower_name(const SpanRecord& r) {
  std::string n(r.method, r.method_len);
  for (char& c : n) c = char(tolower((unsigned char)c));
  return n;
}
}  // namespace

std::string Tracer::encode_v1(const std::vector<SpanRecord>& spans) const {
  std::string ep;
  endpoint_json(&ep);
  std::string out = "[";
  for (size_t i = 0; i < spans.size(); ++i) {
    const SpanRecord& r = spans[i];
    if (i) out += ',';
    out += "{\"traceId\":\"" + trace_id_hex(r.trace_hi, r.trace_id) + "\",\"id\":\"" + hex64(r.span_id) + "\"";
    if (r.has_parent) out += ",\"parentId\":\"" + hex64(r.parent_id) + "\"";
    out += ",\"name\":";
    json::append_string(&out, lower_name(r));
    // The side that starts a span owns timestamp/duration: clients always, servers only
    // for root spans they created themselves (not for a span id shared with the caller).
    if (r.kind == Kind::kClient || !r.shared) {
      out += ",\"timestamp\":" + std::to_string(r.start_us);
      out += ",\"duration\":" + std::to_string(r.end_us > r.start_us ? r.end_us - r.start_us : 1);
    }
    const char* a0 = r.kind == Kind::kServer ? "sr" : "cs";
    const char* a1 = r.kind == Kind::kServer ? "ss" : "cr";
    out += ",\"annotations\":[{\"timestamp\":" + std::to_string(r.start_us) + ",\"value\":\"" + a0 + "\",\"endpoint\":" + ep +
           "},{\"timestamp\":" + std::to_string(r.end_us) + ",\"value\":\"" + a1 + "\",\"endpoint\":" + ep + "}]";
    out += ",\"binaryAnnotations\":[{\"key\":\"http.url\",\"value\":";
    json::append_string(&out, std::string_view(r.url, r.url_len));
    out += ",\"endpoint\":" + ep + "}";
    if (r.status && (r.status < 200 || r.status > 299)) {
      out += ",{\"key\":\"http.status_code\",\"value\":\"" + std::to_string(r.status) + "\",\"endpoint\":" + ep + "}";
    }
    if (r.error_len) {
      out += ",{\"key\":\"error\",\"value\":";
      json::append_string(&out, std::string_view(r.error, r.error_len));
      out += ",\"endpoint\":" + ep + "}";
    }
    out += "]";
    if (r.debug) out += ",\"debug\":true";
    out += "}";
  }
  out += "]";
  return out;
}

std::string Tracer::encode_v2(const std::vector<SpanRecord>& spans) const {
  std::string ep;
  endpoint_json(&ep);
  std::string out = "[";
  for (size_t i = 0; i < spans.size(); ++i) {
    const SpanRecord& r = spans[i];
    if (i) out += ',';
    out += "{\"traceId\":\"" + trace_id_hex(r.trace_hi, r.trace_id) + "\",\"id\":\"" + hex64(r.span_id) + "\"";
    if (r.has_parent) out += ",\"parentId\":\"" + hex64(r.parent_id) + "\"";
    out += r.kind == Kind::kServer ? ",\"kind\":\"SERVER\"" : ",\"kind\":\"CLIENT\"";
    out += ",\"name\":";
    json::append_string(&out, lower_name(r));
    out += ",\"timestamp\":" + std::to_string(r.start_us);
    out += ",\"duration\":" + std::to_string(r.end_us > r.start_us ? r.end_us - r.start_us : 1);
    out += ",\"localEndpoint\":" + ep;
    if (r.shared) out += ",\"shared\":true";
    if (r.debug) out += ",\"debug\":true";
    out += ",\"tags\":{\"http.url\":";
    json::append_string(&out, std::string_view(r.url, r.url_len));
    if (r.status && (r.status < 200 || r.status > 299)) out += ",\"http.status_code\":\"" + std::to_string(r.status) + "\"";
    if (r.error_len) {
      out += ",\"error\":";
      json::append_string(&out, std::string_view(r.error, r.error_len));
    }
    out += "}}";
  }
  out += "]";
  return out;
}

bool Tracer::post(const std::string& body) {
  if (chost_.empty()) return false;
  client::Url u;
  u.host = chost_;
  u.port = cport_;
  u.tls = ctls_;
  client::BlockingResponse resp;
  const char* hdr = "Content-Type: application/json\r\n";
  bool ok;
  if (running_) {
    // the reporter is up, so is the resolver thread: never resolve here
    sockaddr_storage ss{};
    socklen_t len = 0;
    if (!caddr_->get(&ss, &len, nullptr)) len = 0;
    ok = client::blocking_request(u, &cconn_, &ss, len, "POST", cpath_, hdr, body, 2000, &resp);
  } else {
    // tests: flush() without start()
    ok = client::blocking_request(u, &cconn_, nullptr, 0, "POST", cpath_, hdr, body, 2000, &resp);
  }
  return ok && resp.status >= 200 && resp.status < 300;
}

void Tracer::drain_rings() {
  for (auto& w : ws_)
    if (w->ring) w->ring->drain(&pending_);
}

void Tracer::post_pending() {
  if (pending_.empty()) return;
  if (chost_.empty()) {
    dropped_no_collector_.fetch_add(pending_.size());
    pending_.clear();
    return;
  }
  constexpr size_t kChunk = 500;
  for (size_t i = 0; i < pending_.size(); i += kChunk) {
    const size_t end = std::min(pending_.size(), i + kChunk);
    std::vector<SpanRecord> part(pending_.begin() + long(i), pending_.begin() + long(end));
    std::string body = o_.v2 ? encode_v2(part) : encode_v1(part);
    if (post(body)) {
      reported_.fetch_add(part.size());
    } else {
      // One failed POST drops the rest of the batch too: a collector that is down or times
      // out costs one connect timeout per flush, not one per 500 spans.
      post_failures_.fetch_add(1);
      dropped_no_collector_.fetch_add(pending_.size() - i);
      break;
    }
  }
  pending_.clear();
}

void Tracer::flush() {
  std::lock_guard<std::mutex> g(flush_mu_);
  drain_rings();
  post_pending();
}

void Tracer::run() {
  // Rings are drained every drain_interval_ms (so they stay small and cache-resident);
  // batches are POSTed every flush_interval_ms, or earlier when large. The wait is a poll()
  // on an eventfd rather than a timed condition variable (gcc 11's TSan does not intercept
  // pthread_cond_clockwait, which turns timed cv waits into false race reports).
  cpuprof::register_thread();
  int64_t last_post = mono_ms();
  for (;;) {
    pollfd p{stopfd_, POLLIN, 0};
    ::poll(&p, 1, o_.drain_interval_ms);
    if (stopping_.load(std::memory_order_acquire)) break;
    cpuprof::register_thread();  // no-op once armed (or when not profiling)
    std::lock_guard<std::mutex> f(flush_mu_);
    drain_rings();
    int64_t now = mono_ms();
    if (now - last_post >= o_.flush_interval_ms || pending_.size() >= 5000) {
      post_pending();
      if (now - last_post >= o_.flush_interval_ms && o_.queue_spans)
        budget_.store(int64_t(o_.queue_spans), std::memory_order_relaxed);  // next interval's queue
      last_post = now;
    }
  }
}

void Tracer::start() {
  if (!o_.enabled || running_) return;
  if (caddr_) caddr_->start(0);
  running_ = true;
  th_ = std::thread([this] { run(); });
  pthread_setname_np(th_.native_handle(), "hola-tracer");  // bench.py reads its CPU time
}

void Tracer::stop() {
  if (!running_) return;
  stopping_.store(true, std::memory_order_release);
  uint64_t one = 1;
  ssize_t w = ::write(stopfd_, &one, sizeof one);
  (void)w;
  if (th_.joinable()) th_.join();
  flush();
  cconn_.close();
  running_ = false;
  if (caddr_) caddr_->stop();
}

TracerStats Tracer::stats() const {
  TracerStats s;
  for (auto& w : ws_) {
    s.recorded += w->recorded.load(std::memory_order_relaxed);
    s.dropped_ring += w->dropped.load(std::memory_order_relaxed);
    s.dropped_queue += w->over_budget.load(std::memory_order_relaxed);
  }
  s.reported = reported_.load();
  s.dropped_no_collector = dropped_no_collector_.load();
  for (auto& w : ws_) s.dropped_no_collector += w->unreported.load(std::memory_order_relaxed);
  s.post_failures = post_failures_.load();
  return s;
}

}  // namespace hola::tracing
