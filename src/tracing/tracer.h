// Zipkin tracing — the Brave role (ZipkinResource.java:31-41, ZipKinFilter.java:39-44,
// HolaResource.java:97-108).
//
// Request path cost: one B3 parse, one random id, two clock reads and a fixed-size record
// copied into the worker's single-producer ring. One reporter thread drains all rings every
// 50 ms (so they stay cache-resident) and POSTs Zipkin v1 JSON to
// $ZIPKIN_SERVER_URL/api/v1/spans about every second (v2 optional). When the collector is
// unset or down, spans are dropped and counted — never blocking a worker.
//
// Export budget (the explicit drop policy): at most `queue_spans` spans are admitted per
// flush interval — Brave 3's AbstractSpanCollector queues at most 1000 spans between its
// 1 s flushes and drops (and counts) the rest. The budget is one shared counter that the
// reporter refills each flush; a worker reads it before recording, so once it is spent a
// span costs one read of a cache line nobody writes, and is counted as dropped
// ("queue_full"). Trace ids still propagate downstream in B3 headers either way.
#pragma once
#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "client/url.h"
#include "tracing/b3.h"

namespace hola::http {
struct Request;
}
namespace hola::client {
class AddressCache;
}

namespace hola::tracing {

// Records are kept small (~190 B) so a worker's ring stays L2-resident.
constexpr size_t kMaxUrl = 112;

struct ServerSpan {
  // user-provided: `ServerSpan()` then leaves url[] as it is instead of zeroing all of it
  ServerSpan() {}
  SpanContext ctx;
  int64_t start_us = 0;
  bool record = false;  // sampled: emit on end
  bool shared = false;  // joined the caller's span id (caller owns timestamp/duration)
  uint8_t method_len = 0;
  char method[8] = {0};
  uint16_t url_len = 0;
  char url[kMaxUrl];  // the first url_len bytes; not cleared (a span per request, most never recorded)
};

enum class Kind : uint8_t { kServer = 0, kClient = 1 };

struct SpanRecord {
  uint64_t trace_hi, trace_id, span_id, parent_id;
  int64_t start_us, end_us;
  Kind kind;
  bool has_parent, shared, debug;
  uint16_t status;
  uint8_t method_len;
  char method[8];
  uint16_t url_len;
  char url[kMaxUrl];
  uint16_t error_len;
  char error[32];
};

// Bounded single-producer/single-consumer ring.
class SpanRing {
 public:
  explicit SpanRing(size_t capacity_pow2);
  bool push(const SpanRecord& r);
  size_t drain(std::vector<SpanRecord>* out);

 private:
  // Left uninitialised (SpanRecord is trivial): the pages are first touched by the producing
  // worker, on its own NUMA node.
  std::unique_ptr<SpanRecord[]> buf_;
  size_t mask_;
  alignas(64) std::atomic<uint64_t> head_{0};  // consumer
  alignas(64) std::atomic<uint64_t> tail_{0};  // producer
};

struct TracerOptions {
  std::string service_name = "hola";  // Brave.Builder("hola"), ZipkinResource.java:36
  std::string collector_url;          // $ZIPKIN_SERVER_URL; empty => spans dropped (counted)
  bool enabled = true;
  double sample_rate = 1.0;           // Brave default: sample everything
  int flush_interval_ms = 1000;       // HttpSpanCollector default flush interval
  int drain_interval_ms = 50;         // rings -> reporter buffer (keeps rings small)
  bool v2 = false;                    // POST /api/v2/spans instead of /api/v1/spans
  uint32_t ipv4 = 0;                  // endpoint address (network order)
  int port = 8080;
  size_t ring_capacity = 2048;
  // Spans admitted for export per flush interval (Brave 3 AbstractSpanCollector: a 1000-span
  // queue). 0 = unlimited (bounded only by the rings: ring_capacity per drain interval).
  size_t queue_spans = 1000;
};

struct TracerStats {
  uint64_t recorded = 0, dropped_ring = 0, dropped_no_collector = 0, dropped_queue = 0, reported = 0,
           post_failures = 0;
};

class Tracer {
 public:
  Tracer(TracerOptions o, int num_workers);
  ~Tracer();
  bool enabled() const { return o_.enabled; }
  // A collector is configured: spans are recorded (timestamps and all). Without one they are
  // only counted, so callers skip reading the wall clock for them.
  bool collecting() const { return collecting_; }
  void start();
  void stop();  // flushes what is buffered

  // Server side (ServerRequestInterceptor / ServerResponseInterceptor).
  ServerSpan begin_server(int worker, const http::Request& r);
  void end_server(int worker, const ServerSpan& s, int status);
  // Client side (BraveHttpRequestInterceptor / ResponseInterceptor): child of `parent`.
  SpanContext new_child(int worker, const SpanContext& parent);
  void record_client(int worker, const SpanContext& ctx, int64_t start_us, int64_t end_us,
                     std::string_view url, int status, std::string_view error);

  TracerStats stats() const;
  // Zipkin JSON for a batch (exposed for tests).
  std::string encode_v1(const std::vector<SpanRecord>& spans) const;
  std::string encode_v2(const std::vector<SpanRecord>& spans) const;
  const TracerOptions& options() const { return o_; }
  // Drains all rings and reports synchronously (used by shutdown and tests).
  void flush();

 private:
  uint64_t next_id(int worker);
  // Takes one span from this flush interval's export budget; false (and counted) when spent.
  bool admit(int worker);
  void push(int worker, const SpanRecord& r);
  void run();
  bool post(const std::string& body);
  void endpoint_json(std::string* out) const;

  TracerOptions o_;
  struct alignas(64) WorkerState {
    uint64_t s0, s1;  // xorshift128+
    std::unique_ptr<SpanRing> ring;
    std::atomic<uint64_t> recorded{0}, dropped{0}, unreported{0}, over_budget{0};
  };
  std::vector<std::unique_ptr<WorkerState>> ws_;
  std::thread th_;
  int stopfd_ = -1;
  std::atomic<bool> stopping_{false};
  bool running_ = false;  // start()/stop() are called from the owning (main) thread
  std::mutex flush_mu_;
  std::atomic<uint64_t> reported_{0}, dropped_no_collector_{0}, post_failures_{0};
  alignas(64) std::atomic<int64_t> budget_{0};  // spans still admissible this flush interval
  bool collecting_ = false;            // a collector URL is configured
  std::vector<SpanRecord> pending_;    // drained, not yet posted (reporter thread / flush)
  void drain_rings();
  void post_pending();
  // collector connection (reporter thread only); the collector's name is resolved on the
  // cache's own thread while the reporter runs, so a DNS server that does not answer never
  // holds up a flush or shutdown
  std::unique_ptr<client::AddressCache> caddr_;
  client::BlockingConn cconn_;
  std::string chost_, cpath_;
  int cport_ = 0;
  bool ctls_ = false;  // https:// collector
};

}  // namespace hola::tracing
