// Optional Prometheus text endpoint (/metrics), an addition beyond the reference
// (SURVEY.md §5.5): per-route request counts from lock-free per-worker counters, server
// connection stats, tracer and Hystrix counters, and a latency histogram for
// /api/hola-chaining (the one route that waits on anything: the aloha call, its 600 ms
// timeout or the fallback). The other routes answer inline in ~0.1 µs (`hola --profile`).
#pragma once
#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

namespace hola::http {
class Server;
}
namespace hola::tracing {
class Tracer;
}
namespace hola::resilience {
class Command;
}

namespace hola::metrics {

class HystrixStream;

class Prometheus {
 public:
  Prometheus(int num_workers, int num_routes);
  void count(int worker, int route) {
    auto& c = counts_[size_t(worker) * size_t(nroutes_) + size_t(route)].v;
    c.store(c.load(std::memory_order_relaxed) + 1, std::memory_order_relaxed);
  }
  // Upper bounds (µs) of the chaining latency buckets; a final +Inf bucket follows.
  static constexpr int kLatencyBuckets = 12;
  static constexpr uint64_t kLatencyBoundsUs[kLatencyBuckets] = {
      1000, 2500, 5000, 10000, 25000, 50000, 100000, 250000, 500000, 600000, 1000000, 2500000};
  // Called on the worker's own thread: relaxed single-writer updates, read by render().
  void observe_chaining_us(int worker, uint64_t us) {
    LatencyHist& h = chain_lat_[size_t(worker)];
    int b = 0;
    while (b < kLatencyBuckets && us > kLatencyBoundsUs[b]) ++b;
    bump(h.bucket[b], 1);
    bump(h.sum_us, us);
    bump(h.count, 1);
  }
  void set_tracer(tracing::Tracer* t) { tracer_ = t; }
  void set_command(resilience::Command* c) { cmd_ = c; }
  void set_config_reloads(std::function<uint64_t()> f) { reloads_ = std::move(f); }
  void set_stream(const HystrixStream* s) { stream_ = s; }
  // Outbound retry counters (Feign Retryer, HttpClient re-sends).
  void set_retries(std::function<uint64_t()> feign, std::function<uint64_t()> transport) {
    feign_retries_ = std::move(feign);
    transport_retries_ = std::move(transport);
  }
  std::string render(http::Server* server) const;

 private:
  struct alignas(64) Counter {
    std::atomic<uint64_t> v{0};
  };
  struct alignas(64) LatencyHist {
    std::atomic<uint64_t> bucket[kLatencyBuckets + 1] = {};
    std::atomic<uint64_t> sum_us{0}, count{0};
  };
  static void bump(std::atomic<uint64_t>& a, uint64_t n) {
    a.store(a.load(std::memory_order_relaxed) + n, std::memory_order_relaxed);
  }
  int nworkers_, nroutes_;
  std::unique_ptr<Counter[]> counts_;
  std::unique_ptr<LatencyHist[]> chain_lat_;
  tracing::Tracer* tracer_ = nullptr;
  resilience::Command* cmd_ = nullptr;
  std::function<uint64_t()> reloads_;
  const HystrixStream* stream_ = nullptr;
  std::function<uint64_t()> feign_retries_, transport_retries_;
};

}  // namespace hola::metrics
