// Optional Prometheus text endpoint (/metrics), an addition beyond the reference
// (SURVEY.md §5.5): per-route request counts from lock-free per-worker counters, server
// connection stats, tracer and Hystrix counters.
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

class Prometheus {
 public:
  Prometheus(int num_workers, int num_routes);
  void count(int worker, int route) {
    auto& c = counts_[size_t(worker) * size_t(nroutes_) + size_t(route)].v;
    c.store(c.load(std::memory_order_relaxed) + 1, std::memory_order_relaxed);
  }
  void set_tracer(tracing::Tracer* t) { tracer_ = t; }
  void set_command(resilience::Command* c) { cmd_ = c; }
  void set_config_reloads(std::function<uint64_t()> f) { reloads_ = std::move(f); }
  std::string render(http::Server* server) const;

 private:
  struct alignas(64) Counter {
    std::atomic<uint64_t> v{0};
  };
  int nworkers_, nroutes_;
  std::unique_ptr<Counter[]> counts_;
  tracing::Tracer* tracer_ = nullptr;
  resilience::Command* cmd_ = nullptr;
  std::function<uint64_t()> reloads_;
};

}  // namespace hola::metrics
