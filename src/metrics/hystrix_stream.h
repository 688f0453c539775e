// /hystrix.stream — the HystrixMetricsStreamServlet registered by HystrixServlet.java:13-17
// (SURVEY.md C15, CS5). Server-Sent Events, one `data: {json}` line per command and per
// thread pool every `delay` ms (default 500, `?delay=` query parameter), `ping: ` while no
// command has executed yet, at most 5 concurrent subscribers (503 beyond) [lib-default].
// The JSON field set follows the Hystrix dashboard / Turbine schema.
#pragma once
#include <atomic>
#include <string>
#include <vector>

#include "resilience/hystrix.h"

namespace hola::http {
class Connection;
struct Request;
}

namespace hola::metrics {

class HystrixStream {
 public:
  explicit HystrixStream(int max_connections = 5, int default_delay_ms = 500);
  void add_command(resilience::Command* c) { commands_.push_back(c); }
  void subscribe(http::Connection& c, const http::Request& r);
  int subscribers() const { return subscribers_.load(); }
  // Frames not queued because the subscriber had stopped reading, and subscribers closed
  // after staying stalled for stall_close_ms (default 30 s; hola --hystrix-stream-stall-ms).
  uint64_t frames_skipped() const { return skipped_.load(std::memory_order_relaxed); }
  uint64_t stalled_closed() const { return stalled_closed_.load(std::memory_order_relaxed); }
  // A subscriber with more than this many bytes unsent gets no new frame.
  static constexpr size_t kMaxBacklog = 64 * 1024;
  void set_stall_close_ms(int64_t ms) { stall_close_ms_ = ms; }
  // One SSE payload (all commands + pools), exposed for tests.
  std::string render_events();
  static std::string command_json(const resilience::CommandSnapshot& s);
  static std::string threadpool_json(const resilience::CommandSnapshot& s);

 private:
  struct Ticker;
  int max_connections_;
  int default_delay_ms_;
  int64_t stall_close_ms_ = 30000;
  std::vector<resilience::Command*> commands_;
  std::atomic<int> subscribers_{0};
  std::atomic<uint64_t> skipped_{0}, stalled_closed_{0};
};

}  // namespace hola::metrics
