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
  // One SSE payload (all commands + pools), exposed for tests.
  std::string render_events();
  static std::string command_json(const resilience::CommandSnapshot& s);
  static std::string threadpool_json(const resilience::CommandSnapshot& s);

 private:
  struct Ticker;
  int max_connections_;
  int default_delay_ms_;
  std::vector<resilience::Command*> commands_;
  std::atomic<int> subscribers_{0};
};

}  // namespace hola::metrics
