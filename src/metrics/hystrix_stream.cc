#include "metrics/hystrix_stream.h"

#include <sys/socket.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>

#include "core/clock.h"
#include "http/server.h"
#include "json/json.h"

namespace hola::metrics {

using resilience::CommandSnapshot;
using resilience::Event;

HystrixStream::HystrixStream(int max_connections, int default_delay_ms)
    : max_connections_(max_connections), default_delay_ms_(default_delay_ms) {}

namespace {
void kv(std::string* o, const char* k, int64_t v) {
  *o += ",\"";
  *o += k;
  *o += "\":";
  *o += std::to_string(v);
}
void kv(std::string* o, const char* k, bool v) {
  *o += ",\"";
  *o += k;
  *o += "\":";
  *o += v ? "true" : "false";
}
void kvs(std::string* o, const char* k, const std::string& v) {
  *o += ",\"";
  *o += k;
  *o += "\":";
  json::append_string(o, v);
}
std::string pct_obj(const std::array<int64_t, 9>& p) {
  static const char* kKeys[9] = {"0", "25", "50", "75", "90", "95", "99", "99.5", "100"};
  std::string o = "{";
  for (int i = 0; i < 9; ++i) {
    if (i) o += ',';
    o += "\"";
    o += kKeys[i];
    o += "\":";
    o += std::to_string(p[size_t(i)]);
  }
  return o + "}";
}
int64_t ev(const CommandSnapshot& s, Event e) { return s.rolling[size_t(e)]; }
}  // namespace

std::string HystrixStream::command_json(const CommandSnapshot& s) {
  std::string o = "{\"type\":\"HystrixCommand\"";
  kvs(&o, "name", s.name);
  kvs(&o, "group", s.group);
  kv(&o, "currentTime", s.now_wall_ms);
  kv(&o, "isCircuitBreakerOpen", s.circuit_open);
  kv(&o, "errorPercentage", int64_t(s.health.error_pct));
  kv(&o, "errorCount", s.health.errors);
  kv(&o, "requestCount", s.health.total);
  kv(&o, "rollingCountBadRequests", ev(s, Event::kBadRequest));
  kv(&o, "rollingCountCollapsedRequests", ev(s, Event::kCollapsed));
  kv(&o, "rollingCountEmit", ev(s, Event::kEmit));
  kv(&o, "rollingCountExceptionsThrown", ev(s, Event::kExceptionThrown));
  kv(&o, "rollingCountFailure", ev(s, Event::kFailure));
  kv(&o, "rollingCountFallbackEmit", ev(s, Event::kFallbackEmit));
  kv(&o, "rollingCountFallbackFailure", ev(s, Event::kFallbackFailure));
  kv(&o, "rollingCountFallbackMissing", ev(s, Event::kFallbackMissing));
  kv(&o, "rollingCountFallbackRejection", ev(s, Event::kFallbackRejection));
  kv(&o, "rollingCountFallbackSuccess", ev(s, Event::kFallbackSuccess));
  kv(&o, "rollingCountResponsesFromCache", ev(s, Event::kResponseFromCache));
  kv(&o, "rollingCountSemaphoreRejected", ev(s, Event::kSemaphoreRejected));
  kv(&o, "rollingCountShortCircuited", ev(s, Event::kShortCircuited));
  kv(&o, "rollingCountSuccess", ev(s, Event::kSuccess));
  kv(&o, "rollingCountThreadPoolRejected", ev(s, Event::kThreadPoolRejected));
  kv(&o, "rollingCountTimeout", ev(s, Event::kTimeout));
  kv(&o, "currentConcurrentExecutionCount", s.concurrent);
  kv(&o, "rollingMaxConcurrentExecutionCount", s.rolling_max_concurrent);
  kv(&o, "latencyExecute_mean", s.latency_execute_mean);
  o += ",\"latencyExecute\":" + pct_obj(s.latency_execute);
  kv(&o, "latencyTotal_mean", s.latency_total_mean);
  o += ",\"latencyTotal\":" + pct_obj(s.latency_total);
  const resilience::Settings& p = s.settings;
  kv(&o, "propertyValue_circuitBreakerRequestVolumeThreshold", int64_t(p.request_volume_threshold));
  kv(&o, "propertyValue_circuitBreakerSleepWindowInMilliseconds", int64_t(p.sleep_window_ms));
  kv(&o, "propertyValue_circuitBreakerErrorThresholdPercentage", int64_t(p.error_threshold_pct));
  kv(&o, "propertyValue_circuitBreakerForceOpen", p.force_open);
  kv(&o, "propertyValue_circuitBreakerForceClosed", p.force_closed);
  kv(&o, "propertyValue_circuitBreakerEnabled", p.circuit_enabled);
  kvs(&o, "propertyValue_executionIsolationStrategy", p.isolation);
  kv(&o, "propertyValue_executionIsolationThreadTimeoutInMilliseconds", int64_t(p.timeout_ms));
  kv(&o, "propertyValue_executionTimeoutInMilliseconds", int64_t(p.timeout_ms));
  kv(&o, "propertyValue_executionIsolationThreadInterruptOnTimeout", true);
  o += ",\"propertyValue_executionIsolationThreadPoolKeyOverride\":null";
  kv(&o, "propertyValue_executionIsolationSemaphoreMaxConcurrentRequests", int64_t(p.semaphore_max_concurrent));
  kv(&o, "propertyValue_fallbackIsolationSemaphoreMaxConcurrentRequests", int64_t(p.fallback_max_concurrent));
  kv(&o, "propertyValue_metricsRollingStatisticalWindowInMilliseconds", int64_t(p.rolling_window_ms));
  kv(&o, "propertyValue_requestCacheEnabled", p.request_cache_enabled);
  kv(&o, "propertyValue_requestLogEnabled", p.request_log_enabled);
  kv(&o, "reportingHosts", int64_t(1));
  kvs(&o, "threadPool", s.pool);
  return o + "}";
}

std::string HystrixStream::threadpool_json(const CommandSnapshot& s) {
  std::string o = "{\"type\":\"HystrixThreadPool\"";
  kvs(&o, "name", s.pool);
  kv(&o, "currentTime", s.now_wall_ms);
  kv(&o, "currentActiveCount", s.pool_active);
  kv(&o, "currentCompletedTaskCount", s.pool_completed);
  kv(&o, "currentCorePoolSize", int64_t(s.settings.pool_core_size));
  kv(&o, "currentLargestPoolSize", s.pool_largest);
  kv(&o, "currentMaximumPoolSize", int64_t(s.settings.pool_core_size));
  kv(&o, "currentPoolSize", s.pool_largest);
  kv(&o, "currentQueueSize", s.pool_queue_size);
  kv(&o, "currentTaskCount", s.pool_completed + s.pool_active + s.pool_queue_size);
  kv(&o, "rollingCountThreadsExecuted", s.pool_rolling_executed);
  kv(&o, "rollingMaxActiveThreads", s.pool_rolling_max_active);
  kv(&o, "rollingCountCommandRejections", s.pool_rolling_rejected);
  kv(&o, "propertyValue_queueSizeRejectionThreshold", int64_t(s.settings.pool_queue_reject_threshold));
  kv(&o, "propertyValue_metricsRollingStatisticalWindowInMilliseconds", int64_t(s.settings.rolling_window_ms));
  kv(&o, "reportingHosts", int64_t(1));
  return o + "}";
}

std::string HystrixStream::render_events() {
  std::string out;
  for (resilience::Command* c : commands_) {
    CommandSnapshot s = c->snapshot();
    if (!s.has_executed) continue;  // Hystrix only knows commands that have run
    out += "data: " + command_json(s) + "\n\n";
    // HystrixMetricsPoller publishes a pool only once a task has completed on it
    // (hasExecutedCommandsOnThread): never for SEMAPHORE isolation
    if (s.pool_completed > 0) out += "data: " + threadpool_json(s) + "\n\n";
  }
  if (out.empty()) out = "ping: \n\n";
  return out;
}

namespace {
struct Sub {
  bool alive = true;
  bool chunked = true;
  int delay_ms = 500;
  int64_t stalled_since_ms = 0;  // first tick with bytes pending and no progress (0 = none)
  uint64_t last_sent = 0;        // conn->bytes_sent() at the previous tick
};

std::string chunk(const std::string& data, bool chunked) {
  if (!chunked) return data;
  char hex[20];
  snprintf(hex, sizeof hex, "%zx\r\n", data.size());
  return std::string(hex) + data + "\r\n";
}
}  // namespace

// The pending timer owns the ticker, and the ticker holds the connection (ConnRef): when a
// tick does not re-arm, or the loop drops its timers at shutdown, the connection is released.
struct HystrixStream::Ticker : std::enable_shared_from_this<HystrixStream::Ticker> {
  Ticker(std::shared_ptr<Sub> s, HystrixStream* st, http::Connection* c)
      : sub(std::move(s)), stream(st), conn(c), loop(&c->worker().loop()) {}
  std::shared_ptr<Sub> sub;
  HystrixStream* stream;
  http::ConnRef conn;
  EventLoop* loop;
  void fire() {
    if (!sub->alive || conn->closed()) return;
    // Hystrix's servlet writes block, so a subscriber that stops reading stalls only its own
    // servlet thread. Here writes are queued: past kMaxBacklog unsent bytes the frame is
    // skipped (memory stays bounded), and a subscriber whose socket has taken no bytes for
    // stall_close_ms while some are pending is closed, so that it does not hold one of the
    // max_connections slots forever.
    const uint64_t sent = conn->bytes_sent();
    if (conn->unsent() > 0 && sent == sub->last_sent) {
      const int64_t now = mono_ms();
      if (sub->stalled_since_ms == 0) {
        sub->stalled_since_ms = now;
      } else if (now - sub->stalled_since_ms >= stream->stall_close_ms_) {
        stream->stalled_closed_.fetch_add(1, std::memory_order_relaxed);
        conn->close();
        return;
      }
    } else {
      sub->stalled_since_ms = 0;
    }
    sub->last_sent = sent;
    if (conn->unsent() > kMaxBacklog) stream->skipped_.fetch_add(1, std::memory_order_relaxed);
    else conn->send(chunk(stream->render_events(), sub->chunked));
    auto self = shared_from_this();
    loop->add_timer(sub->delay_ms, [self] { self->fire(); });
  }
};

void HystrixStream::subscribe(http::Connection& c, const http::Request& r) {
  if (subscribers_.fetch_add(1) >= max_connections_) {
    subscribers_.fetch_sub(1);
    const std::string msg = "MaxConcurrentConnections reached: " + std::to_string(max_connections_);
    std::string resp = "HTTP/1.1 503 Service Unavailable\r\nConnection: close\r\nContent-Type: text/plain\r\nContent-Length: " +
                       std::to_string(msg.size()) + "\r\n\r\n" + msg;
    c.send(resp);
    c.close_after_response();
    return;
  }
  auto sub = std::make_shared<Sub>();
  sub->delay_ms = default_delay_ms_;
  // ?delay=<ms>
  std::string_view q = r.query;
  size_t d = q.find("delay=");
  if (d != std::string_view::npos && (d == 0 || q[d - 1] == '&')) {
    int v = atoi(std::string(q.substr(d + 6)).c_str());
    if (v > 0) sub->delay_ms = v < 10 ? 10 : v;
  }
  sub->chunked = r.version_minor >= 1;
  std::string head = "HTTP/1.1 200 OK\r\nContent-Type: text/event-stream;charset=UTF-8\r\n"
                     "Cache-Control: no-cache, no-store, max-age=0, must-revalidate\r\nPragma: no-cache\r\n";
  head += sub->chunked ? "Transfer-Encoding: chunked\r\n\r\n" : "Connection: close\r\n\r\n";
  // A fixed socket send buffer (no autotuning up to tcp_wmem's max, megabytes) bounds what
  // the kernel holds for a subscriber that stops reading; kMaxBacklog bounds the rest.
  const int sndbuf = int(kMaxBacklog);
  setsockopt(c.fd(), SOL_SOCKET, SO_SNDBUF, &sndbuf, sizeof sndbuf);
  c.send(head);
  HystrixStream* self = this;
  c.start_streaming([sub, self] {
    sub->alive = false;
    self->subscribers_.fetch_sub(1);
  });
  auto t = std::make_shared<Ticker>(sub, this, &c);
  // Emit immediately, then every delay_ms until the subscriber goes away.
  t->loop->add_timer(0, [t] { t->fire(); });
}

}  // namespace hola::metrics
