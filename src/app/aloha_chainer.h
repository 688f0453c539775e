// The aloha call of /api/hola-chaining: the HystrixFeign proxy built in
// HolaResource.getNextService() (HolaResource.java:94-113) re-designed for an event loop.
//
//   Feign target      http://aloha:8080/ + GET /api/aloha-chaining  (AlohaService.java:25)
//   Hystrix command   "aloha" (method name), group = pool = target URL [lib-default keying,
//                     feign-hystrix 8.15.1 HystrixInvocationHandler; see docs/PARITY.md]
//   retries           Feign's default Retryer.Default(100 ms, 1 s, 5): IO errors and
//                     Retry-After responses re-execute with 1.5x backoff, inside the Hystrix
//                     timeout (HolaResource.java:104-112 configures no .retryer())
//   timeouts          Feign Request.Options defaults, 10 s connect / 60 s read; the read
//                     timeout is armed only when the Hystrix timeout would not come first
//   fallback          ["Aloha response (fallback)"]                  (HolaResource.java:111-112)
//   tracing           one client span per HTTP attempt, child of the server span, + B3
//                     headers (HolaResource.java:97-108)
//   logging           Feign Logger.ErrorLogger at Level.BASIC        (HolaResource.java:109)
#pragma once
#include <atomic>
#include <deque>
#include <memory>
#include <string>
#include <vector>

#include "app/chaining.h"
#include "client/http_client.h"
#include "resilience/hystrix.h"

namespace hola::tracing {
class Tracer;
}

namespace hola::app {

// feign.Retryer.Default: after the n-th failed execution (n = 1, 2, ...) it sleeps
// min(period * 1.5^n, max_period) and executes again, up to max_attempts executions; a
// Retry-After date replaces the backoff (capped at max_period; in the past = no sleep).
struct RetryPolicy {
  int period_ms = 100;
  int max_period_ms = 1000;
  int max_attempts = 5;  // 1 = never retry (Retryer.NEVER_RETRY)
  // Sleep before execution attempt `attempt` + 1, given `attempt` executions have failed.
  int64_t backoff_ms(int attempt) const;
};
bool parse_retry_policy(const std::string& s, RetryPolicy* out);  // "default" | "off" | "P,MAX,N"

struct AlohaOptions {
  std::string url = "http://aloha:8080/";  // HolaResource.java:103
  std::string path = "api/aloha-chaining";  // AlohaService.java:25
  bool feign_log_basic = true;
  // Feign.configKey(AlohaService.class, aloha): the BASIC log tag ("[AlohaService#aloha] ")
  // and the FeignException message.
  std::string config_key = "AlohaService#aloha()";
  std::string command_key = "aloha";  // Hystrix command key (--hystrix-command-key)
  RetryPolicy retry;
  // Feign 8 Request.Options defaults (the reference builds none): 10 s to connect, 60 s to
  // read. They matter only when the Hystrix timeout is disabled or longer: the read timeout
  // is armed per request only then (--feign-timeouts CONNECT_MS,READ_MS).
  int connect_timeout_ms = 10000;
  int read_timeout_ms = 60000;
  // HTTP/1.1 pipelining of concurrent aloha calls over each pooled connection
  // (--aloha-pipeline N, opt-in: the reference's HttpClient sends one request per
  // connection at a time). 1 = off.
  int pipeline = 1;
};

class AlohaChainer final : public Chainer {
 public:
  // `clock` times the Hystrix command (latencies, the breaker's window) and must be monotonic
  // and on mono_ms()'s scale: the timeout deadlines themselves are kept on mono_ms().
  AlohaChainer(AlohaOptions o, resilience::Settings s, int num_workers, tracing::Tracer* tracer,
               const Clock& clock = LoopClock::instance());
  ~AlohaChainer() override;
  bool ok() const { return url_ok_; }
  void start();  // DNS refresher
  void stop();

  void call(http::Worker& w, const tracing::SpanContext* parent,
            ChainDone done) override;

  resilience::Command& command() { return *cmd_; }
  void update_settings(const resilience::Settings& s) {
    cmd_->update_settings(s);
    timeout_ms_.store(s.timeout_enabled ? s.timeout_ms : 0, std::memory_order_relaxed);
    fallback_enabled_.store(s.fallback_enabled, std::memory_order_relaxed);
    read_timeout_armed_.store(read_timeout_for(s), std::memory_order_relaxed);
  }
  const std::string& full_url() const { return full_url_; }
  // Feign re-executions (Retryer) and HttpClient re-sends on a fresh connection, since start.
  uint64_t feign_retries() const { return feign_retries_.load(std::memory_order_relaxed); }
  uint64_t transport_retries() const { return transport_retries_.load(std::memory_order_relaxed); }

 private:
  struct Call;
  struct WorkerCalls;
  client::ClientPool& pool(http::Worker& w);
  WorkerCalls& calls(http::Worker& w);
  uint32_t acquire(WorkerCalls& wc);
  static void release(WorkerCalls& wc, uint32_t slot);
  static bool dead(const WorkerCalls& wc, uint32_t slot, uint32_t gen);
  void execute(http::Worker& w, WorkerCalls& wc, uint32_t slot, uint32_t gen);
  void on_response(http::Worker& w, WorkerCalls& wc, uint32_t slot, uint32_t gen, client::ClientResult&& r);
  void finish(WorkerCalls& wc, uint32_t slot, const ChainResult& res);
  // Pool queue (hystrix.threadpool.*.maxQueueSize > 0): after a bulkhead slot is released,
  // start the calls that were waiting for one, each on its own worker's loop.
  void pump();
  void start_queued(http::Worker& w, uint32_t slot, uint32_t gen);
  static resilience::Command::Queued queued_ref(http::Worker& w, uint32_t slot, uint32_t gen) {
    return {uint64_t(reinterpret_cast<uintptr_t>(&w)), (uint64_t(slot) << 32) | gen};
  }
  void expire(EventLoop& loop, WorkerCalls& wc, client::ClientPool& p, int worker_index);
  void arm(EventLoop& loop, WorkerCalls& wc, client::ClientPool& p, int worker_index);
  AlohaOptions o_;
  client::Url target_;
  bool url_ok_ = false;
  std::string full_url_;
  std::unique_ptr<client::AddressCache> addr_;
  std::unique_ptr<resilience::Command> cmd_;
  std::vector<std::unique_ptr<client::ClientPool>> pools_;
  std::vector<std::unique_ptr<WorkerCalls>> calls_;
  std::string req_path_;  // target base path + aloha path
  std::string log_tag_;   // "[AlohaService#aloha] "
  std::string log_request_line_;  // Feign BASIC request line (constant per target)
  tracing::Tracer* tracer_;
  const Clock& clock_;
  std::atomic<int> timeout_ms_{0};  // 0 = execution timeout disabled (read per call, lock-free)
  std::atomic<uint64_t> feign_retries_{0}, transport_retries_{0};
  // hystrix.command.*.fallback.enabled: false turns every failed call into an error (500)
  std::atomic<bool> fallback_enabled_{true};
  // Feign's read timeout, armed per request only when the Hystrix timeout would not end the
  // call first (0 = not armed).
  std::atomic<int> read_timeout_armed_{0};
  int read_timeout_for(const resilience::Settings& s) const {
    return (!s.timeout_enabled || s.timeout_ms > o_.read_timeout_ms) ? o_.read_timeout_ms : 0;
  }
  // The fallback, or the escaped HystrixRuntimeException when fallbacks are disabled.
  ChainResult failed_result(const char* why) const;
};

}  // namespace hola::app
