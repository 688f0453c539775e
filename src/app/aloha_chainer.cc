#include "app/aloha_chainer.h"

#include "core/log.h"
#include "http/server.h"
#include "json/json.h"
#include "tracing/tracer.h"

namespace hola::app {

using resilience::Command;
using resilience::Event;

AlohaChainer::AlohaChainer(AlohaOptions o, resilience::Settings s, int num_workers, tracing::Tracer* tracer,
                           const Clock& clock)
    : o_(std::move(o)), tracer_(tracer), clock_(clock) {
  url_ok_ = client::parse_url(o_.url, &target_);
  if (!url_ok_) LOG_ERROR("aloha url '%s' is not an http:// URL; every call will fall back", o_.url.c_str());
  full_url_ = "http://" + target_.host + ":" + std::to_string(target_.port) + target_.base_path + o_.path;
  // HystrixFeign keys: command = Feign configKey, group (and pool) = target name (the URL).
  cmd_ = std::make_unique<Command>(o_.command_key, o_.url, o_.url, s, clock_);
  timeout_ms_.store(s.timeout_enabled ? s.timeout_ms : 0);
  if (url_ok_) addr_ = std::make_unique<client::AddressCache>(target_.host, target_.port);
  pools_.resize(size_t(num_workers));
}

AlohaChainer::~AlohaChainer() { stop(); }

void AlohaChainer::start() {
  if (addr_) {
    addr_->resolve_now();
    addr_->start();
  }
}

void AlohaChainer::stop() {
  if (addr_) addr_->stop();
}

client::ClientPool& AlohaChainer::pool(http::Worker& w) {
  auto& p = pools_[size_t(w.index())];
  if (!p) p = std::make_unique<client::ClientPool>(w.loop(), target_, addr_.get());
  return *p;
}

namespace {
struct Call {
  bool done = false;
  uint64_t req_id = 0;
  EventLoop::TimerId timer = 0;
  int64_t start_ms = 0;
  int64_t start_us = 0;
  tracing::SpanContext ctx;
  bool traced = false;
  std::function<void(const ChainResult&)> cb;
};

ChainResult fallback_result(const char* why) {
  ChainResult r;
  r.fallback = true;
  r.reason = why;
  r.items.push_back(std::string(kFallbackGreeting));
  return r;
}

// Short-circuited / rejected calls are the hot fallbacks when aloha is down: built once.
const ChainResult& static_fallback(Command::Admit a) {
  static const ChainResult short_circuited = fallback_result("short-circuited");
  static const ChainResult rejected = fallback_result("thread-pool-rejected");
  return a == Command::Admit::kShortCircuited ? short_circuited : rejected;
}
}  // namespace

void AlohaChainer::call(http::Worker& w, const tracing::SpanContext* parent,
                        std::function<void(const ChainResult&)> done) {
  auto call = std::make_shared<Call>();
  call->cb = std::move(done);
  call->start_ms = clock_.now_ms();
  EventLoop& loop = w.loop();
  Command* cmd = cmd_.get();

  Command::Admit a = url_ok_ ? cmd->try_start() : Command::Admit::kRun;
  if (a != Command::Admit::kRun) {
    cmd->rejected(clock_.now_ms() - call->start_ms);
    call->cb(static_fallback(a));
    return;
  }
  if (!url_ok_) {
    call->cb(fallback_result("bad-url"));
    return;
  }
  std::string headers;
  if (tracer_ && tracer_->enabled() && parent && parent->sampled) {
    call->ctx = tracer_->new_child(w.index(), *parent);
    call->traced = true;
    tracing::inject(call->ctx, &headers);
  }
  call->start_us = wall_us();
  if (o_.feign_log_basic) LOG_INFO("[%s] ---> GET %s HTTP/1.1", o_.command_key.c_str(), full_url_.c_str());

  const int worker_index = w.index();
  client::ClientPool& p = pool(w);
  const int timeout_ms = timeout_ms_.load(std::memory_order_relaxed);
  bool log = o_.feign_log_basic;
  const std::string key = o_.command_key;
  const std::string url = full_url_;
  tracing::Tracer* tracer = tracer_;
  const Clock* clock = &clock_;

  call->req_id = p.get(target_.base_path + o_.path, headers,
                       [call, cmd, &loop, log, key, url, tracer, worker_index, clock](client::ClientResult&& r) {
    if (call->done) return;
    call->done = true;
    if (call->timer) loop.cancel_timer(call->timer);
    int64_t elapsed = clock->now_ms() - call->start_ms;
    ChainResult res;
    std::string err;
    bool success = false;
    if (r.ok && r.status >= 200 && r.status < 300) {
      std::vector<std::optional<std::string>> items;
      if (json::decode_string_list(r.body, &items, &err)) {
        success = true;
        res.items = std::move(items);
      } else {
        err = "DecodeException: " + err;
      }
    } else if (r.ok) {
      err = "FeignException: status " + std::to_string(r.status) + " reading AlohaService#aloha()";
    } else {
      err = r.error;
    }
    if (log) {
      if (r.ok) LOG_INFO("[%s] <--- HTTP/1.1 %d (%lldms)", key.c_str(), r.status, (long long)elapsed);
      else LOG_INFO("[%s] <--- ERROR %s (%lldms)", key.c_str(), r.error.c_str(), (long long)elapsed);
    }
    if (call->traced && tracer)
      tracer->record_client(worker_index, call->ctx, call->start_us, wall_us(), url, r.ok ? r.status : 0,
                            success ? std::string_view() : std::string_view(err));
    if (success) {
      cmd->complete(Event::kSuccess, elapsed, false, clock->now_ms() - call->start_ms);
    } else {
      cmd->complete(Event::kFailure, elapsed, true, clock->now_ms() - call->start_ms);
      res = fallback_result("failure");
      res.reason = err;
    }
    call->cb(res);
  });

  if (timeout_ms > 0 && !call->done) {
    client::ClientPool* pp = &p;
    call->timer = loop.add_timer(timeout_ms, [call, cmd, pp, log, key, tracer, worker_index, url, clock] {
      if (call->done) return;
      call->done = true;
      call->timer = 0;
      pp->cancel(call->req_id);  // abandon the socket (HystrixTimeoutException)
      int64_t elapsed = clock->now_ms() - call->start_ms;
      if (log) LOG_INFO("[%s] <--- ERROR HystrixTimeoutException (%lldms)", key.c_str(), (long long)elapsed);
      if (call->traced && tracer)
        tracer->record_client(worker_index, call->ctx, call->start_us, wall_us(), url, 0, "timeout");
      cmd->complete(Event::kTimeout, elapsed, true, elapsed);
      call->cb(fallback_result("timeout"));
    });
  }
}

}  // namespace hola::app
