#include "app/aloha_chainer.h"

#include <algorithm>

#include "core/clock.h"

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
  calls_.resize(size_t(num_workers));
  req_path_ = target_.base_path + o_.path;
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

// One aloha call in flight. Calls live in reusable slots of their worker's table; a slot's
// generation changes when it is released, so a late response or timeout for a finished call
// is recognised and ignored.
struct AlohaChainer::Call {
  uint32_t gen = 0;
  bool live = false;
  uint64_t req_id = 0;
  int64_t start_ms = 0;
  int64_t start_us = 0;
  tracing::SpanContext ctx;
  bool traced = false;
  std::function<void(const ChainResult&)> cb;
};

// Per worker, touched only on its loop thread. Every call's execution timeout has the same
// delay, so deadlines arrive in arming order: a FIFO replaces a timer-heap entry per call,
// and one loop timer is armed for the oldest deadline. Finished calls at the front are popped
// as they finish, so the FIFO holds about as many entries as there are calls in flight.
struct AlohaChainer::WorkerCalls {
  std::vector<std::unique_ptr<Call>> slots;
  std::vector<uint32_t> free;
  struct Pending {
    int64_t deadline_ms;
    uint32_t slot, gen;
  };
  std::deque<Pending> fifo;
  EventLoop::TimerId timer = 0;
  int64_t timer_at = 0;  // deadline the armed timer fires for (0 = none armed)
};

AlohaChainer::WorkerCalls& AlohaChainer::calls(http::Worker& w) {
  auto& c = calls_[size_t(w.index())];
  if (!c) c = std::make_unique<WorkerCalls>();
  return *c;
}

uint32_t AlohaChainer::acquire(WorkerCalls& wc) {
  uint32_t s;
  if (!wc.free.empty()) {
    s = wc.free.back();
    wc.free.pop_back();
  } else {
    s = uint32_t(wc.slots.size());
    wc.slots.push_back(std::make_unique<Call>());
  }
  Call& c = *wc.slots[s];
  c.live = true;
  c.req_id = 0;
  c.traced = false;
  c.ctx = tracing::SpanContext();
  return s;
}

void AlohaChainer::release(WorkerCalls& wc, uint32_t slot) {
  Call& c = *wc.slots[slot];
  c.live = false;
  ++c.gen;
  c.cb = nullptr;
  wc.free.push_back(slot);
  // Drop finished calls from the front of the timeout FIFO (see WorkerCalls).
  while (!wc.fifo.empty() && dead(wc, wc.fifo.front().slot, wc.fifo.front().gen)) wc.fifo.pop_front();
}

bool AlohaChainer::dead(const WorkerCalls& wc, uint32_t slot, uint32_t gen) {
  const Call& c = *wc.slots[slot];
  return !c.live || c.gen != gen;
}

namespace {
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
  const int64_t start_ms = clock_.now_ms();
  Command* cmd = cmd_.get();
  Command::Admit a = url_ok_ ? cmd->try_start() : Command::Admit::kRun;
  if (a != Command::Admit::kRun) {
    cmd->rejected(clock_.now_ms() - start_ms);
    done(static_fallback(a));
    return;
  }
  if (!url_ok_) {
    done(fallback_result("bad-url"));
    return;
  }
  WorkerCalls& wc = calls(w);
  const uint32_t slot = acquire(wc);
  Call& c = *wc.slots[slot];
  const uint32_t gen = c.gen;
  c.cb = std::move(done);
  c.start_ms = start_ms;
  std::string headers;
  if (tracer_ && tracer_->enabled() && parent && parent->sampled) {
    c.ctx = tracer_->new_child(w.index(), *parent);
    c.traced = true;
    tracing::inject(c.ctx, &headers);
  }
  c.start_us = wall_us();
  if (o_.feign_log_basic) LOG_INFO("[%s] ---> GET %s HTTP/1.1", o_.command_key.c_str(), full_url_.c_str());

  const int worker_index = w.index();
  client::ClientPool& p = pool(w);
  const uint64_t id = p.get(req_path_, headers, [this, &wc, slot, gen, worker_index](client::ClientResult&& r) {
    on_response(wc, slot, gen, worker_index, std::move(r));
  });
  if (dead(wc, slot, gen)) return;  // answered (or failed) synchronously
  c.req_id = id;

  const int timeout_ms = timeout_ms_.load(std::memory_order_relaxed);
  if (timeout_ms <= 0) return;
  const WorkerCalls::Pending e{mono_ms() + timeout_ms, slot, gen};
  if (wc.fifo.empty() || wc.fifo.back().deadline_ms <= e.deadline_ms) {
    wc.fifo.push_back(e);
  } else {
    // The timeout was shortened by a config reload: keep the FIFO in deadline order.
    auto it = std::upper_bound(wc.fifo.begin(), wc.fifo.end(), e.deadline_ms,
                               [](int64_t d, const WorkerCalls::Pending& x) { return d < x.deadline_ms; });
    wc.fifo.insert(it, e);
  }
  arm(w.loop(), wc, p, worker_index);
}

void AlohaChainer::on_response(WorkerCalls& wc, uint32_t slot, uint32_t gen, int worker_index,
                               client::ClientResult&& r) {
  if (dead(wc, slot, gen)) return;
  Call& c = *wc.slots[slot];
  Command* cmd = cmd_.get();
  const int64_t elapsed = clock_.now_ms() - c.start_ms;
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
  if (o_.feign_log_basic) {
    if (r.ok) LOG_INFO("[%s] <--- HTTP/1.1 %d (%lldms)", o_.command_key.c_str(), r.status, (long long)elapsed);
    else LOG_INFO("[%s] <--- ERROR %s (%lldms)", o_.command_key.c_str(), r.error.c_str(), (long long)elapsed);
  }
  if (c.traced && tracer_)
    tracer_->record_client(worker_index, c.ctx, c.start_us, wall_us(), full_url_, r.ok ? r.status : 0,
                           success ? std::string_view() : std::string_view(err));
  if (success) {
    cmd->complete(Event::kSuccess, elapsed, false, clock_.now_ms() - c.start_ms);
  } else {
    cmd->complete(Event::kFailure, elapsed, true, clock_.now_ms() - c.start_ms);
    res = fallback_result("failure");
    res.reason = err;
  }
  auto cb = std::move(c.cb);
  release(wc, slot);  // before the callback: it may start the next call on this worker
  cb(res);
}

// Arms the worker's one timeout timer for the oldest pending deadline, if it is not armed for
// that deadline or an earlier one already.
void AlohaChainer::arm(EventLoop& loop, WorkerCalls& wc, client::ClientPool& p, int worker_index) {
  if (wc.fifo.empty()) return;
  const int64_t at = wc.fifo.front().deadline_ms;
  if (wc.timer_at != 0 && wc.timer_at <= at) return;
  if (wc.timer) loop.cancel_timer(wc.timer);
  wc.timer_at = at;
  wc.timer = loop.add_timer(at - mono_ms(), [this, &loop, &wc, &p, worker_index] {
    wc.timer = 0;
    wc.timer_at = 0;
    expire(loop, wc, p, worker_index);
  });
}

// Times out every call whose deadline has passed (HystrixTimeoutException), then re-arms.
void AlohaChainer::expire(EventLoop& loop, WorkerCalls& wc, client::ClientPool& p, int worker_index) {
  const int64_t now = mono_ms();
  while (!wc.fifo.empty()) {
    const WorkerCalls::Pending e = wc.fifo.front();
    if (dead(wc, e.slot, e.gen)) {
      wc.fifo.pop_front();
      continue;
    }
    if (e.deadline_ms > now) break;
    wc.fifo.pop_front();
    Call& c = *wc.slots[e.slot];
    p.cancel(c.req_id);  // abandon the socket
    const int64_t elapsed = clock_.now_ms() - c.start_ms;
    if (o_.feign_log_basic)
      LOG_INFO("[%s] <--- ERROR HystrixTimeoutException (%lldms)", o_.command_key.c_str(), (long long)elapsed);
    if (c.traced && tracer_) tracer_->record_client(worker_index, c.ctx, c.start_us, wall_us(), full_url_, 0, "timeout");
    cmd_->complete(Event::kTimeout, elapsed, true, elapsed);
    auto cb = std::move(c.cb);
    release(wc, e.slot);
    cb(fallback_result("timeout"));
  }
  arm(loop, wc, p, worker_index);
}

}  // namespace hola::app
