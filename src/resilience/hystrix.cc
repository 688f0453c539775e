#include "resilience/hystrix.h"

#include <algorithm>
#include <cstdlib>

namespace hola::resilience {

const char* event_name(Event e) {
  static const char* kNames[] = {"SUCCESS", "FAILURE", "TIMEOUT", "SHORT_CIRCUITED", "THREAD_POOL_REJECTED",
                                 "SEMAPHORE_REJECTED", "BAD_REQUEST", "FALLBACK_SUCCESS", "FALLBACK_FAILURE",
                                 "FALLBACK_REJECTION", "FALLBACK_MISSING", "EXCEPTION_THROWN",
                                 "RESPONSE_FROM_CACHE", "EMIT", "FALLBACK_EMIT", "COLLAPSED"};
  int i = int(e);
  return (i >= 0 && i < kNumEvents) ? kNames[i] : "?";
}

// ---------------------------------------------------------------- settings

namespace {
bool parse_bool(const std::string& v, bool def) {
  if (v == "true" || v == "TRUE" || v == "True") return true;
  if (v == "false" || v == "FALSE" || v == "False") return false;
  return def;
}
}  // namespace

Settings settings_from(const std::map<std::string, std::string>& p, const std::string& cmd, const std::string& pool) {
  Settings s;
  auto get = [&](const std::string& prefix, const std::string& key, std::string* out) {
    auto it = p.find(prefix + "." + key);
    if (it != p.end()) {
      *out = it->second;
      return true;
    }
    return false;
  };
  auto cmd_str = [&](const std::string& key, std::string* out) {
    return get("hystrix.command." + cmd, key, out) || get("hystrix.command.default", key, out);
  };
  auto pool_str = [&](const std::string& key, std::string* out) {
    return get("hystrix.threadpool." + pool, key, out) || get("hystrix.threadpool.default", key, out);
  };
  std::string v;
  auto ci = [&](const std::string& key, int* dst) {
    if (cmd_str(key, &v)) *dst = atoi(v.c_str());
  };
  auto cb = [&](const std::string& key, bool* dst) {
    if (cmd_str(key, &v)) *dst = parse_bool(v, *dst);
  };
  auto pi = [&](const std::string& key, int* dst) {
    if (pool_str(key, &v)) *dst = atoi(v.c_str());
  };
  // execution.timeout.* is the 1.5 name; execution.isolation.thread.timeoutInMilliseconds the
  // original one still honoured (and the one config.properties:17 uses).
  ci("execution.isolation.thread.timeoutInMilliseconds", &s.timeout_ms);
  ci("execution.timeout.timeoutInMilliseconds", &s.timeout_ms);
  cb("execution.timeout.enabled", &s.timeout_enabled);
  if (cmd_str("execution.isolation.strategy", &v)) s.isolation = v;
  ci("execution.isolation.semaphore.maxConcurrentRequests", &s.semaphore_max_concurrent);
  cb("circuitBreaker.enabled", &s.circuit_enabled);
  ci("circuitBreaker.requestVolumeThreshold", &s.request_volume_threshold);
  ci("circuitBreaker.errorThresholdPercentage", &s.error_threshold_pct);
  ci("circuitBreaker.sleepWindowInMilliseconds", &s.sleep_window_ms);
  cb("circuitBreaker.forceOpen", &s.force_open);
  cb("circuitBreaker.forceClosed", &s.force_closed);
  ci("metrics.rollingStats.timeInMilliseconds", &s.rolling_window_ms);
  ci("metrics.rollingStats.numBuckets", &s.rolling_buckets);
  ci("metrics.healthSnapshot.intervalInMilliseconds", &s.health_snapshot_ms);
  ci("metrics.rollingPercentile.timeInMilliseconds", &s.percentile_window_ms);
  ci("metrics.rollingPercentile.numBuckets", &s.percentile_buckets);
  cb("metrics.rollingPercentile.enabled", &s.percentile_enabled);
  cb("fallback.enabled", &s.fallback_enabled);
  ci("fallback.isolation.semaphore.maxConcurrentRequests", &s.fallback_max_concurrent);
  cb("requestCache.enabled", &s.request_cache_enabled);
  cb("requestLog.enabled", &s.request_log_enabled);
  pi("coreSize", &s.pool_core_size);
  pi("maxQueueSize", &s.pool_max_queue);
  pi("queueSizeRejectionThreshold", &s.pool_queue_reject_threshold);
  pi("keepAliveTimeMinutes", &s.pool_keep_alive_minutes);
  // sanity (Hystrix rejects window % buckets != 0; fall back to defaults instead)
  if (s.rolling_buckets <= 0 || s.rolling_window_ms <= 0 || s.rolling_window_ms % s.rolling_buckets) {
    s.rolling_window_ms = 10000;
    s.rolling_buckets = 10;
  }
  if (s.percentile_buckets <= 0 || s.percentile_window_ms <= 0 || s.percentile_window_ms % s.percentile_buckets) {
    s.percentile_window_ms = 60000;
    s.percentile_buckets = 6;
  }
  if (s.health_snapshot_ms < 0) s.health_snapshot_ms = 500;
  if (s.pool_core_size < 1) s.pool_core_size = 1;
  return s;
}

// ---------------------------------------------------------------- RollingCounter

RollingCounter::RollingCounter(int window_ms, int buckets)
    : window_ms_(window_ms), nb_(buckets), bucket_ms_(window_ms / buckets), b_(size_t(buckets)) {}

RollingCounter::Bucket& RollingCounter::current(int64_t now) {
  int64_t start = now - (now % bucket_ms_);
  Bucket& b = b_[size_t((now / bucket_ms_) % nb_)];
  if (b.start != start) {
    b.start = start;
    b.c.fill(0);
    b.max_conc = 0;
  }
  return b;
}

void RollingCounter::add(int64_t now, Event e, int64_t n) {
  current(now).c[size_t(e)] += n;
  cumulative_[size_t(e)] += n;
}

void RollingCounter::update_max_concurrency(int64_t now, int64_t v) {
  Bucket& b = current(now);
  b.max_conc = std::max(b.max_conc, v);
}

std::array<int64_t, kNumEvents> RollingCounter::sums(int64_t now) {
  std::array<int64_t, kNumEvents> s{};
  int64_t lo = now - (now % bucket_ms_) - int64_t(window_ms_) + bucket_ms_;
  for (const Bucket& b : b_)
    if (b.start >= lo && b.start <= now)
      for (int i = 0; i < kNumEvents; ++i) s[size_t(i)] += b.c[size_t(i)];
  return s;
}

int64_t RollingCounter::max_concurrency(int64_t now) {
  int64_t m = 0;
  int64_t lo = now - (now % bucket_ms_) - int64_t(window_ms_) + bucket_ms_;
  for (const Bucket& b : b_)
    if (b.start >= lo && b.start <= now) m = std::max(m, b.max_conc);
  return m;
}

void RollingCounter::reset(int64_t) {
  for (Bucket& b : b_) {
    b.start = -1;
    b.c.fill(0);
    b.max_conc = 0;
  }
}

// ---------------------------------------------------------------- RollingPercentile

RollingPercentile::RollingPercentile(int window_ms, int buckets)
    : window_ms_(window_ms), nb_(buckets), bucket_ms_(window_ms / buckets), b_(size_t(buckets)) {}

int RollingPercentile::bin_of(int64_t v) {
  if (v < 0) v = 0;
  if (v < 64) return int(v);
  int msb = 63 - __builtin_clzll(uint64_t(v));
  int sub = int((uint64_t(v) >> (msb - 5)) & 31);
  int b = 64 + (msb - 6) * 32 + sub;
  return b >= kBins ? kBins - 1 : b;
}

int64_t RollingPercentile::bin_value(int b) {
  if (b < 64) return b;
  int oct = (b - 64) / 32, sub = (b - 64) % 32;
  int msb = oct + 6;
  return (int64_t(1) << msb) + (int64_t(sub) << (msb - 5));
}

RollingPercentile::Bucket& RollingPercentile::current(int64_t now) {
  int64_t start = now - (now % bucket_ms_);
  Bucket& b = b_[size_t((now / bucket_ms_) % nb_)];
  if (b.start != start) {
    b.start = start;
    b.h.fill(0);
    b.sum = b.count = 0;
  }
  return b;
}

void RollingPercentile::add(int64_t now, int64_t v) {
  Bucket& b = current(now);
  ++b.h[size_t(bin_of(v))];
  b.sum += v;
  ++b.count;
}

void RollingPercentile::merged(int64_t now, std::array<uint64_t, kBins>* h, int64_t* sum, int64_t* count) {
  h->fill(0);
  *sum = *count = 0;
  int64_t lo = now - (now % bucket_ms_) - int64_t(window_ms_) + bucket_ms_;
  for (const Bucket& b : b_) {
    if (b.start < lo || b.start > now) continue;
    for (int i = 0; i < kBins; ++i) (*h)[size_t(i)] += b.h[size_t(i)];
    *sum += b.sum;
    *count += b.count;
  }
}

int64_t RollingPercentile::percentile(int64_t now, double p) {
  std::array<uint64_t, kBins> h;
  int64_t sum, count;
  merged(now, &h, &sum, &count);
  if (count == 0) return 0;
  if (p <= 0) {
    for (int i = 0; i < kBins; ++i)
      if (h[size_t(i)]) return bin_value(i);
  }
  double rank = p / 100.0 * double(count);
  uint64_t need = uint64_t(rank + 0.999999);
  if (need < 1) need = 1;
  uint64_t acc = 0;
  for (int i = 0; i < kBins; ++i) {
    acc += h[size_t(i)];
    if (acc >= need) return bin_value(i);
  }
  return bin_value(kBins - 1);
}

int64_t RollingPercentile::mean(int64_t now) {
  std::array<uint64_t, kBins> h;
  int64_t sum, count;
  merged(now, &h, &sum, &count);
  return count ? sum / count : 0;
}

// ---------------------------------------------------------------- Command

Command::Command(std::string name, std::string group, std::string pool, Settings s, const Clock& clock)
    : name_(std::move(name)),
      group_(std::move(group)),
      pool_(std::move(pool)),
      s_(s),
      clock_(clock),
      counter_(s.rolling_window_ms, s.rolling_buckets),
      pool_counter_(s.rolling_window_ms, s.rolling_buckets),
      exec_lat_(s.percentile_window_ms, s.percentile_buckets),
      total_lat_(s.percentile_window_ms, s.percentile_buckets) {}

HealthCounts Command::health_locked(int64_t now) {
  if (health_at_ >= 0 && now - health_at_ < s_.health_snapshot_ms) return health_cache_;
  auto c = counter_.sums(now);
  HealthCounts h;
  h.errors = c[size_t(Event::kFailure)] + c[size_t(Event::kTimeout)] + c[size_t(Event::kThreadPoolRejected)] +
             c[size_t(Event::kSemaphoreRejected)];
  h.total = h.errors + c[size_t(Event::kSuccess)];
  h.error_pct = h.total > 0 ? int(double(h.errors) / double(h.total) * 100.0) : 0;
  health_cache_ = h;
  health_at_ = now;
  return h;
}

bool Command::is_open_locked(int64_t now) {
  if (open_) return true;
  HealthCounts h = health_locked(now);
  if (h.total < s_.request_volume_threshold) return false;
  if (h.error_pct < s_.error_threshold_pct) return false;
  open_ = true;
  opened_or_tested_ = now;
  return true;
}

bool Command::allow_request_locked(int64_t now) {
  if (!s_.circuit_enabled) return true;
  if (s_.force_open) return false;
  if (s_.force_closed) {
    is_open_locked(now);  // still tracks the would-be state
    return true;
  }
  if (!is_open_locked(now)) return true;
  // allowSingleTest(): one trial per sleep window
  if (open_ && now > opened_or_tested_ + s_.sleep_window_ms) {
    opened_or_tested_ = now;
    return true;
  }
  return false;
}

Command::Admit Command::try_start() {
  std::lock_guard<std::mutex> g(mu_);
  int64_t now = clock_.now_ms();
  executed_ = true;
  if (!allow_request_locked(now)) {
    counter_.add(now, Event::kShortCircuited);
    return Admit::kShortCircuited;
  }
  if (active_ >= s_.pool_core_size) {  // SynchronousQueue: no waiting room
    counter_.add(now, Event::kThreadPoolRejected);
    pool_counter_.add(now, Event::kThreadPoolRejected);
    return Admit::kRejected;
  }
  ++active_;
  largest_ = std::max(largest_, active_);
  counter_.update_max_concurrency(now, active_);
  pool_counter_.update_max_concurrency(now, active_);
  pool_counter_.add(now, Event::kSuccess);  // "threads executed"
  return Admit::kRun;
}

void Command::finish_locked(int64_t now, Event outcome, int64_t execute_ms) {
  if (active_ > 0) --active_;
  ++completed_;
  counter_.add(now, outcome);
  if (outcome == Event::kSuccess) {
    exec_lat_.add(now, execute_ms);
    if (open_) {  // markSuccess(): close and reset the health stream
      open_ = false;
      counter_.reset(now);
      health_at_ = -1;
    }
  } else if (outcome == Event::kFailure) {
    exec_lat_.add(now, execute_ms);
  }
}

void Command::finish(Event outcome, int64_t execute_ms) {
  std::lock_guard<std::mutex> g(mu_);
  finish_locked(clock_.now_ms(), outcome, execute_ms);
}

void Command::complete(Event outcome, int64_t execute_ms, bool with_fallback, int64_t total_ms) {
  std::lock_guard<std::mutex> g(mu_);
  int64_t now = clock_.now_ms();
  finish_locked(now, outcome, execute_ms);
  if (with_fallback) counter_.add(now, Event::kFallbackSuccess);
  total_lat_.add(now, total_ms);
}

void Command::rejected(int64_t total_ms) {
  std::lock_guard<std::mutex> g(mu_);
  int64_t now = clock_.now_ms();
  counter_.add(now, Event::kFallbackSuccess);
  total_lat_.add(now, total_ms);
}

void Command::fallback(Event e) {
  std::lock_guard<std::mutex> g(mu_);
  counter_.add(clock_.now_ms(), e);
}

void Command::total_latency(int64_t total_ms) {
  std::lock_guard<std::mutex> g(mu_);
  total_lat_.add(clock_.now_ms(), total_ms);
}

bool Command::circuit_open() {
  std::lock_guard<std::mutex> g(mu_);
  return is_open_locked(clock_.now_ms());
}

HealthCounts Command::health() {
  std::lock_guard<std::mutex> g(mu_);
  return health_locked(clock_.now_ms());
}

void Command::update_settings(const Settings& s) {
  std::lock_guard<std::mutex> g(mu_);
  // Window geometry is fixed at construction (as in Hystrix); the rest is dynamic.
  int rw = s_.rolling_window_ms, rb = s_.rolling_buckets, pw = s_.percentile_window_ms, pb = s_.percentile_buckets;
  s_ = s;
  s_.rolling_window_ms = rw;
  s_.rolling_buckets = rb;
  s_.percentile_window_ms = pw;
  s_.percentile_buckets = pb;
}

Settings Command::settings() {
  std::lock_guard<std::mutex> g(mu_);
  return s_;
}

CommandSnapshot Command::snapshot() {
  std::lock_guard<std::mutex> g(mu_);
  int64_t now = clock_.now_ms();
  CommandSnapshot s;
  s.name = name_;
  s.group = group_;
  s.pool = pool_;
  s.now_wall_ms = wall_ms();
  s.circuit_open = is_open_locked(now);
  s.health = health_locked(now);
  s.rolling = counter_.sums(now);
  s.cumulative = counter_.cumulative();
  s.concurrent = active_;
  s.rolling_max_concurrent = counter_.max_concurrency(now);
  static const double kPcts[9] = {0, 25, 50, 75, 90, 95, 99, 99.5, 100};
  for (int i = 0; i < 9; ++i) {
    s.latency_execute[size_t(i)] = exec_lat_.percentile(now, kPcts[i]);
    s.latency_total[size_t(i)] = total_lat_.percentile(now, kPcts[i]);
  }
  s.latency_execute_mean = exec_lat_.mean(now);
  s.latency_total_mean = total_lat_.mean(now);
  s.settings = s_;
  auto pc = pool_counter_.sums(now);
  s.pool_active = active_;
  s.pool_largest = largest_;
  s.pool_completed = completed_;
  s.pool_rolling_executed = pc[size_t(Event::kSuccess)];
  s.pool_rolling_rejected = pc[size_t(Event::kThreadPoolRejected)];
  s.pool_rolling_max_active = pool_counter_.max_concurrency(now);
  s.has_executed = executed_;
  return s;
}

}  // namespace hola::resilience
