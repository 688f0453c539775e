#include "resilience/hystrix.h"

#include <sched.h>

#include <algorithm>
#include <array>
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
  // Hystrix 1.5.1 reads the timeout from this key only (config.properties:17 sets it); the
  // execution.timeout.* namespace holds just `enabled`. Each key is resolved command-first,
  // then default (cmd_str), which is Archaius' precedence.
  ci("execution.isolation.thread.timeoutInMilliseconds", &s.timeout_ms);
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
  if (cur_ && now >= cur_start_ && now - cur_start_ < bucket_ms_) return *cur_;
  int64_t start = now - (now % bucket_ms_);
  Bucket& b = b_[size_t((now / bucket_ms_) % nb_)];
  if (b.start != start) {
    b.start = start;
    b.c.fill(0);
    b.max_conc = 0;
  }
  cur_ = &b;
  cur_start_ = start;
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
  cur_ = nullptr;
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
  if (cur_ && now >= cur_start_ && now - cur_start_ < bucket_ms_) return *cur_;
  int64_t start = now - (now % bucket_ms_);
  Bucket& b = b_[size_t((now / bucket_ms_) % nb_)];
  if (b.start != start) {
    b.start = start;
    b.h.fill(0);
    b.sum = b.count = 0;
  }
  cur_ = &b;
  cur_start_ = start;
  return b;
}

void RollingPercentile::add(int64_t now, int64_t v) {
  Bucket& b = current(now);
  ++b.h[size_t(bin_of(v))];
  b.sum += v;
  ++b.count;
}

void RollingPercentile::accumulate(int64_t now, Bins* h, int64_t* sum, int64_t* count) const {
  int64_t lo = now - (now % bucket_ms_) - int64_t(window_ms_) + bucket_ms_;
  for (const Bucket& b : b_) {
    if (b.start < lo || b.start > now) continue;
    for (int i = 0; i < kBins; ++i) (*h)[size_t(i)] += b.h[size_t(i)];
    *sum += b.sum;
    *count += b.count;
  }
}

int64_t RollingPercentile::percentile_of(const Bins& h, int64_t count, double p) {
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

int64_t RollingPercentile::percentile(int64_t now, double p) {
  Bins h{};
  int64_t sum = 0, count = 0;
  accumulate(now, &h, &sum, &count);
  return percentile_of(h, count, p);
}

int64_t RollingPercentile::mean(int64_t now) {
  Bins h{};
  int64_t sum = 0, count = 0;
  accumulate(now, &h, &sum, &count);
  return count ? sum / count : 0;
}

// ---------------------------------------------------------------- Command

// The lock of one shard: taken by its worker twice per call, by a reader every snapshot
// period. A test-and-set lock released with a plain release store: one locked instruction per
// critical section where std::mutex has two (its unlock is an atomic exchange too). Each locked
// instruction waits for the store buffer to drain, which made the shard locks 16.6 % of hola
// A's user cycles on the chaining path (profiles/round4/14_user_cycles). Critical sections are
// short; a reader's wait is a few microseconds.
class ShardLock {
 public:
  void lock() {
    while (locked_.exchange(true, std::memory_order_acquire)) {
      // a holder that was descheduled mid-section (another tenant on its CPU): stop spinning
      // after a while and let it run
      for (int spins = 0; locked_.load(std::memory_order_relaxed); ++spins) {
        if (spins < 1024) __builtin_ia32_pause();
        else sched_yield();
      }
    }
  }
  void unlock() { locked_.store(false, std::memory_order_release); }

 private:
  std::atomic<bool> locked_{false};
};

struct alignas(64) Command::Shard {
  ShardLock mu;
  RollingCounter counter, pool_counter;
  RollingPercentile exec_lat, total_lat;
  int64_t completed = 0;
  // Per-thread bulkhead: slots charged to this share (its thread's calls, and slots other
  // threads borrowed from it), on a line of its own; what this shard's thread borrowed from
  // each other share, and how many of its calls in flight were admitted this way (both
  // touched by the owning thread only).
  alignas(64) std::atomic<int64_t> used{0};
  std::array<int32_t, 16> borrowed{};
  int32_t borrowed_total = 0;  // sum of `borrowed`: a release scans it only when non-zero
  int64_t per_thread_inflight = 0;
  explicit Shard(const Settings& s)
      : counter(s.rolling_window_ms, s.rolling_buckets),
        pool_counter(s.rolling_window_ms, s.rolling_buckets),
        exec_lat(s.percentile_window_ms, s.percentile_buckets),
        total_lat(s.percentile_window_ms, s.percentile_buckets) {}
};

Command::Command(std::string name, std::string group, std::string pool, Settings s, const Clock& clock)
    : name_(std::move(name)), group_(std::move(group)), pool_(std::move(pool)), clock_(clock), s_(s) {
  max_queue_.store(s.pool_max_queue, std::memory_order_relaxed);
  apply_hot(s);
  for (int i = 0; i < kShards; ++i) shards_.push_back(std::make_unique<Shard>(s));
}

Command::~Command() = default;

void Command::apply_hot(const Settings& s) {
  circuit_enabled_.store(s.circuit_enabled, std::memory_order_relaxed);
  force_open_.store(s.force_open, std::memory_order_relaxed);
  force_closed_.store(s.force_closed, std::memory_order_relaxed);
  volume_.store(s.request_volume_threshold, std::memory_order_relaxed);
  error_pct_.store(s.error_threshold_pct, std::memory_order_relaxed);
  sleep_window_ms_.store(s.sleep_window_ms, std::memory_order_relaxed);
  pool_core_.store(s.pool_core_size, std::memory_order_relaxed);
  queue_threshold_.store(s.pool_queue_reject_threshold, std::memory_order_relaxed);
  semaphore_.store(s.isolation == "SEMAPHORE", std::memory_order_relaxed);
  sem_max_.store(s.semaphore_max_concurrent, std::memory_order_relaxed);
  health_ms_.store(s.health_snapshot_ms, std::memory_order_relaxed);
}

void Command::hold_shard_for_test(int i, const std::function<void()>& while_held) {
  std::lock_guard<ShardLock> l(shards_[size_t(i) % shards_.size()]->mu);
  while_held();
}

int Command::shard_index() {
  // Threads are dealt shards round-robin on first use: one event-loop worker per shard up
  // to kShards workers, so shard mutexes are in practice uncontended.
  static std::atomic<unsigned> next{0};
  thread_local unsigned idx = next.fetch_add(1, std::memory_order_relaxed);
  return int(idx % kShards);
}

bool Command::per_thread_mode(int64_t core) const {
  return per_thread_.load(std::memory_order_relaxed) && core >= kPerThreadMinPool &&
         !semaphore_.load(std::memory_order_relaxed) && max_queue_.load(std::memory_order_relaxed) <= 0;
}

int64_t Command::per_thread_in_flight() const {
  int64_t n = 0;
  for (const auto& sh : shards_) n += sh->used.load(std::memory_order_relaxed);
  return n;
}

Command::Admit Command::try_start_per_thread(int64_t now, int64_t core) {
  const int si = shard_index();
  Shard& sh = *shards_[size_t(si)];
  if (!per_thread_used_.load(std::memory_order_relaxed)) per_thread_used_.store(true, std::memory_order_relaxed);
  // Calls admitted through the shared count before a reload switched modes still hold their
  // slots: the shares divide what they leave (a line only shared-mode calls write, so this
  // read stays in the cache while the mode holds)
  const int64_t cap = core - active_.load(std::memory_order_relaxed);
  auto share = [cap](int j) { return cap / kShards + (j < cap % kShards ? 1 : 0); };
  auto take = [](Shard& s, int64_t q) {
    int64_t u = s.used.load(std::memory_order_relaxed);
    while (u < q)
      if (s.used.compare_exchange_weak(u, u + 1, std::memory_order_acq_rel, std::memory_order_relaxed)) return true;
    return false;
  };
  int lender = -1;
  bool ok = take(sh, share(si));
  for (int k = 1; !ok && k < kShards; ++k) {
    const int j = (si + k) % kShards;
    if (take(*shards_[size_t(j)], share(j))) {
      ok = true;
      lender = j;
    }
  }
  if (!ok) {
    // every share is full: the pool is (SynchronousQueue, no waiting room)
    std::lock_guard<ShardLock> g(sh.mu);
    sh.counter.add(now, Event::kThreadPoolRejected);
    sh.pool_counter.add(now, Event::kThreadPoolRejected);
    return Admit::kRejected;
  }
  if (lender >= 0) {
    ++sh.borrowed[size_t(lender)];
    ++sh.borrowed_total;
  }
  ++sh.per_thread_inflight;
  const int64_t mine = sh.used.load(std::memory_order_relaxed);
  // the pool's largest size, at least this share's count (a read of a line that is rarely
  // written; snapshots raise it to the pool's total as they see it)
  if (int64_t l = largest_.load(std::memory_order_relaxed); mine > l)
    while (mine > l && !largest_.compare_exchange_weak(l, mine, std::memory_order_relaxed)) {
    }
  std::lock_guard<ShardLock> g(sh.mu);
  sh.counter.update_max_concurrency(now, mine);
  sh.pool_counter.update_max_concurrency(now, mine);
  sh.pool_counter.add(now, Event::kSuccess);  // "threads executed"
  return Admit::kRun;
}

void Command::release_in(Shard& sh) {
  if (sh.per_thread_inflight > 0) {
    // a per-thread admission: give a borrowed slot back to its lender first, else our own
    --sh.per_thread_inflight;
    if (sh.borrowed_total > 0)
      for (size_t j = 0; j < sh.borrowed.size(); ++j)
        if (sh.borrowed[j] > 0) {
          --sh.borrowed[j];
          --sh.borrowed_total;
          shards_[j]->used.fetch_sub(1, std::memory_order_acq_rel);
          return;
        }
    sh.used.fetch_sub(1, std::memory_order_acq_rel);
    return;
  }
  release_slot();
}

HealthCounts Command::health_at(int64_t now) {
  int64_t at = health_at_.load(std::memory_order_acquire);
  if (at < 0 || now - at >= health_ms_.load(std::memory_order_relaxed)) {
    // One thread refreshes; the others keep deciding on the previous snapshot meanwhile
    // (Hystrix's HealthCountsStream publishes snapshots the same way).
    std::unique_lock<std::mutex> g(health_mu_, std::try_to_lock);
    if (g.owns_lock()) {
      at = health_at_.load(std::memory_order_relaxed);
      if (at < 0 || now - at >= health_ms_.load(std::memory_order_relaxed)) {
        std::array<int64_t, kNumEvents> c{};
        for (auto& sh : shards_) {
          std::lock_guard<ShardLock> l(sh->mu);
          auto part = sh->counter.sums(now);
          for (int i = 0; i < kNumEvents; ++i) c[size_t(i)] += part[size_t(i)];
        }
        uint64_t errors = uint64_t(c[size_t(Event::kFailure)] + c[size_t(Event::kTimeout)] +
                                   c[size_t(Event::kThreadPoolRejected)] + c[size_t(Event::kSemaphoreRejected)]);
        uint64_t total = errors + uint64_t(c[size_t(Event::kSuccess)]);
        health_packed_.store((std::min<uint64_t>(total, 0xffffffffu) << 32) | std::min<uint64_t>(errors, 0xffffffffu),
                             std::memory_order_relaxed);
        health_at_.store(now, std::memory_order_release);
      }
    }
  }
  uint64_t packed = health_packed_.load(std::memory_order_relaxed);
  HealthCounts h;
  h.total = int64_t(packed >> 32);
  h.errors = int64_t(packed & 0xffffffffu);
  h.error_pct = h.total > 0 ? int(double(h.errors) / double(h.total) * 100.0) : 0;
  return h;
}

bool Command::is_open(int64_t now) {
  if (open_.load(std::memory_order_acquire)) return true;
  HealthCounts h = health_at(now);
  if (h.total < volume_.load(std::memory_order_relaxed)) return false;
  if (h.error_pct < error_pct_.load(std::memory_order_relaxed)) return false;
  bool expected = false;
  if (open_.compare_exchange_strong(expected, true)) {
    opened_or_tested_.store(now, std::memory_order_release);
    opened_at_.store(now, std::memory_order_relaxed);
    opened_n_.fetch_add(1, std::memory_order_relaxed);
  }
  return true;
}

bool Command::allow_request(int64_t now) {
  if (!circuit_enabled_.load(std::memory_order_relaxed)) return true;
  if (force_open_.load(std::memory_order_relaxed)) return false;
  if (force_closed_.load(std::memory_order_relaxed)) {
    is_open(now);  // still tracks the would-be state
    return true;
  }
  if (!is_open(now)) return true;
  // allowSingleTest(): one trial per sleep window, won by a single CAS.
  int64_t t = opened_or_tested_.load(std::memory_order_acquire);
  if (open_.load(std::memory_order_acquire) && now > t + sleep_window_ms_.load(std::memory_order_relaxed))
    return opened_or_tested_.compare_exchange_strong(t, now);
  return false;
}

bool Command::try_acquire_slot() {
  int64_t a = active_.load(std::memory_order_relaxed);
  const int64_t core = pool_core_.load(std::memory_order_relaxed);
  while (a < core)
    if (active_.compare_exchange_weak(a, a + 1, std::memory_order_acq_rel)) return true;
  return false;
}

void Command::slot_started(int64_t now, int64_t active) {
  int64_t largest = largest_.load(std::memory_order_relaxed);
  while (active > largest && !largest_.compare_exchange_weak(largest, active, std::memory_order_relaxed)) {
  }
  Shard& sh = shard();
  std::lock_guard<ShardLock> g(sh.mu);
  sh.counter.update_max_concurrency(now, active);
  sh.pool_counter.update_max_concurrency(now, active);
  sh.pool_counter.add(now, Event::kSuccess);  // "threads executed"
}

Command::Admit Command::try_start(const Queued* q) {
  int64_t now = clock_.now_ms();
  if (!executed_.load(std::memory_order_relaxed)) executed_.store(true, std::memory_order_relaxed);
  if (!allow_request(now)) {
    Shard& sh = shard();
    std::lock_guard<ShardLock> g(sh.mu);
    sh.counter.add(now, Event::kShortCircuited);
    return Admit::kShortCircuited;
  }
  if (const int64_t core = pool_core_.load(std::memory_order_relaxed); per_thread_mode(core))
    return try_start_per_thread(now, core);
  const bool sem = semaphore_.load(std::memory_order_relaxed);
  int64_t active = active_.fetch_add(1, std::memory_order_acq_rel) + 1;
  // calls admitted per thread before a reload switched modes count against the pool too
  if (per_thread_used_.load(std::memory_order_relaxed)) active += per_thread_in_flight();
  if (sem) {
    // TryableSemaphoreActual.tryAcquire(): the caller's own thread runs the command
    if (active <= sem_max_.load(std::memory_order_relaxed)) {
      Shard& sh = shard();
      std::lock_guard<ShardLock> g(sh.mu);
      sh.counter.update_max_concurrency(now, active);
      return Admit::kRun;
    }
    active_.fetch_sub(1, std::memory_order_acq_rel);
    Shard& sh = shard();
    std::lock_guard<ShardLock> g(sh.mu);
    sh.counter.add(now, Event::kSemaphoreRejected);
    return Admit::kRejected;
  }
  if (active <= pool_core_.load(std::memory_order_relaxed)) {
    slot_started(now, active);
    return Admit::kRun;
  }
  active_.fetch_sub(1, std::memory_order_acq_rel);
  const int max_queue = max_queue_.load(std::memory_order_relaxed);
  if (q && max_queue > 0) {
    // HystrixThreadPool.isQueueSpaceAvailable() (queue size < queueSizeRejectionThreshold),
    // then the LinkedBlockingQueue(maxQueueSize) offer. Under the queue lock, retry the slot
    // first: one released since the check above would otherwise find an empty queue and
    // leave this call waiting beside a free slot.
    std::lock_guard<std::mutex> g(queue_mu_);
    if (try_acquire_slot()) {
      slot_started(now, active_.load(std::memory_order_relaxed));
      return Admit::kRun;
    }
    const size_t cap = size_t(std::max(0, std::min(max_queue, queue_threshold_.load(std::memory_order_relaxed))));
    if (queue_.size() < cap) {
      queue_.push_back(*q);
      return Admit::kQueued;
    }
  }
  // SynchronousQueue (no waiting room), or the queue is at its limit
  Shard& sh = shard();
  std::lock_guard<ShardLock> g(sh.mu);
  sh.counter.add(now, Event::kThreadPoolRejected);
  sh.pool_counter.add(now, Event::kThreadPoolRejected);
  return Admit::kRejected;
}

bool Command::next_queued(Queued* out) {
  if (max_queue_.load(std::memory_order_relaxed) <= 0) return false;  // no queue: no lock per call
  {
    std::lock_guard<std::mutex> g(queue_mu_);
    if (queue_.empty() || !try_acquire_slot()) return false;
    *out = queue_.front();
    queue_.pop_front();
  }
  slot_started(clock_.now_ms(), active_.load(std::memory_order_relaxed));
  return true;
}

bool Command::cancel_queued(const Queued& q) {
  std::lock_guard<std::mutex> g(queue_mu_);
  for (auto it = queue_.begin(); it != queue_.end(); ++it) {
    if (*it == q) {
      queue_.erase(it);
      return true;
    }
  }
  return false;
}

void Command::release_slot() {
  // One read-modify-write on the shared counter (every worker's calls update it): a CAS loop
  // guarding against going below 0 retried under contention, and was most of finish_in's
  // cycles on the chaining path (profiles/round4/14_user_cycles). A release without its
  // acquisition cannot happen; should one, the count is put back at once.
  if (active_.fetch_sub(1, std::memory_order_acq_rel) <= 0) active_.fetch_add(1, std::memory_order_relaxed);
}

void Command::queued_timeout(int64_t total_ms, bool with_fallback) {
  int64_t now = clock_.now_ms();
  Shard& sh = shard();
  std::lock_guard<ShardLock> g(sh.mu);
  sh.counter.add(now, Event::kTimeout);
  if (with_fallback) sh.counter.add(now, Event::kFallbackSuccess);
  sh.total_lat.add(now, total_ms);
}

int64_t Command::queue_size() {
  std::lock_guard<std::mutex> g(queue_mu_);
  return int64_t(queue_.size());
}

void Command::finish_in(Shard& sh, int64_t now, Event outcome, int64_t execute_ms) {
  release_in(sh);
  if (!semaphore_.load(std::memory_order_relaxed)) ++sh.completed;  // tasks run on the pool
  sh.counter.add(now, outcome);
  if (outcome == Event::kSuccess || outcome == Event::kFailure) sh.exec_lat.add(now, execute_ms);
}

void Command::mark_success(int64_t now) {
  // markSuccess(): close the circuit and reset the health stream (only the thread whose CAS
  // closes it does the reset).
  if (!open_.load(std::memory_order_acquire)) return;
  const int64_t since = opened_at_.load(std::memory_order_relaxed);
  bool expected = true;
  if (!open_.compare_exchange_strong(expected, false)) return;
  // No trial runs before the sleep window is over: a success earlier than that is a call that
  // was admitted before the circuit opened.
  (now > since + sleep_window_ms_.load(std::memory_order_relaxed) ? closed_trial_n_ : closed_inflight_n_)
      .fetch_add(1, std::memory_order_relaxed);
  std::lock_guard<std::mutex> h(health_mu_);  // no snapshot refresh may straddle the reset
  for (auto& sh : shards_) {
    std::lock_guard<ShardLock> g(sh->mu);
    sh->counter.reset(now);
  }
  health_packed_.store(0, std::memory_order_relaxed);
  health_at_.store(-1, std::memory_order_release);
}

void Command::finish(Event outcome, int64_t execute_ms) {
  int64_t now = clock_.now_ms();
  {
    Shard& sh = shard();
    std::lock_guard<ShardLock> g(sh.mu);
    finish_in(sh, now, outcome, execute_ms);
  }
  if (outcome == Event::kSuccess) mark_success(now);
}

void Command::complete(Event outcome, int64_t execute_ms, bool with_fallback, int64_t total_ms) {
  int64_t now = clock_.now_ms();
  {
    Shard& sh = shard();
    std::lock_guard<ShardLock> g(sh.mu);
    finish_in(sh, now, outcome, execute_ms);
    if (with_fallback) sh.counter.add(now, Event::kFallbackSuccess);
    sh.total_lat.add(now, total_ms);
  }
  if (outcome == Event::kSuccess) mark_success(now);
}

void Command::rejected(int64_t total_ms, bool with_fallback) {
  int64_t now = clock_.now_ms();
  Shard& sh = shard();
  std::lock_guard<ShardLock> g(sh.mu);
  if (with_fallback) sh.counter.add(now, Event::kFallbackSuccess);
  sh.total_lat.add(now, total_ms);
}

void Command::fallback(Event e) {
  int64_t now = clock_.now_ms();
  Shard& sh = shard();
  std::lock_guard<ShardLock> g(sh.mu);
  sh.counter.add(now, e);
}

void Command::total_latency(int64_t total_ms) {
  int64_t now = clock_.now_ms();
  Shard& sh = shard();
  std::lock_guard<ShardLock> g(sh.mu);
  sh.total_lat.add(now, total_ms);
}

bool Command::circuit_open() { return is_open(clock_.now_ms()); }

HealthCounts Command::health() { return health_at(clock_.now_ms()); }

void Command::update_settings(const Settings& s) {
  std::lock_guard<std::mutex> g(settings_mu_);
  // Window geometry is fixed at construction (as in Hystrix); the rest is dynamic.
  int rw = s_.rolling_window_ms, rb = s_.rolling_buckets, pw = s_.percentile_window_ms, pb = s_.percentile_buckets;
  s_ = s;
  s_.rolling_window_ms = rw;
  s_.rolling_buckets = rb;
  s_.percentile_window_ms = pw;
  s_.percentile_buckets = pb;
  apply_hot(s_);
  if (!executed_.load(std::memory_order_relaxed)) max_queue_.store(s.pool_max_queue, std::memory_order_relaxed);
}

Settings Command::settings() {
  std::lock_guard<std::mutex> g(settings_mu_);
  return s_;
}

CommandSnapshot Command::snapshot() {
  int64_t now = clock_.now_ms();
  CommandSnapshot s;
  s.name = name_;
  s.group = group_;
  s.pool = pool_;
  s.now_wall_ms = wall_ms();
  s.circuit_open = is_open(now);
  s.circuit_opened = opened_n_.load(std::memory_order_relaxed);
  s.circuit_closed_trial = closed_trial_n_.load(std::memory_order_relaxed);
  s.circuit_closed_inflight = closed_inflight_n_.load(std::memory_order_relaxed);
  s.health = health_at(now);
  RollingPercentile::Bins exec_h{}, total_h{};
  int64_t exec_sum = 0, exec_n = 0, total_sum = 0, total_n = 0;
  std::array<int64_t, kNumEvents> pc{};
  for (auto& sh : shards_) {
    std::lock_guard<ShardLock> g(sh->mu);
    auto r = sh->counter.sums(now);
    auto c = sh->counter.cumulative();
    auto p = sh->pool_counter.sums(now);
    for (int i = 0; i < kNumEvents; ++i) {
      s.rolling[size_t(i)] += r[size_t(i)];
      s.cumulative[size_t(i)] += c[size_t(i)];
      pc[size_t(i)] += p[size_t(i)];
    }
    // per-thread bulkhead: each share records its own count, so the pool's maximum is
    // bounded by their sum; one shared count: every shard records the pool's, take the max
    if (per_thread_.load(std::memory_order_relaxed)) {
      s.rolling_max_concurrent += sh->counter.max_concurrency(now);
      s.pool_rolling_max_active += sh->pool_counter.max_concurrency(now);
    } else {
      s.rolling_max_concurrent = std::max(s.rolling_max_concurrent, sh->counter.max_concurrency(now));
      s.pool_rolling_max_active = std::max(s.pool_rolling_max_active, sh->pool_counter.max_concurrency(now));
    }
    s.concurrent += sh->used.load(std::memory_order_relaxed);
    s.pool_completed += sh->completed;
    sh->exec_lat.accumulate(now, &exec_h, &exec_sum, &exec_n);
    sh->total_lat.accumulate(now, &total_h, &total_sum, &total_n);
  }
  s.concurrent += active_.load(std::memory_order_relaxed);
  if (per_thread_.load(std::memory_order_relaxed)) {  // largest pool size as the snapshots see it
    int64_t l = largest_.load(std::memory_order_relaxed);
    while (s.concurrent > l && !largest_.compare_exchange_weak(l, s.concurrent, std::memory_order_relaxed)) {
    }
  }
  static const double kPcts[9] = {0, 25, 50, 75, 90, 95, 99, 99.5, 100};
  for (int i = 0; i < 9; ++i) {
    s.latency_execute[size_t(i)] = RollingPercentile::percentile_of(exec_h, exec_n, kPcts[i]);
    s.latency_total[size_t(i)] = RollingPercentile::percentile_of(total_h, total_n, kPcts[i]);
  }
  s.latency_execute_mean = exec_n ? exec_sum / exec_n : 0;
  s.latency_total_mean = total_n ? total_sum / total_n : 0;
  s.settings = settings();
  if (!s.settings.percentile_enabled) {
    // HystrixRollingPercentile with metrics.rollingPercentile.enabled=false reports -1
    s.latency_execute.fill(-1);
    s.latency_total.fill(-1);
    s.latency_execute_mean = s.latency_total_mean = -1;
  }
  s.pool_active = s.concurrent;
  s.pool_largest = largest_.load(std::memory_order_relaxed);
  s.pool_rolling_executed = pc[size_t(Event::kSuccess)];
  s.pool_rolling_rejected = pc[size_t(Event::kThreadPoolRejected)];
  s.pool_queue_size = queue_size();
  s.has_executed = executed_.load(std::memory_order_relaxed);
  return s;
}

}  // namespace hola::resilience
