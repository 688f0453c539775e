// Hystrix-compatible resilience for the aloha call:
// circuit breaker + bulkhead + timeout + fallback, with Hystrix's rolling-window metrics
// so /hystrix.stream can report dashboard-compatible JSON.
//
// Semantics follow Hystrix 1.5.1 (pom.xml:60) [lib-default]:
//  * health counts over a rolling window (10 s in 10 buckets), recomputed at most every
//    healthSnapshot interval (500 ms);
//  * the breaker trips when requests >= requestVolumeThreshold (tuned to 5 in
//    config.properties:19) and error% >= errorThresholdPercentage (50);
//    errors = FAILURE + TIMEOUT + THREAD_POOL_REJECTED + SEMAPHORE_REJECTED;
//  * while open, one trial request is let through every sleepWindow (5 s); a success closes
//    the circuit and resets the counts;
//  * bulkhead = thread pool of coreSize 10 with no queue (maxQueueSize -1): the 11th
//    concurrent call is rejected straight to the fallback. With maxQueueSize > 0 (fixed when
//    the pool is created) calls beyond coreSize wait in a FIFO while it holds fewer than
//    min(maxQueueSize, queueSizeRejectionThreshold) (the threshold is dynamic), and are
//    rejected beyond that; a queued call's timeout runs from its start, queue wait included;
//  * execution.isolation.strategy=SEMAPHORE swaps the pool for a semaphore of
//    semaphore.maxConcurrentRequests (10): rejections are SEMAPHORE_REJECTED, nothing queues,
//    and the pool reports no tasks (so the stream shows no HystrixThreadPool frame);
//  * execution timeout 1000 ms by default, 600 ms per config.properties:17.
// All time comes from an injectable Clock so tests can drive the state machine.
#pragma once
#include <array>
#include <atomic>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <functional>
#include <mutex>
#include <string>
#include <vector>

#include "core/clock.h"

namespace hola::resilience {

enum class Event : int {
  kSuccess = 0, kFailure, kTimeout, kShortCircuited, kThreadPoolRejected, kSemaphoreRejected,
  kBadRequest, kFallbackSuccess, kFallbackFailure, kFallbackRejection, kFallbackMissing,
  kExceptionThrown, kResponseFromCache, kEmit, kFallbackEmit, kCollapsed, kNumEvents
};
constexpr int kNumEvents = int(Event::kNumEvents);
const char* event_name(Event e);

struct Settings {
  // command
  int timeout_ms = 1000;
  bool timeout_enabled = true;
  bool circuit_enabled = true;
  int request_volume_threshold = 20;
  int error_threshold_pct = 50;
  int sleep_window_ms = 5000;
  bool force_open = false;
  bool force_closed = false;
  int rolling_window_ms = 10000;
  int rolling_buckets = 10;
  int health_snapshot_ms = 500;
  int percentile_window_ms = 60000;
  int percentile_buckets = 6;
  bool percentile_enabled = true;
  bool fallback_enabled = true;
  int fallback_max_concurrent = 10;
  int semaphore_max_concurrent = 10;
  std::string isolation = "THREAD";
  bool request_cache_enabled = true;
  bool request_log_enabled = true;
  // thread pool (bulkhead)
  int pool_core_size = 10;
  int pool_max_queue = -1;
  int pool_queue_reject_threshold = 5;
  int pool_keep_alive_minutes = 1;
};

// Resolves `hystrix.command.<cmd>.*` > `hystrix.command.default.*` > built-in defaults, and
// `hystrix.threadpool.<pool>.*` > `hystrix.threadpool.default.*`.
Settings settings_from(const std::map<std::string, std::string>& props, const std::string& command_key,
                       const std::string& pool_key);

// Bucketed rolling event counter.
class RollingCounter {
 public:
  RollingCounter(int window_ms, int buckets);
  RollingCounter(const RollingCounter&) = delete;  // cur_ points into b_
  RollingCounter& operator=(const RollingCounter&) = delete;
  void add(int64_t now_ms, Event e, int64_t n = 1);
  void update_max_concurrency(int64_t now_ms, int64_t v);
  std::array<int64_t, kNumEvents> sums(int64_t now_ms);
  int64_t max_concurrency(int64_t now_ms);
  std::array<int64_t, kNumEvents> cumulative() const { return cumulative_; }
  void reset(int64_t now_ms);

 private:
  struct Bucket {
    int64_t start = -1;
    std::array<int64_t, kNumEvents> c{};
    int64_t max_conc = 0;
  };
  Bucket& current(int64_t now_ms);
  int window_ms_, nb_, bucket_ms_;
  std::vector<Bucket> b_;
  std::array<int64_t, kNumEvents> cumulative_{};
  // The bucket the last call landed in: a call in the same bucket interval finds it with two
  // compares instead of three integer divisions. Reset with the buckets.
  Bucket* cur_ = nullptr;
  int64_t cur_start_ = 0;
};

// Rolling latency percentiles (log-linear histogram per bucket, 0.1 ms .. ~1 h).
class RollingPercentile {
 public:
  static constexpr int kBins = 512;
  using Bins = std::array<uint64_t, kBins>;
  RollingPercentile(int window_ms, int buckets);
  RollingPercentile(const RollingPercentile&) = delete;  // cur_ points into b_
  RollingPercentile& operator=(const RollingPercentile&) = delete;
  void add(int64_t now_ms, int64_t value_ms);
  // Percentile in ms for p in [0,100]; mean. Returns 0 when empty.
  int64_t percentile(int64_t now_ms, double p);
  int64_t mean(int64_t now_ms);
  // Adds this window's live buckets into (*h, *sum, *count): merging across shards.
  void accumulate(int64_t now_ms, Bins* h, int64_t* sum, int64_t* count) const;
  static int64_t percentile_of(const Bins& h, int64_t count, double p);

 private:
  static int bin_of(int64_t v);
  static int64_t bin_value(int b);
  struct Bucket {
    int64_t start = -1;
    Bins h{};
    int64_t sum = 0, count = 0;
  };
  Bucket& current(int64_t now_ms);
  int window_ms_, nb_, bucket_ms_;
  std::vector<Bucket> b_;
  Bucket* cur_ = nullptr;  // as RollingCounter's
  int64_t cur_start_ = 0;
};

struct HealthCounts {
  int64_t total = 0, errors = 0;
  int error_pct = 0;
};

struct CommandSnapshot {
  std::string name, group, pool;
  int64_t now_wall_ms = 0;
  bool circuit_open = false;
  uint64_t circuit_opened = 0, circuit_closed_trial = 0, circuit_closed_inflight = 0;
  HealthCounts health;
  std::array<int64_t, kNumEvents> rolling{}, cumulative{};
  int64_t concurrent = 0, rolling_max_concurrent = 0;
  // percentiles 0,25,50,75,90,95,99,99.5,100 + mean
  std::array<int64_t, 9> latency_execute{}, latency_total{};
  int64_t latency_execute_mean = 0, latency_total_mean = 0;
  Settings settings;
  // thread pool view
  int64_t pool_active = 0, pool_largest = 0, pool_completed = 0, pool_rolling_executed = 0,
          pool_rolling_max_active = 0, pool_rolling_rejected = 0, pool_queue_size = 0;
  bool has_executed = false;
};

// Concurrency: the request path never takes a shared lock. Breaker state, the health
// snapshot and the bulkhead are atomics (as in Hystrix: AtomicBoolean circuitOpen, AtomicLong
// circuitOpenedOrLastTestedTime, a volatile HealthCounts). Rolling counters and latency
// histograms are sharded per thread, each shard behind its own (uncontended) mutex, and
// merged when the health snapshot is refreshed or the stream/metrics read them.
class Command {
 public:
  Command(std::string name, std::string group, std::string pool, Settings s, const Clock& clock);
  ~Command();

  // The caller's handle for a call waiting in the pool queue (opaque to the command).
  struct Queued {
    uint64_t a = 0, b = 0;
    bool operator==(const Queued& o) const { return a == o.a && b == o.b; }
  };
  enum class Admit { kRun, kQueued, kShortCircuited, kRejected };
  // Breaker + bulkhead admission. kRun takes a bulkhead slot that finish()/complete()
  // releases. kQueued (only with a queue handle and maxQueueSize > 0) parks `q` in the pool
  // queue: it gets a slot through next_queued().
  Admit try_start(const Queued* q = nullptr);
  // After a slot is released: if a call waits, takes a slot for it and pops it (the caller
  // starts it, or hands the slot back with release_slot()). Call until it returns false.
  bool next_queued(Queued* out);
  // Removes a call from the queue (its timeout fired first); false if it was already popped.
  bool cancel_queued(const Queued& q);
  // Hands back a slot taken by next_queued() for a call that can no longer run.
  void release_slot();
  // A queued call that timed out before getting a slot: TIMEOUT + fallback + total latency,
  // no slot to release.
  void queued_timeout(int64_t total_ms, bool with_fallback = true);
  int64_t queue_size();
  // Outcome of an admitted execution: kSuccess, kFailure, kTimeout or kBadRequest.
  void finish(Event outcome, int64_t execute_ms);
  // After a short-circuit/rejection/failure/timeout the fallback runs; record its result
  // and the total latency of the whole command.
  void fallback(Event fallback_event);
  void total_latency(int64_t total_ms);
  // finish() + optional fallback() + total_latency() in one shard visit.
  void complete(Event outcome, int64_t execute_ms, bool with_fallback, int64_t total_ms);
  // Short-circuit / rejection path: fallback (unless disabled) + total latency in one shard visit.
  void rejected(int64_t total_ms, bool with_fallback = true);

  // Per-thread bulkhead (opt-in, for callers whose calls finish on the thread that started
  // them: the event-loop workers). With a thread pool of kPerThreadMinPool or more and no
  // queue, each thread's calls take slots from its own share of the pool (pool / 16 per
  // shard) with a compare-and-swap on its own cache line; a thread whose share is used up
  // borrows a slot from another share, so a call is still only rejected when every share is
  // full, as with one shared count. The shared count was two contended read-modify-writes
  // per call from every worker. In this mode the pool's rolling maximum concurrency is the
  // sum of each share's maximum in the window (an upper bound of the pool's), and its
  // largest size is taken when snapshots are read. Smaller pools (the reference's 10) and
  // queued pools keep the one exact shared count.
  static constexpr int64_t kPerThreadMinPool = 64;
  void set_per_thread_bulkhead(bool on) { per_thread_.store(on, std::memory_order_relaxed); }

  bool circuit_open();            // evaluates health like HystrixCircuitBreaker.isOpen()
  HealthCounts health();
  CommandSnapshot snapshot();
  void update_settings(const Settings& s);
  Settings settings();
  const std::string& name() const { return name_; }
  // Tests (bench/probes/hystrix_shard_race.cc under TSan): runs `while_held` with shard `i`'s
  // lock held, as a worker's finish() holds it, so that refreshes and other workers' calls
  // can be driven against a held shard.
  void hold_shard_for_test(int i, const std::function<void()>& while_held);

 private:
  struct Shard;
  static constexpr int kShards = 16;
  static int shard_index();
  Shard& shard() { return *shards_[size_t(shard_index())]; }
  void finish_in(Shard& sh, int64_t now, Event outcome, int64_t execute_ms);
  // per-thread bulkhead (see set_per_thread_bulkhead)
  std::atomic<bool> per_thread_{false};
  // set by the first per-thread admission: from then on a shared-mode admission also counts
  // the calls still holding per-thread slots (a reload that shrinks the pool below
  // kPerThreadMinPool switches modes with calls in flight)
  std::atomic<bool> per_thread_used_{false};
  int64_t per_thread_in_flight() const;
  bool per_thread_mode(int64_t core) const;
  Admit try_start_per_thread(int64_t now, int64_t core);
  void release_in(Shard& sh);
  void mark_success(int64_t now);
  bool is_open(int64_t now);
  bool allow_request(int64_t now);
  HealthCounts health_at(int64_t now);
  void apply_hot(const Settings& s);

  std::string name_, group_, pool_;
  const Clock& clock_;
  std::mutex settings_mu_;  // full Settings (snapshot/settings(); rare)
  Settings s_;
  // Settings read on every call, updated by config reloads.
  std::atomic<bool> circuit_enabled_{true}, force_open_{false}, force_closed_{false};
  std::atomic<int> volume_{20}, error_pct_{50}, sleep_window_ms_{5000}, pool_core_{10}, health_ms_{500},
      sem_max_{10};
  std::atomic<bool> semaphore_{false};  // execution.isolation.strategy=SEMAPHORE
  std::vector<std::unique_ptr<Shard>> shards_;
  // Cache lines: the breaker state and health snapshot are read by every call and written
  // rarely; the bulkhead count is written by every call from every worker. They sit on
  // separate lines so that the count's traffic does not evict the read-mostly state.
  // breaker (HystrixCircuitBreakerImpl)
  alignas(64) std::atomic<bool> open_{false};
  std::atomic<int64_t> opened_or_tested_{0};
  // transitions (for /metrics): opened; closed by the sleep window's trial call, or earlier by
  // a call that was already running when the circuit opened (markSuccess closes on any success)
  std::atomic<uint64_t> opened_n_{0}, closed_trial_n_{0}, closed_inflight_n_{0};
  std::atomic<int64_t> opened_at_{0};  // when it last opened (trials start a sleep window later)
  // health snapshot: (total << 32 | errors), refreshed at most every health_ms_
  std::mutex health_mu_;
  std::atomic<int64_t> health_at_{-1};
  std::atomic<uint64_t> health_packed_{0};
  // bulkhead (thread pool of pool_core_ threads, and a queue when max_queue_ > 0)
  alignas(64) std::atomic<int64_t> active_{0};
  std::atomic<int64_t> largest_{0};
  bool try_acquire_slot();
  void slot_started(int64_t now, int64_t active);
  // maxQueueSize: Hystrix sizes the pool's queue once, when the pool is created at the first
  // execution, so later property changes do not resize it (update_settings() before the
  // first call still does: the start-up configuration arrives after construction)
  alignas(64) std::atomic<int> max_queue_{-1};
  std::atomic<int> queue_threshold_{5};
  std::mutex queue_mu_;
  std::deque<Queued> queue_;
  std::atomic<bool> executed_{false};
};

}  // namespace hola::resilience
