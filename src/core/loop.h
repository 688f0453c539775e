// Single-threaded epoll event loop with a timer heap and a cross-thread task queue.
//
// This replaces Undertow's IO-thread + worker-thread-pool pair (SURVEY.md T1, §2d "request
// concurrency"): each loop is pinned to one host core and owns its connections outright, so
// the hot path has no locks, no thread hand-off and no per-request allocation. Timers drive
// the outbound 600 ms timeout (config.properties:17) instead of Hystrix's timer thread.
#pragma once
#include <sys/epoll.h>

#include <atomic>
#include <cstdint>
#include <functional>
#include <mutex>
#include <queue>
#include <unordered_map>
#include <vector>

namespace hola {

class EventLoop {
 public:
  struct Handler {
    virtual ~Handler() = default;
    virtual void on_event(uint32_t events) = 0;
  };
  using TimerId = uint64_t;

  EventLoop();
  ~EventLoop();
  EventLoop(const EventLoop&) = delete;
  EventLoop& operator=(const EventLoop&) = delete;

  bool add(int fd, uint32_t events, Handler* h);
  bool mod(int fd, uint32_t events, Handler* h);
  void del(int fd);

  // One-shot timer; callback runs on the loop thread. Returns an id usable with cancel_timer.
  TimerId add_timer(int64_t delay_ms, std::function<void()> cb);
  void cancel_timer(TimerId id);
  // Timers armed and not yet fired or cancelled; readable from any thread (a leak detector:
  // the /metrics gauge hola_event_loop_timers).
  size_t pending_timers() const { return pending_.load(std::memory_order_relaxed); }

  // Thread-safe: run fn on the loop thread soon.
  void post(std::function<void()> fn);
  // Handlers whose lifetime ends inside an event batch are deleted after the batch.
  void retire(Handler* h) { retired_.push_back(h); }
  // Loop thread only: run fn once the current batch of events and timers has been handled
  // (before the loop polls again), e.g. to send what a batch queued in one write.
  void defer(std::function<void()> fn) { deferred_.push_back(std::move(fn)); }

  void run();
  void stop();  // thread-safe
  bool stopping() const { return stop_.load(std::memory_order_relaxed); }

  // Millisecond monotonic time cached at the top of each iteration.
  int64_t now_ms() const { return now_ms_; }
  // Called once per iteration, after the wait and before the pass's events are handled
  // (e.g. refresh the cached Date header as of the pass's time).
  void set_tick(std::function<void()> fn) { tick_ = std::move(fn); }
  // Optional callback when the loop exits run().
  void set_on_exit(std::function<void()> fn) { on_exit_ = std::move(fn); }
  // Before blocking in epoll_wait, poll without sleeping for up to `us` microseconds
  // (trades idle CPU for fewer sleep/wake-up cycles under closed-loop load). 0 = off.
  void set_busy_poll_us(int us) { busy_poll_ns_ = int64_t(us) * 1000; }
  // While busy-polling, execute this many PAUSE instructions after each empty poll, so a
  // spinning thread leaves issue slots to its SMT sibling. 0 = poll back to back.
  void set_busy_poll_pause(int n) { busy_poll_pause_ = n; }
  // Adaptive busy-polling: the spin stays on while it mostly finds work before its budget
  // runs out (a saturated loop, where it saves the sleep/wake-up per request), and is
  // switched off for a growing interval (50 ms .. 1.6 s) while it mostly waits in vain (light
  // load, where it would only burn CPU). Each interval ends with a short re-probe. While it is
  // off, the blocking waits tell whether a spin would have found work (the next event came
  // within twice the spin budget): when 90 % of the last 64 would have, spinning resumes at
  // once instead of at the interval's end. Without that, a saturated loop that was pushed off
  // (a stall elsewhere drains the pipeline for a moment) serves every request through a sleep
  // and a wake-up, which slows its peers, whose spins then miss too: a second, slower steady
  // state (profiles/round5/02_chain_modes).
  void set_busy_poll_auto(bool on) { busy_auto_ = on; }
  // Adaptive spin statistics (loop thread; tests and metrics): spins that found work, spins
  // that ran out, how many times spinning was switched off, and for how many milliseconds
  // in total (the back-off intervals as scheduled).
  uint64_t spin_hits() const { return spin_hits_total_.load(std::memory_order_relaxed); }
  uint64_t spin_misses() const { return spin_misses_total_.load(std::memory_order_relaxed); }
  uint64_t spin_offs() const { return spin_offs_.load(std::memory_order_relaxed); }
  uint64_t spin_off_ms() const { return spin_off_ms_.load(std::memory_order_relaxed); }
  uint64_t spin_resumes() const { return spin_resumes_.load(std::memory_order_relaxed); }
  // Where a loop's time goes (loop thread writes, any thread reads; every mode, not only
  // adaptive): nanoseconds of polls that came back empty while spinning (CPU that did no
  // work: process CPU minus this is the loop's busy CPU), and epoll waits that could block.
  uint64_t idle_spin_ns() const { return idle_spin_ns_.load(std::memory_order_relaxed); }
  uint64_t blocking_waits() const { return blocking_waits_.load(std::memory_order_relaxed); }
  // Gaps between polls: from the end of one pass's poll to the next poll (the pass's own
  // handlers, and any time the thread was descheduled then), and between two empty polls of a
  // spin (descheduled while spinning). Counted when longer than 100 us / 1 ms / 10 ms, and the
  // longest since start: a latency outlier on this loop's connections that matches none of
  // these was not made here (a tail attribution).
  static constexpr int kGapBuckets = 3;
  static constexpr int64_t kGapNs[kGapBuckets] = {100000, 1000000, 10000000};
  uint64_t gaps_over(int i) const { return gaps_over_[i].load(std::memory_order_relaxed); }
  uint64_t gap_max_ns() const { return gap_max_ns_.load(std::memory_order_relaxed); }

  // What the loop thread is doing, published with relaxed stores as it goes, so another
  // thread can say where a loop that stopped answering is: Server::shutdown logs it for a
  // worker that misses the drain deadline, the exit watchdog for every worker. `passes` counts
  // loop iterations (a loop stuck inside one handler shows a count that stops); `subject` and
  // `state` are set by the handler being run (a connection: its id and state bits, see
  // http::Connection::on_event), `pass_ns` is the mono_ns() at which the current pass began.
  enum Phase : uint32_t { kStarting = 0, kWait, kEvents, kTimers, kDeferred, kPosted, kTick, kExited };
  struct Activity {
    std::atomic<uint64_t> passes{0};
    std::atomic<uint32_t> phase{kStarting};
    std::atomic<uint32_t> handler_kind{0};  // handler-defined tag of the running handler
    std::atomic<uint64_t> subject{0};
    std::atomic<uint64_t> state{0};
    std::atomic<int64_t> pass_ns{0};
  };
  static const char* phase_name(uint32_t p);
  const Activity& activity() const { return act_; }
  // Loop thread: the handler now running and its state (cheap: three relaxed stores).
  void note(uint32_t kind, uint64_t subject, uint64_t state) {
    act_.handler_kind.store(kind, std::memory_order_relaxed);
    act_.subject.store(subject, std::memory_order_relaxed);
    act_.state.store(state, std::memory_order_relaxed);
  }
  void note_state(uint64_t state) { act_.state.store(state, std::memory_order_relaxed); }

 private:
  void set_phase(Phase p) { act_.phase.store(p, std::memory_order_relaxed); }
  struct WakeHandler : Handler {
    EventLoop* loop;
    void on_event(uint32_t) override;
  };
  struct TimerEntry {
    int64_t deadline;
    TimerId id;
    bool operator>(const TimerEntry& o) const {
      return deadline != o.deadline ? deadline > o.deadline : id > o.id;
    }
  };
  void run_timers();
  void drain_posted();
  int next_timeout_ms(int64_t now_ns);

  int epfd_ = -1;
  int wakefd_ = -1;
  WakeHandler wake_;
  std::atomic<bool> stop_{false};
  int64_t now_ms_ = 0;
  int64_t now_ns_ = 0;  // the pass's mono_ns() (t_loop_now_ns)
  std::priority_queue<TimerEntry, std::vector<TimerEntry>, std::greater<TimerEntry>> heap_;
  std::unordered_map<TimerId, std::function<void()>> timers_;
  std::atomic<size_t> pending_{0};  // timers_.size(), published for other threads
  TimerId next_timer_ = 1;
  std::mutex post_mu_;
  std::vector<std::function<void()>> posted_;
  std::vector<Handler*> retired_;
  std::vector<std::function<void()>> deferred_, deferred_run_;
  std::function<void()> tick_, on_exit_;
  int64_t busy_poll_ns_ = 0;
  int busy_poll_pause_ = 0;
  bool busy_auto_ = false;
  uint32_t spin_hits_ = 0, spin_misses_ = 0;  // current measurement window
  int64_t spin_off_until_ms_ = 0, spin_backoff_ms_ = 0;
  std::atomic<uint64_t> spin_hits_total_{0}, spin_misses_total_{0}, spin_offs_{0}, spin_off_ms_{0}, spin_resumes_{0};
  uint32_t off_hits_ = 0, off_waits_ = 0;  // blocking waits while spinning is off (current window)
  void note_spin(bool hit);
  void note_off_wait(bool would_hit);
  void note_gap(int64_t ns);
  int64_t pass_end_ns_ = 0;  // mono_ns() when the last pass's polling ended
  // single writer (the loop thread): load + store, no locked read-modify-write
  std::atomic<uint64_t> idle_spin_ns_{0}, blocking_waits_{0}, gap_max_ns_{0};
  std::atomic<uint64_t> gaps_over_[kGapBuckets] = {};
  alignas(64) Activity act_;  // own cache line: written by the loop thread only
};

}  // namespace hola
