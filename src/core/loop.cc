#include "core/loop.h"

#include <errno.h>
#include <sys/eventfd.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "core/clock.h"

namespace hola {

EventLoop::EventLoop() {
  epfd_ = epoll_create1(EPOLL_CLOEXEC);
  wakefd_ = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
  if (epfd_ < 0 || wakefd_ < 0) {
    perror("event loop init");
    abort();
  }
  wake_.loop = this;
  add(wakefd_, EPOLLIN, &wake_);
  now_ms_ = mono_ms();
}

EventLoop::~EventLoop() {
  // Callbacks that never ran may own references that hand handlers back to this loop when
  // destroyed (a ConnRef releasing its connection retires it): drop them first, then free
  // every retired handler.
  {
    auto timers = std::move(timers_);
    timers.clear();
    deferred_.clear();
    deferred_run_.clear();
    std::vector<std::function<void()>> posted;
    {
      std::lock_guard<std::mutex> g(post_mu_);
      posted.swap(posted_);
    }
  }
  for (Handler* h : retired_) delete h;
  if (wakefd_ >= 0) ::close(wakefd_);
  if (epfd_ >= 0) ::close(epfd_);
}

bool EventLoop::add(int fd, uint32_t events, Handler* h) {
  epoll_event ev{};
  ev.events = events;
  ev.data.ptr = h;
  return epoll_ctl(epfd_, EPOLL_CTL_ADD, fd, &ev) == 0;
}

bool EventLoop::mod(int fd, uint32_t events, Handler* h) {
  epoll_event ev{};
  ev.events = events;
  ev.data.ptr = h;
  return epoll_ctl(epfd_, EPOLL_CTL_MOD, fd, &ev) == 0;
}

void EventLoop::del(int fd) { epoll_ctl(epfd_, EPOLL_CTL_DEL, fd, nullptr); }

EventLoop::TimerId EventLoop::add_timer(int64_t delay_ms, std::function<void()> cb) {
  TimerId id = next_timer_++;
  heap_.push({mono_ms() + (delay_ms < 0 ? 0 : delay_ms), id});
  timers_.emplace(id, std::move(cb));
  pending_.store(timers_.size(), std::memory_order_relaxed);
  return id;
}

void EventLoop::cancel_timer(TimerId id) {
  timers_.erase(id);
  pending_.store(timers_.size(), std::memory_order_relaxed);
}

void EventLoop::post(std::function<void()> fn) {
  {
    std::lock_guard<std::mutex> g(post_mu_);
    posted_.push_back(std::move(fn));
  }
  uint64_t one = 1;
  ssize_t r = ::write(wakefd_, &one, sizeof one);
  (void)r;
}

void EventLoop::stop() {
  stop_.store(true, std::memory_order_relaxed);
  uint64_t one = 1;
  ssize_t r = ::write(wakefd_, &one, sizeof one);
  (void)r;
}

const char* EventLoop::phase_name(uint32_t p) {
  static const char* const names[] = {"starting", "wait", "events", "timers", "deferred", "posted", "tick", "exited"};
  return p < sizeof names / sizeof names[0] ? names[p] : "?";
}

void EventLoop::WakeHandler::on_event(uint32_t) {
  uint64_t v;
  while (::read(loop->wakefd_, &v, sizeof v) > 0) {
  }
  loop->set_phase(kPosted);
  loop->drain_posted();
  loop->set_phase(kEvents);
}

void EventLoop::drain_posted() {
  std::vector<std::function<void()>> fns;
  {
    std::lock_guard<std::mutex> g(post_mu_);
    fns.swap(posted_);
  }
  for (auto& f : fns) f();
}

void EventLoop::run_timers() {
  while (!heap_.empty() && heap_.top().deadline <= now_ms_) {
    TimerId id = heap_.top().id;
    heap_.pop();
    auto it = timers_.find(id);
    if (it == timers_.end()) continue;  // cancelled
    auto cb = std::move(it->second);
    timers_.erase(it);
    pending_.store(timers_.size(), std::memory_order_relaxed);
    note(0, id, 0);
    cb();
  }
}

int EventLoop::next_timeout_ms(int64_t now_ns) {
  // About to block: drop cancelled entries at the top first, so that a cancelled timer cannot
  // wake the loop at its old deadline (passes that find work skip this lookup; see run()).
  while (!heap_.empty() && !timers_.count(heap_.top().id)) heap_.pop();
  if (heap_.empty()) return -1;
  int64_t d = heap_.top().deadline - now_ns / 1000000;
  if (d <= 0) return 0;
  return d > 1000000 ? 1000000 : int(d);
}

namespace {
constexpr uint32_t kSpinWindow = 64;        // spins per decision
constexpr uint32_t kSpinHitPercent = 75;    // keep spinning while >= this share finds work
constexpr int64_t kSpinBackoffMinMs = 50, kSpinBackoffMaxMs = 1600;
// While backed off: resume when this share of the window's blocking waits ended within twice
// the spin budget (wake-up latency included). Stricter than the spin's own 75 %, so a loop
// whose events come 20..40 us apart does not flip between the two states.
constexpr uint32_t kResumeHitPercent = 90;
}  // namespace

void EventLoop::note_spin(bool hit) {
  if (hit) ++spin_hits_;
  else ++spin_misses_;
  if (spin_hits_ + spin_misses_ < kSpinWindow) return;
  spin_hits_total_.fetch_add(spin_hits_, std::memory_order_relaxed);
  spin_misses_total_.fetch_add(spin_misses_, std::memory_order_relaxed);
  if (spin_hits_ * 100 < kSpinHitPercent * (spin_hits_ + spin_misses_)) {
    // mostly waiting in vain: stop spinning for a while, longer each time it repeats
    spin_backoff_ms_ = spin_backoff_ms_ ? std::min(kSpinBackoffMaxMs, spin_backoff_ms_ * 2) : kSpinBackoffMinMs;
    spin_off_until_ms_ = now_ms_ + spin_backoff_ms_;
    spin_offs_.fetch_add(1, std::memory_order_relaxed);
    spin_off_ms_.fetch_add(uint64_t(spin_backoff_ms_), std::memory_order_relaxed);
    off_hits_ = off_waits_ = 0;
  } else {
    spin_backoff_ms_ = 0;
  }
  spin_hits_ = spin_misses_ = 0;
}

void EventLoop::note_off_wait(bool would_hit) {
  off_hits_ += would_hit;
  if (++off_waits_ < kSpinWindow) return;
  if (off_hits_ * 100 >= kResumeHitPercent * off_waits_) {
    // events keep arriving within the spin budget: the loop is busy, spin again now (and count
    // only the part of the interval that was spent off)
    if (spin_off_until_ms_ > now_ms_) spin_off_ms_.fetch_sub(uint64_t(spin_off_until_ms_ - now_ms_), std::memory_order_relaxed);
    spin_off_until_ms_ = 0;
    spin_backoff_ms_ = 0;
    spin_resumes_.fetch_add(1, std::memory_order_relaxed);
  }
  off_hits_ = off_waits_ = 0;
}

void EventLoop::note_gap(int64_t ns) {
  if (ns <= kGapNs[0]) return;
  for (int i = 0; i < kGapBuckets; ++i)
    if (ns > kGapNs[i]) gaps_over_[i].store(gaps_over_[i].load(std::memory_order_relaxed) + 1, std::memory_order_relaxed);
  if (uint64_t(ns) > gap_max_ns_.load(std::memory_order_relaxed)) gap_max_ns_.store(uint64_t(ns), std::memory_order_relaxed);
}

void EventLoop::run() {
  constexpr int kMaxEvents = 256;
  epoll_event evs[kMaxEvents];
  t_loop_now_ms = &now_ms_;  // LoopClock on this thread reads the pass's time
  t_loop_now_ns = &now_ns_;
  pass_end_ns_ = now_ns_ = mono_ns();
  uint64_t passes = 0;
  while (!stop_.load(std::memory_order_relaxed)) {
    act_.passes.store(++passes, std::memory_order_relaxed);
    set_phase(kWait);
    int n = 0;
    int wait_errno = 0;  // errno of a failed epoll_wait, taken before the clock reads below
    int64_t t = 0;  // mono_ns() at (or just before) the moment events were found
    bool polled = false;  // a spin ran: the gap to the last pass is taken
    if (busy_poll_ns_ > 0 && (!busy_auto_ || now_ms_ >= spin_off_until_ms_)) {
      t = mono_ns();
      note_gap(t - pass_end_ns_);
      polled = true;
      const int64_t spin0 = t, until = t + busy_poll_ns_;
      bool spun = false;  // the first poll came back empty: this pass is a real spin
      for (;;) {
        n = epoll_wait(epfd_, evs, kMaxEvents, 0);
        if (n < 0) wait_errno = errno;
        if (n != 0 || stop_.load(std::memory_order_relaxed)) break;
        spun = true;
        const int64_t prev = t;
        t = mono_ns();
        if (t - prev > kGapNs[0]) note_gap(t - prev);  // descheduled while spinning
        if (t >= until) break;
        for (int i = 0; i < busy_poll_pause_; ++i) __builtin_ia32_pause();
      }
      // CPU time of the polls that found nothing (up to the end of the last empty one): the
      // part of a spinning loop's CPU that did no work (the /metrics busy-CPU figure)
      if (spun) idle_spin_ns_.store(idle_spin_ns_.load(std::memory_order_relaxed) + uint64_t(t - spin0),
                                    std::memory_order_relaxed);
      if (busy_auto_ && spun) note_spin(n > 0);
    }
    if (n == 0) {
      // backed off from spinning: time the blocking wait (would a spin have found this event?)
      const bool off = busy_auto_ && busy_poll_ns_ > 0 && now_ms_ < spin_off_until_ms_;
      const int64_t w0 = polled ? t : mono_ns();
      if (!polled) note_gap(w0 - pass_end_ns_);
      const int timeout = next_timeout_ms(w0);  // w0: read just now (no clock read of its own)
      n = epoll_wait(epfd_, evs, kMaxEvents, timeout);
      if (n < 0) wait_errno = errno;
      t = mono_ns();
      if (timeout != 0) blocking_waits_.store(blocking_waits_.load(std::memory_order_relaxed) + 1,
                                              std::memory_order_relaxed);
      if (off && n > 0) note_off_wait(t - w0 <= 2 * busy_poll_ns_);
    }
    if (n < 0 && wait_errno != EINTR) {
      // Only a broken epoll descriptor gets here (EBADF, EINVAL, EFAULT). The loop cannot serve
      // its connections or answer posted tasks any more; leaving the thread would leave a
      // replica that looks alive with a dead worker and a drain that waits for it. Fail fast
      // (the supervisor or kubelet restarts the process), saying why, straight to stderr.
      char line[128];
      const int k = snprintf(line, sizeof line, "hola: event loop: epoll_wait(%d) failed: %s; aborting\n", epfd_,
                             strerror(wait_errno));
      ssize_t w = ::write(2, line, size_t(k));
      (void)w;
      std::abort();
    }
    now_ms_ = t / 1000000;
    now_ns_ = t;
    act_.pass_ns.store(t, std::memory_order_relaxed);
    if (tick_) {  // after the wait: the pass's handlers see state as of its own time
      set_phase(kTick);
      tick_();
    }
    if (n > 0) {
      set_phase(kEvents);
      for (int i = 0; i < n; ++i) static_cast<Handler*>(evs[i].data.ptr)->on_event(evs[i].events);
    }
    if (!heap_.empty() && heap_.top().deadline <= now_ms_) {  // a heap peek per pass, no lookup
      set_phase(kTimers);
      run_timers();
    }
    if (!deferred_.empty()) {
      set_phase(kDeferred);
      uint64_t rounds = 0;
      while (!deferred_.empty()) {
        note(0, ++rounds, deferred_.size());
        deferred_run_.swap(deferred_);
        for (auto& f : deferred_run_) f();
        deferred_run_.clear();
      }
    }
    if (!retired_.empty()) {
      for (Handler* h : retired_) delete h;
      retired_.clear();
    }
    pass_end_ns_ = t;  // the next pass's first poll measures its gap from here
  }
  t_loop_now_ms = nullptr;
  t_loop_now_ns = nullptr;
  set_phase(kPosted);
  drain_posted();
  if (on_exit_) on_exit_();
  set_phase(kExited);
}

}  // namespace hola
