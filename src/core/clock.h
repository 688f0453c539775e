// Clocks. The service never reads time through anything but these helpers so that the
// resilience code (rolling windows, breaker sleep window) can be driven by a fake clock in
// tests — the reference relies on Hystrix's wall-clock timers (config.properties:17,19).
#pragma once
#include <atomic>
#include <cstdint>
#include <ctime>

namespace hola {

// -DHOLA_COUNT_CLOCK_READS (CMake preset `clockcount`): every clock read below is counted,
// process-wide, and /metrics exports the total (hola_clock_reads_total), so a test can state
// how many clock reads a request costs. Off in every other build.
// The coarse clock (no TSC read: a few loads from the vDSO page) is counted apart.
#ifdef HOLA_COUNT_CLOCK_READS
inline std::atomic<uint64_t> g_clock_reads{0}, g_coarse_clock_reads{0};
inline void note_clock_read() { g_clock_reads.fetch_add(1, std::memory_order_relaxed); }
inline void note_coarse_clock_read() { g_coarse_clock_reads.fetch_add(1, std::memory_order_relaxed); }
#else
inline void note_clock_read() {}
inline void note_coarse_clock_read() {}
#endif

inline int64_t mono_ns() {
  note_clock_read();
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return int64_t(ts.tv_sec) * 1000000000 + ts.tv_nsec;
}
inline int64_t mono_ms() { return mono_ns() / 1000000; }
inline int64_t wall_us() {
  note_clock_read();
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return int64_t(ts.tv_sec) * 1000000 + ts.tv_nsec / 1000;
}
inline int64_t wall_ms() { return wall_us() / 1000; }
// Coarse (jiffy-resolution) wall clock seconds: used for the HTTP Date header.
inline int64_t wall_sec_coarse() {
  note_coarse_clock_read();
  timespec ts;
  clock_gettime(CLOCK_REALTIME_COARSE, &ts);
  return ts.tv_sec;
}

// Millisecond clock abstraction for the resilience layer.
class Clock {
 public:
  virtual ~Clock() = default;
  virtual int64_t now_ms() const = 0;
};

class SystemClock final : public Clock {
 public:
  int64_t now_ms() const override { return mono_ms(); }
  static SystemClock& instance() {
    static SystemClock c;
    return c;
  }
};

// The time of the event loop running on this thread, read once per loop pass (EventLoop::run
// publishes it here): millisecond bookkeeping on the request path (Hystrix windows and
// timeouts, Feign timings) costs no clock read per call. Off a loop thread, mono_ms().
inline thread_local const int64_t* t_loop_now_ms = nullptr;
// ... and in nanoseconds: the mono_ns() at which the pass found its events. A duration between
// two passes measured with it (a parked request's latency) is exact to the passes' own
// handling time, with no clock read of its own.
inline thread_local const int64_t* t_loop_now_ns = nullptr;
inline int64_t loop_now_ms() {
  const int64_t* p = t_loop_now_ms;
  return p ? *p : mono_ms();
}
inline int64_t loop_now_ns() {
  const int64_t* p = t_loop_now_ns;
  return p ? *p : mono_ns();
}

class LoopClock final : public Clock {
 public:
  int64_t now_ms() const override { return loop_now_ms(); }
  static LoopClock& instance() {
    static LoopClock c;
    return c;
  }
};

class FakeClock final : public Clock {
 public:
  explicit FakeClock(int64_t start = 1000000) : t_(start) {}
  int64_t now_ms() const override { return t_.load(std::memory_order_relaxed); }
  void advance(int64_t ms) { t_.fetch_add(ms, std::memory_order_relaxed); }
  void set(int64_t ms) { t_.store(ms, std::memory_order_relaxed); }

 private:
  std::atomic<int64_t> t_;
};

// Formats `sec` (Unix time) as an IMF-fixdate, e.g. "Thu, 15 Oct 2026 21:52:00 GMT".
// Writes exactly 29 bytes to out.
void format_http_date(int64_t sec, char out[29]);

}  // namespace hola
