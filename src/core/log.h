// Asynchronous console logger. Request threads only enqueue; one background
// thread writes to stderr. The reference instead println()s the config path on every request
// (Configuration.java:28), serialising all workers on the stdout lock; here log lines happen
// only on events (config change, outbound call with Feign BASIC logging, errors).
//
// Each logging thread owns a single-producer byte ring, so a log line costs its formatting
// and a copy: no lock, no allocation and no wake-up syscall while the writer thread is
// polling. Feign BASIC logging (the default, HolaResource.java:109) writes two lines per aloha
// call from every worker at once, which a shared queue behind one mutex turned into the
// chaining path's bottleneck. The writer polls the rings every millisecond while lines are
// coming and sleeps on a condition variable when they stop; a producer wakes it only then.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdarg>
#include <cstdint>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>

namespace hola {

enum class LogLevel : int { kDebug = 0, kInfo = 1, kWarn = 2, kError = 3, kOff = 4 };

class Logger {
 public:
  static Logger& instance();
  void set_level(LogLevel l) { level_.store(int(l), std::memory_order_relaxed); }
  LogLevel level() const { return LogLevel(level_.load(std::memory_order_relaxed)); }
  bool enabled(LogLevel l) const { return int(l) >= level_.load(std::memory_order_relaxed); }
  void log(LogLevel l, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
  void vlog(LogLevel l, const char* fmt, va_list ap);
  // One line exactly as formatted (a newline is appended), without the timestamp/level
  // prefix: for output whose format belongs to the reference's libraries, e.g. Feign's
  // Logger.ErrorLogger, which System.err.printf()s its lines (HolaResource.java:109).
  // Suppressed only when the level is off.
  void raw(const char* fmt, ...) __attribute__((format(printf, 2, 3)));
  // raw() for a line that is already built (no printf); a newline is appended.
  void raw_line(std::string_view line);
  // Blocks until every line logged before the call (by any thread) has been written.
  void flush();
  // Lines dropped because their thread's ring was full (the writer fell behind).
  uint64_t dropped() const { return dropped_.load(std::memory_order_relaxed); }
  ~Logger();

  struct Ring;  // one per logging thread (log.cc)

 private:
  Logger();
  void run();
  void enqueue(const char* line, size_t n, bool newline = false);  // newline: append '\n'
  Ring* ring_for_this_thread();
  size_t drain(std::string* out);  // appends every ring's lines; returns how many
  bool rings_empty() const;
  void wake();

  static constexpr int kMaxRings = 1024;
  std::atomic<int> level_{int(LogLevel::kInfo)};
  std::atomic<Ring*> rings_[kMaxRings] = {};
  std::atomic<int> nrings_{0};
  std::mutex reg_mu_;  // ring registration only
  std::mutex mu_;      // writer sleep / flush hand-shake
  std::condition_variable cv_, flushed_;
  std::atomic<bool> sleeping_{false};
  bool stop_ = false;
  uint64_t flush_req_ = 0, flush_done_ = 0;
  std::atomic<uint64_t> dropped_{0};
  std::thread th_;
};

bool parse_log_level(const std::string& s, LogLevel* out);

}  // namespace hola

#define HOLA_LOG(lvl, ...)                                                 \
  do {                                                                     \
    if (::hola::Logger::instance().enabled(lvl))                           \
      ::hola::Logger::instance().log(lvl, __VA_ARGS__);                    \
  } while (0)
#define LOG_DEBUG(...) HOLA_LOG(::hola::LogLevel::kDebug, __VA_ARGS__)
#define LOG_INFO(...) HOLA_LOG(::hola::LogLevel::kInfo, __VA_ARGS__)
#define LOG_WARN(...) HOLA_LOG(::hola::LogLevel::kWarn, __VA_ARGS__)
#define LOG_ERROR(...) HOLA_LOG(::hola::LogLevel::kError, __VA_ARGS__)
