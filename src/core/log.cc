#include "core/log.h"

#include <pthread.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <ctime>

#include "core/clock.h"
#include "core/cpuprof.h"

namespace hola {

namespace {
const char* level_name(LogLevel l) {
  switch (l) {
    case LogLevel::kDebug: return "DEBUG";
    case LogLevel::kInfo: return "INFO";
    case LogLevel::kWarn: return "WARN";
    case LogLevel::kError: return "ERROR";
    default: return "?";
  }
}
}  // namespace

Logger& Logger::instance() {
  static Logger* l = new Logger();  // intentionally leaked: usable during static destruction
  return *l;
}

// A single-producer / single-consumer byte ring of length-prefixed lines. head and tail
// count bytes ever written / consumed; the producer publishes a line by advancing head.
struct Logger::Ring {
  static constexpr size_t kSize = 128 * 1024;  // power of two
  alignas(64) std::atomic<uint64_t> head{0};
  uint64_t seen_tail = 0;  // producer's last look at tail: it re-reads tail only when this looks full
  alignas(64) std::atomic<uint64_t> tail{0};
  std::atomic<bool> orphan{false};  // its thread has exited: free for the next new thread
  char buf[kSize];

  void put(uint64_t pos, const void* p, size_t n) {
    const size_t at = size_t(pos & (kSize - 1)), first = std::min(n, kSize - at);
    memcpy(buf + at, p, first);
    memcpy(buf, static_cast<const char*>(p) + first, n - first);
  }
  void get(uint64_t pos, void* p, size_t n) const {
    const size_t at = size_t(pos & (kSize - 1)), first = std::min(n, kSize - at);
    memcpy(p, buf + at, first);
    memcpy(static_cast<char*>(p) + first, buf, n - first);
  }
};

namespace {
struct ThreadRing {
  Logger::Ring* r = nullptr;
  ~ThreadRing() {
    if (r) r->orphan.store(true, std::memory_order_release);
  }
};
thread_local ThreadRing tls_ring;

// Bounded waits against the system clock: libstdc++ implements steady-clock waits with
// pthread_cond_clockwait, which the toolchain's ThreadSanitizer does not intercept.
constexpr auto kPoll = std::chrono::milliseconds(1);
constexpr int kIdlePolls = 10;  // empty polls in a row before the writer sleeps longer
// The writer's longest sleep, and so the longest a line can wait when no producer wakes it.
constexpr auto kIdleSleep = std::chrono::milliseconds(50);
}  // namespace

Logger::Logger() {
  // The writer may be started before main() blocks its termination signals (`--log-level`
  // touches the logger while the flags are parsed). A process-directed SIGTERM must never be
  // delivered there, where its default action would kill the process: main takes it with
  // sigwait/sigtimedwait. So they are blocked before the thread exists (it inherits the mask:
  // no window after its start), and only they: SIGPROF (--cpu-profile samples the writer too)
  // and the stall reports' capture signal stay deliverable.
  sigset_t term, saved;
  sigemptyset(&term);
  sigaddset(&term, SIGTERM);
  sigaddset(&term, SIGINT);
  sigaddset(&term, SIGHUP);
  pthread_sigmask(SIG_BLOCK, &term, &saved);
  th_ = std::thread([this] { run(); });
  pthread_sigmask(SIG_SETMASK, &saved, nullptr);
  pthread_setname_np(th_.native_handle(), "hola-log");
}

Logger::~Logger() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
}

void Logger::log(LogLevel l, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vlog(l, fmt, ap);
  va_end(ap);
}

void Logger::vlog(LogLevel l, const char* fmt, va_list ap) {
  char msg[2048];
  int n = vsnprintf(msg, sizeof msg, fmt, ap);
  if (n < 0) return;
  if (n >= int(sizeof msg)) n = sizeof msg - 1;
  int64_t us = wall_us();
  time_t sec = us / 1000000;
  tm t;
  gmtime_r(&sec, &t);
  char line[2200];
  int m = snprintf(line, sizeof line, "%04d-%02d-%02dT%02d:%02d:%02d.%03dZ %-5s [%d] %.*s\n",
                   t.tm_year + 1900, t.tm_mon + 1, t.tm_mday, t.tm_hour, t.tm_min, t.tm_sec,
                   int(us / 1000 % 1000), level_name(l), int(getpid()), n, msg);
  enqueue(line, size_t(m < int(sizeof line) ? m : sizeof line - 1));
}

void Logger::raw(const char* fmt, ...) {
  if (level() == LogLevel::kOff) return;
  char line[2048];
  va_list ap;
  va_start(ap, fmt);
  int n = vsnprintf(line, sizeof line - 1, fmt, ap);
  va_end(ap);
  if (n < 0) return;
  if (n > int(sizeof line) - 2) n = int(sizeof line) - 2;
  line[n++] = '\n';
  enqueue(line, size_t(n));
}

void Logger::raw_line(std::string_view line) {
  if (level() == LogLevel::kOff) return;
  enqueue(line.data(), std::min(line.size(), size_t(2047)), true);
}

Logger::Ring* Logger::ring_for_this_thread() {
  if (tls_ring.r) return tls_ring.r;
  std::lock_guard<std::mutex> g(reg_mu_);
  const int n = nrings_.load(std::memory_order_relaxed);
  for (int i = 0; i < n; ++i) {
    Ring* r = rings_[i].load(std::memory_order_relaxed);
    // A ring whose thread has exited is reused once the writer has emptied it.
    if (r->orphan.load(std::memory_order_acquire) &&
        r->head.load(std::memory_order_acquire) == r->tail.load(std::memory_order_acquire)) {
      r->orphan.store(false, std::memory_order_relaxed);
      return tls_ring.r = r;
    }
  }
  if (n == kMaxRings) return nullptr;
  Ring* r = new Ring();
  rings_[n].store(r, std::memory_order_release);
  nrings_.store(n + 1, std::memory_order_release);
  return tls_ring.r = r;
}

void Logger::enqueue(const char* line, size_t n, bool newline) {
  Ring* r = ring_for_this_thread();
  const uint32_t len = uint32_t(n + newline);
  const uint64_t need = sizeof len + len;
  if (!r) {
    dropped_.fetch_add(1, std::memory_order_relaxed);
    return;
  }
  const uint64_t h = r->head.load(std::memory_order_relaxed);
  if (Ring::kSize - (h - r->seen_tail) < need) {
    // only now touch the writer's cache line
    r->seen_tail = r->tail.load(std::memory_order_acquire);
    if (Ring::kSize - (h - r->seen_tail) < need) {
      dropped_.fetch_add(1, std::memory_order_relaxed);
      return;
    }
  }
  r->put(h, &len, sizeof len);
  r->put(h + sizeof len, line, n);
  if (newline) r->put(h + sizeof len + n, "\n", 1);
  // A release store, not a full fence: on x86 a seq_cst store would wait here for every
  // store into the ring (lines the writer last read, so each is a cross-core miss) to
  // complete. The price is that this thread may miss the writer falling asleep; the writer
  // therefore never sleeps longer than kIdleSleep.
  r->head.store(h + need, std::memory_order_release);
  if (sleeping_.load(std::memory_order_relaxed)) wake();
}

void Logger::wake() {
  {
    std::lock_guard<std::mutex> g(mu_);
    sleeping_.store(false, std::memory_order_seq_cst);
  }
  cv_.notify_one();
}

bool Logger::rings_empty() const {
  const int n = nrings_.load(std::memory_order_acquire);
  for (int i = 0; i < n; ++i) {
    const Ring* r = rings_[i].load(std::memory_order_acquire);
    if (r->head.load(std::memory_order_acquire) != r->tail.load(std::memory_order_relaxed)) return false;
  }
  return true;
}

size_t Logger::drain(std::string* out) {
  size_t lines = 0;
  const int n = nrings_.load(std::memory_order_acquire);
  for (int i = 0; i < n; ++i) {
    Ring* r = rings_[i].load(std::memory_order_acquire);
    uint64_t t = r->tail.load(std::memory_order_relaxed);
    const uint64_t h = r->head.load(std::memory_order_acquire);
    if (t == h) continue;
    if (t > h) {  // cannot happen either; resynchronise instead of reporting a non-empty ring forever
      dropped_.fetch_add(1, std::memory_order_relaxed);
      r->tail.store(h, std::memory_order_release);
      continue;
    }
    while (t < h) {
      uint32_t len;
      r->get(t, &len, sizeof len);
      if (len > Ring::kSize || h - t < sizeof len + len || h - t > Ring::kSize) {
        // Cannot happen with one producer per ring. Should it anyway, the rest of the ring
        // is dropped (and counted) rather than read past its head or spun on forever.
        dropped_.fetch_add(1, std::memory_order_relaxed);
        t = h;
        break;
      }
      const size_t old = out->size();
      out->resize(old + len);
      r->get(t + sizeof len, &(*out)[old], len);
      t += sizeof len + len;
      ++lines;
    }
    r->tail.store(t, std::memory_order_release);
  }
  return lines;
}

void Logger::flush() {
  std::unique_lock<std::mutex> g(mu_);
  const uint64_t ticket = ++flush_req_;
  cv_.notify_one();
  flushed_.wait(g, [&] { return flush_done_ >= ticket || stop_; });
}

void Logger::run() {
  std::string out;
  int idle = 0;
  for (;;) {
    cpuprof::register_thread();  // no-op once armed (or when not profiling)
    uint64_t req;
    bool stop;
    {
      std::lock_guard<std::mutex> g(mu_);
      req = flush_req_;
      stop = stop_;
    }
    out.clear();
    const size_t got = drain(&out);
    size_t off = 0;
    while (off < out.size()) {
      ssize_t w = ::write(2, out.data() + off, out.size() - off);
      if (w <= 0) break;
      off += size_t(w);
    }
    std::unique_lock<std::mutex> g(mu_);
    if (flush_done_ < req) {
      flush_done_ = req;  // every line logged before those flush() calls is written
      flushed_.notify_all();
    }
    if (stop && got == 0) break;
    if (stop_ || flush_req_ != flush_done_) continue;
    auto woken = [&] { return stop_ || flush_req_ != flush_done_; };
    if (got) idle = 0;
    if (got || ++idle < kIdlePolls) {
      cv_.wait_until(g, std::chrono::system_clock::now() + kPoll, woken);
      continue;
    }
    // Idle: sleep until a producer sees sleeping_ (best effort, see enqueue) or kIdleSleep
    // passes. idle stays >= kIdlePolls, so an empty look afterwards sleeps long again.
    sleeping_.store(true, std::memory_order_relaxed);
    if (!rings_empty()) {
      sleeping_.store(false, std::memory_order_relaxed);
      continue;
    }
    cv_.wait_until(g, std::chrono::system_clock::now() + kIdleSleep,
                   [&] { return !sleeping_.load(std::memory_order_relaxed) || woken(); });
    sleeping_.store(false, std::memory_order_relaxed);
  }
  std::lock_guard<std::mutex> g(mu_);
  flush_done_ = flush_req_;
  flushed_.notify_all();
}

bool parse_log_level(const std::string& s, LogLevel* out) {
  if (s == "debug") *out = LogLevel::kDebug;
  else if (s == "info") *out = LogLevel::kInfo;
  else if (s == "warn") *out = LogLevel::kWarn;
  else if (s == "error") *out = LogLevel::kError;
  else if (s == "off") *out = LogLevel::kOff;
  else return false;
  return true;
}

}  // namespace hola
