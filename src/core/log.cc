#include "core/log.h"

#include <unistd.h>

#include <cstdio>
#include <ctime>

#include "core/clock.h"

namespace hola {

namespace {
constexpr size_t kMaxQueued = 65536;  // beyond this, lines are dropped and counted
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

Logger::Logger() : th_([this] { run(); }) {}

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

void Logger::enqueue(const char* line, size_t n) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (q_.size() >= kMaxQueued) {
      dropped_.fetch_add(1, std::memory_order_relaxed);
      return;
    }
    q_.emplace_back(line, n);
    ++enqueued_;
  }
  cv_.notify_one();
}

void Logger::flush() {
  std::unique_lock<std::mutex> g(mu_);
  uint64_t target = enqueued_;
  flushed_.wait(g, [&] { return written_ >= target || stop_; });
}

void Logger::run() {
  std::deque<std::string> batch;
  for (;;) {
    {
      std::unique_lock<std::mutex> g(mu_);
      cv_.wait(g, [&] { return stop_ || !q_.empty(); });
      if (q_.empty() && stop_) break;
      batch.swap(q_);
    }
    std::string out;
    for (auto& s : batch) out += s;
    size_t off = 0;
    while (off < out.size()) {
      ssize_t w = ::write(2, out.data() + off, out.size() - off);
      if (w <= 0) break;
      off += size_t(w);
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      written_ += batch.size();
    }
    batch.clear();
    flushed_.notify_all();
  }
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
