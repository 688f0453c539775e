#include "core/perfcount.h"

#include <linux/perf_event.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <cstring>

namespace hola {

namespace {
int open_counter(uint64_t config, int group) {
  perf_event_attr a;
  memset(&a, 0, sizeof a);
  a.type = PERF_TYPE_HARDWARE;
  a.size = sizeof a;
  a.config = config;
  a.exclude_kernel = 1;
  a.exclude_hv = 1;
  a.read_format = PERF_FORMAT_GROUP | PERF_FORMAT_TOTAL_TIME_ENABLED | PERF_FORMAT_TOTAL_TIME_RUNNING;
  // pid 0, cpu -1: this thread, wherever it runs
  return int(syscall(SYS_perf_event_open, &a, 0, -1, group, PERF_FLAG_FD_CLOEXEC));
}
}  // namespace

ThreadCounters::~ThreadCounters() {
  if (fd_cycles_ >= 0) ::close(fd_cycles_);
  const int fd = fd_.load(std::memory_order_relaxed);
  if (fd >= 0) ::close(fd);
}

bool ThreadCounters::open() {
  if (fd_.load(std::memory_order_relaxed) >= 0) return true;
  const int fd = open_counter(PERF_COUNT_HW_INSTRUCTIONS, -1);
  if (fd < 0) return false;
  fd_cycles_ = open_counter(PERF_COUNT_HW_CPU_CYCLES, fd);
  if (fd_cycles_ < 0) {
    ::close(fd);
    return false;
  }
  fd_.store(fd, std::memory_order_release);
  return true;
}

bool ThreadCounters::read(uint64_t* instructions, uint64_t* cycles) const {
  const int fd = fd_.load(std::memory_order_acquire);
  if (fd < 0) return false;
  // PERF_FORMAT_GROUP: nr, time_enabled, time_running, then one value per member
  uint64_t buf[5] = {};
  if (::read(fd, buf, sizeof buf) != ssize_t(sizeof buf) || buf[0] != 2) return false;
  const uint64_t enabled = buf[1], running = buf[2];
  auto scaled = [&](uint64_t v) {
    return running && running < enabled ? uint64_t(double(v) * double(enabled) / double(running)) : v;
  };
  *instructions = scaled(buf[3]);
  *cycles = scaled(buf[4]);
  return true;
}

}  // namespace hola
