#include "core/cpuprof.h"

#include <errno.h>
#include <pthread.h>
#include <signal.h>
#include <sys/syscall.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

namespace hola::cpuprof {

namespace {
constexpr int kDepth = 10;
constexpr size_t kCapacity = 1 << 19;  // samples; the pages are touched only as they fill

struct Sample {
  uint16_t thread;  // index into g_names
  uint8_t depth;
  uintptr_t pc[kDepth];
};

std::string g_path;
long g_period_ns = 0;
std::unique_ptr<Sample[]> g_samples;
std::atomic<size_t> g_next{0};
std::atomic<bool> g_on{false};
std::mutex g_mu;                  // g_names, g_timers
std::vector<std::string> g_names;  // one per registered thread
std::vector<timer_t> g_timers;

thread_local int t_index = -1;
thread_local timer_t t_timer;
thread_local bool t_armed = false;
// The sampled thread's stack, for bounds-checking the frame-pointer walk.
thread_local uintptr_t t_stack_lo = 0, t_stack_hi = 0;

// Executable mappings at start(): a return address must fall in one of them. Read-only while
// sampling (the handler takes no lock and calls nothing).
constexpr int kMaxRanges = 512;
uintptr_t g_exec_lo[kMaxRanges], g_exec_hi[kMaxRanges];
int g_nexec = 0;

int exec_range(uintptr_t pc) {
  for (int i = 0; i < g_nexec; ++i)
    if (pc >= g_exec_lo[i] && pc < g_exec_hi[i]) return i;
  return -1;
}
bool executable(uintptr_t pc) { return exec_range(pc) >= 0; }
int g_own_range = -1;  // the mapping holding this file's code (built with frame pointers)

void load_exec_ranges() {
  std::ifstream maps("/proc/self/maps");
  g_nexec = 0;
  for (std::string line; std::getline(maps, line) && g_nexec < kMaxRanges;) {
    unsigned long lo = 0, hi = 0;
    char perms[5] = {};
    if (sscanf(line.c_str(), "%lx-%lx %4s", &lo, &hi, perms) == 3 && perms[2] == 'x') {
      g_exec_lo[g_nexec] = lo;
      g_exec_hi[g_nexec] = hi;
      ++g_nexec;
    }
  }
}

// Async-signal-safe: walks the interrupted thread's frame-pointer chain from the ucontext's
// RBP (the native code is built with -fno-omit-frame-pointer), reading only inside the
// thread's own stack and stopping at the first address that is not code. No unwinder, no
// locks, no allocation. When the sample lands in code from another object (libc's syscall
// wrappers: send, recv, epoll_wait), which keeps no frame pointer, the caller is found by
// scanning the top of the stack for the first return address into a different mapping.
void on_prof(int, siginfo_t*, void* ucv) {
  if (!g_on.load(std::memory_order_relaxed) || t_index < 0) return;
  const size_t i = g_next.fetch_add(1, std::memory_order_relaxed);
  if (i >= kCapacity) return;
  const int saved_errno = errno;
  Sample& s = g_samples[i];
  s.thread = uint16_t(t_index);
  const auto* uc = static_cast<const ucontext_t*>(ucv);
  const uintptr_t pc = uintptr_t(uc->uc_mcontext.gregs[REG_RIP]);
  const uintptr_t sp = uintptr_t(uc->uc_mcontext.gregs[REG_RSP]);
  uintptr_t fp = uintptr_t(uc->uc_mcontext.gregs[REG_RBP]);
  s.pc[0] = pc;
  s.depth = 1;
  const bool bounded = t_stack_hi > t_stack_lo;
  auto in_stack = [&](uintptr_t a) { return bounded && a >= t_stack_lo && a + 16 <= t_stack_hi && !(a & 7); };
  const int pc_range = exec_range(pc);
  uintptr_t caller = 0;
  if (pc_range != g_own_range) {
    for (int k = 0; k < 16 && in_stack(sp + 8 * uintptr_t(k)); ++k) {
      const uintptr_t w = *reinterpret_cast<const uintptr_t*>(sp + 8 * uintptr_t(k));
      const int r = exec_range(w);
      if (r >= 0 && r != pc_range) {
        caller = w;
        s.pc[s.depth++] = w;
        break;
      }
    }
  }
  bool first = true;
  while (s.depth < kDepth && in_stack(fp)) {
    const uintptr_t ret = *reinterpret_cast<const uintptr_t*>(fp + 8);
    const uintptr_t next = *reinterpret_cast<const uintptr_t*>(fp);
    if (!executable(ret)) break;
    if (!(first && ret == caller)) s.pc[s.depth++] = ret;
    first = false;
    if (next <= fp) break;  // the chain must climb the stack
    fp = next;
  }
  errno = saved_errno;
}

void note_stack_bounds() {
  pthread_attr_t attr;
  if (pthread_getattr_np(pthread_self(), &attr) != 0) return;
  void* addr = nullptr;
  size_t size = 0;
  if (pthread_attr_getstack(&attr, &addr, &size) == 0) {
    t_stack_lo = uintptr_t(addr);
    t_stack_hi = uintptr_t(addr) + size;
  }
  pthread_attr_destroy(&attr);
}
}  // namespace

bool start(const std::string& path, int hz) {
  if (g_on.load() || hz <= 0) return false;
  g_path = path;
  g_period_ns = 1000000000L / hz;
  g_samples.reset(new Sample[kCapacity]);
  load_exec_ranges();
  g_own_range = exec_range(uintptr_t(&on_prof));
  struct sigaction sa {};
  sa.sa_sigaction = on_prof;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  if (sigaction(SIGPROF, &sa, nullptr) != 0) return false;
  g_on.store(true);
  return true;
}

void register_thread() {
  if (!g_on.load() || t_armed) return;
  char name[32] = "?";
  pthread_getname_np(pthread_self(), name, sizeof name);
  sigevent sev{};
  sev.sigev_notify = SIGEV_THREAD_ID;
  sev.sigev_signo = SIGPROF;
  sev._sigev_un._tid = pid_t(syscall(SYS_gettid));
  note_stack_bounds();
  if (timer_create(CLOCK_THREAD_CPUTIME_ID, &sev, &t_timer) != 0) return;
  {
    std::lock_guard<std::mutex> g(g_mu);
    t_index = int(g_names.size());
    g_names.push_back(name);
    g_timers.push_back(t_timer);
  }
  itimerspec its{};
  its.it_interval.tv_nsec = its.it_value.tv_nsec = g_period_ns % 1000000000L;
  its.it_interval.tv_sec = its.it_value.tv_sec = g_period_ns / 1000000000L;
  timer_settime(t_timer, 0, &its, nullptr);
  t_armed = true;
}

void unregister_thread() {
  if (!t_armed) return;
  itimerspec off{};
  timer_settime(t_timer, 0, &off, nullptr);
  t_armed = false;
}

bool write() {
  if (!g_on.exchange(false)) return false;
  {
    std::lock_guard<std::mutex> g(g_mu);
    itimerspec off{};
    for (timer_t t : g_timers) timer_settime(t, 0, &off, nullptr);
  }
  const size_t n = std::min(g_next.load(), kCapacity);
  // identical (thread, stack) samples are written once with their count
  std::map<std::pair<int, std::vector<uintptr_t>>, uint64_t> stacks;
  for (size_t i = 0; i < n; ++i) {
    const Sample& s = g_samples[i];
    stacks[{s.thread, std::vector<uintptr_t>(s.pc, s.pc + s.depth)}]++;
  }
  std::ofstream f(g_path);
  if (!f) return false;
  f << "# hola cpu profile\nperiod_ns " << g_period_ns << "\nsamples " << n << "\ndropped "
    << (g_next.load() > kCapacity ? g_next.load() - kCapacity : 0) << "\n";
  {
    std::lock_guard<std::mutex> g(g_mu);
    for (size_t i = 0; i < g_names.size(); ++i) f << "thread " << i << " " << g_names[i] << "\n";
  }
  // executable mappings, to turn addresses into (object, offset)
  std::ifstream maps("/proc/self/maps");
  for (std::string line; std::getline(maps, line);) {
    const size_t sp = line.find(' ');
    if (sp != std::string::npos && line.size() > sp + 3 && line[sp + 3] == 'x') f << "map " << line << "\n";
  }
  char buf[32];
  for (const auto& [key, count] : stacks) {
    f << "stack " << count << " " << key.first;
    for (uintptr_t pc : key.second) {
      snprintf(buf, sizeof buf, " %lx", (unsigned long)pc);
      f << buf;
    }
    f << "\n";
  }
  return bool(f);
}

}  // namespace hola::cpuprof
