#include "core/cpuprof.h"

#include <errno.h>
#include <pthread.h>
#include <signal.h>
#include <sys/syscall.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>
#include <unwind.h>

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

struct Walk {
  uintptr_t* out;
  int n;
};

_Unwind_Reason_Code walk_frame(_Unwind_Context* ctx, void* arg) {
  auto* w = static_cast<Walk*>(arg);
  const uintptr_t ip = _Unwind_GetIP(ctx);
  if (!ip || w->n >= 2 * kDepth + 8) return _URC_END_OF_STACK;
  w->out[w->n++] = ip;
  return _URC_NO_REASON;
}

void on_prof(int, siginfo_t*, void* ucv) {
  if (!g_on.load(std::memory_order_relaxed) || t_index < 0) return;
  const size_t i = g_next.fetch_add(1, std::memory_order_relaxed);
  if (i >= kCapacity) return;
  const int saved_errno = errno;
  Sample& s = g_samples[i];
  s.thread = uint16_t(t_index);
  const auto* uc = static_cast<const ucontext_t*>(ucv);
  const uintptr_t pc = uintptr_t(uc->uc_mcontext.gregs[REG_RIP]);
  s.pc[0] = pc;
  s.depth = 1;
  // The unwinder starts in this handler, passes the signal trampoline, then reaches the
  // interrupted frame (its IP is `pc`); the frames after it are the callers.
  uintptr_t frames[2 * kDepth + 8];
  Walk w{frames, 0};
  _Unwind_Backtrace(walk_frame, &w);
  int k = 0;
  while (k < w.n && frames[k] != pc) ++k;
  for (++k; k < w.n && s.depth < kDepth; ++k) s.pc[s.depth++] = frames[k];
  errno = saved_errno;
}
}  // namespace

bool start(const std::string& path, int hz) {
  if (g_on.load() || hz <= 0) return false;
  g_path = path;
  g_period_ns = 1000000000L / hz;
  g_samples.reset(new Sample[kCapacity]);
  {
    uintptr_t warm[4];
    Walk w{warm, 0};
    _Unwind_Backtrace(walk_frame, &w);  // first use initialises the unwinder outside a handler
  }
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
