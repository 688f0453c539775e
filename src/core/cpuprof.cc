#include "core/cpuprof.h"

#include <errno.h>
#include <fcntl.h>
#include <linux/perf_event.h>
#include <pthread.h>
#include <sys/ioctl.h>
#include <sched.h>
#include <signal.h>
#include <sys/syscall.h>
#include <time.h>
#include <ucontext.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <string>
#include <thread>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
// Sampling handlers running right now. write() turns g_on off and then waits for this to reach
// 0 before it reads the samples: a handler that passed the g_on check just before may still be
// filling its slot (the store of g_on and the load of this count, and the handler's increment
// and its load of g_on, are sequentially consistent, so one of the two sides sees the other).
// The handler's release decrement publishes its slot to write()'s acquire load.
std::atomic<int> g_inflight{0};
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
// locks, no allocation. When the context is in code from another object (libc's syscall
// wrappers: send, recv, epoll_wait), which keeps no frame pointer, the caller is found by
// scanning the top of the stack for the first return address into a different mapping.
// Not instrumented by the sanitizers: it reads saved frame pointers and return addresses of
// another function's frames, which AddressSanitizer's stack redzones would flag.
__attribute__((no_sanitize("address", "thread", "undefined")))
int walk(const ucontext_t* uc, uintptr_t* out, int max) {
  const uintptr_t pc = uintptr_t(uc->uc_mcontext.gregs[REG_RIP]);
  const uintptr_t sp = uintptr_t(uc->uc_mcontext.gregs[REG_RSP]);
  uintptr_t fp = uintptr_t(uc->uc_mcontext.gregs[REG_RBP]);
  int depth = 0;
  out[depth++] = pc;
  const bool bounded = t_stack_hi > t_stack_lo;
  auto in_stack = [&](uintptr_t a) { return bounded && a >= t_stack_lo && a + 16 <= t_stack_hi && !(a & 7); };
  const int pc_range = exec_range(pc);
  uintptr_t caller = 0;
  if (pc_range != g_own_range) {
    for (int k = 0; k < 16 && depth < max && in_stack(sp + 8 * uintptr_t(k)); ++k) {
      const uintptr_t w = *reinterpret_cast<const uintptr_t*>(sp + 8 * uintptr_t(k));
      const int r = exec_range(w);
      if (r >= 0 && r != pc_range) {
        caller = w;
        out[depth++] = w;
        break;
      }
    }
  }
  bool first = true;
  while (depth < max && in_stack(fp)) {
    const uintptr_t ret = *reinterpret_cast<const uintptr_t*>(fp + 8);
    const uintptr_t next = *reinterpret_cast<const uintptr_t*>(fp);
    if (!executable(ret)) break;
    if (!(first && ret == caller)) out[depth++] = ret;
    first = false;
    if (next <= fp) break;  // the chain must climb the stack
    fp = next;
  }
  return depth;
}

void on_prof(int, siginfo_t*, void* ucv) {
  if (t_index < 0) return;
  g_inflight.fetch_add(1, std::memory_order_seq_cst);
  if (g_on.load(std::memory_order_seq_cst)) {
    const size_t i = g_next.fetch_add(1, std::memory_order_relaxed);
    if (i < kCapacity) {
      const int saved_errno = errno;
      Sample& s = g_samples[i];
      s.thread = uint16_t(t_index);
      s.depth = uint8_t(walk(static_cast<const ucontext_t*>(ucv), s.pc, kDepth));
      errno = saved_errno;
    }
  }
  g_inflight.fetch_sub(1, std::memory_order_release);
}

// ---- on-demand capture of another thread's stack (stall reports) ----
constexpr int kCaptureSignal = 40;  // a real-time signal no thread blocks (SIGRTMIN is 34)
std::mutex g_cap_mu;                // one capture at a time
// Request word: (sequence << 2) | state, state 0 idle, 1 requested, 3 being written, 2 done.
// The handler walks into its own buffer and publishes only if the word still names its
// request, so a signal that arrives after its capture gave up can never write into a later
// capture's result.
std::atomic<uint64_t> g_cap_word{0};
std::atomic<int> g_cap_tid{0};      // the thread asked
uintptr_t g_cap_pcs[kMaxCaptureDepth];
int g_cap_depth = 0;
std::atomic<bool> g_cap_installed{false};

void on_capture(int, siginfo_t*, void* ucv) {
  uint64_t w = g_cap_word.load(std::memory_order_acquire);
  if ((w & 3) != 1) return;
  if (int(syscall(SYS_gettid)) != g_cap_tid.load(std::memory_order_relaxed)) return;
  const int saved_errno = errno;
  uintptr_t pcs[kMaxCaptureDepth];
  const int n = walk(static_cast<const ucontext_t*>(ucv), pcs, kMaxCaptureDepth);
  if (g_cap_word.compare_exchange_strong(w, (w & ~uint64_t(3)) | 3, std::memory_order_acq_rel)) {
    for (int i = 0; i < n; ++i) g_cap_pcs[i] = pcs[i];
    g_cap_depth = n;
    g_cap_word.store((w & ~uint64_t(3)) | 2, std::memory_order_release);
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

int current_tid() { return int(syscall(SYS_gettid)); }

void note_thread() {
  if (t_stack_hi <= t_stack_lo) note_stack_bounds();
}

bool enable_capture() {
  if (g_cap_installed.load()) return true;
  struct sigaction sa {};
  sa.sa_sigaction = on_capture;
  sa.sa_flags = SA_SIGINFO | SA_RESTART;
  sigemptyset(&sa.sa_mask);
  if (sigaction(kCaptureSignal, &sa, nullptr) != 0) return false;
  g_cap_installed.store(true);
  return true;
}

int capture(int tid, uintptr_t* pcs, int max, int timeout_ms) {
  if (!g_cap_installed.load() || max <= 0 || tid <= 0) return 0;
  std::lock_guard<std::mutex> g(g_cap_mu);
  if (!g_on.load()) {
    load_exec_ranges();  // the profiler keeps its own (read by its handler meanwhile)
    g_own_range = exec_range(uintptr_t(&on_prof));
  }
  g_cap_tid.store(tid, std::memory_order_relaxed);
  const uint64_t seq = (g_cap_word.load() >> 2) + 1;
  const uint64_t requested = seq << 2 | 1;
  g_cap_word.store(requested, std::memory_order_release);
  if (syscall(SYS_tgkill, getpid(), tid, kCaptureSignal) != 0) {
    g_cap_word.store(seq << 2);
    return 0;
  }
  const auto until = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
  for (;;) {
    const uint64_t w = g_cap_word.load(std::memory_order_acquire);
    if ((w & 3) == 2) break;
    if ((w & 3) == 1 && std::chrono::steady_clock::now() >= until) {
      // No answer (a stopped thread, or one that blocks the signal): withdraw the request; a
      // handler that runs later finds it gone. If the handler is writing right now (state 3),
      // wait for it instead.
      uint64_t expect = requested;
      if (g_cap_word.compare_exchange_strong(expect, seq << 2, std::memory_order_acq_rel)) return 0;
      continue;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  const int n = std::min(max, g_cap_depth);
  for (int i = 0; i < n; ++i) pcs[i] = g_cap_pcs[i];
  g_cap_word.store(seq << 2, std::memory_order_release);
  return n;
}

std::string describe_pcs(const uintptr_t* pcs, int n) {
  // Each frame as object+offset (symbolise with `addr2line -f -C -e OBJECT OFFSET`, or
  // bench/cpuprof_report.py): the maps are read now, outside any signal handler.
  struct Map {
    uintptr_t lo, hi, off;
    std::string path;
  };
  std::vector<Map> maps;
  std::ifstream f("/proc/self/maps");
  for (std::string line; std::getline(f, line);) {
    unsigned long lo = 0, hi = 0, off = 0;
    char perms[5] = {};
    int pos = 0;
    if (sscanf(line.c_str(), "%lx-%lx %4s %lx %*s %*s%n", &lo, &hi, perms, &off, &pos) < 4 || perms[2] != 'x') continue;
    std::string path = pos > 0 && size_t(pos) < line.size() ? line.substr(size_t(pos)) : "";
    path.erase(0, path.find_first_not_of(' '));
    maps.push_back({lo, hi, off, path.empty() ? "?" : path});
  }
  std::string out;
  char buf[64];
  for (int i = 0; i < n; ++i) {
    const uintptr_t pc = i ? pcs[i] - 1 : pcs[i];  // return addresses: the call's own line
    auto it = std::find_if(maps.begin(), maps.end(), [pc](const Map& m) { return pc >= m.lo && pc < m.hi; });
    if (it == maps.end()) {
      snprintf(buf, sizeof buf, " #%d ?(0x%lx)", i, (unsigned long)pc);
      out += buf;
      continue;
    }
    const std::string base = it->path.substr(it->path.rfind('/') == std::string::npos ? 0 : it->path.rfind('/') + 1);
    snprintf(buf, sizeof buf, "+0x%lx", (unsigned long)(pc - it->lo + it->off));
    out += " #" + std::to_string(i) + " " + base + buf;
  }
  return out;
}

// HOLA_CPUPROF_EVENT=user-cycles: sample every HOLA_CPUPROF_PERIOD (default 200,000) cycles
// spent in user space instead of every period of CPU time. The hardware counter's overflow
// signal is routed to the thread as SIGPROF (same handler, same stacks). The CPU-time profile
// of a syscall-bound server is ~93 % send/recv/epoll_wait; this one shows only the server's
// own work (and libc's). Threads fall back to the CPU-time timer where no PMU is present.
// HOLA_CPUPROF_EVENT=user-instructions samples retired user-space instructions instead (same
// period variable): where a request's instructions are, for instruction-count work.
bool g_user_cycles = false;
uint64_t g_cycles_period = 200000;
uint64_t g_event_config = PERF_COUNT_HW_CPU_CYCLES;
std::vector<int> g_event_fds;  // under g_mu
thread_local int t_event_fd = -1;

int open_user_cycles() {
  perf_event_attr a;
  memset(&a, 0, sizeof a);
  a.type = PERF_TYPE_HARDWARE;
  a.size = sizeof a;
  a.config = g_event_config;
  a.sample_period = g_cycles_period;
  a.wakeup_events = 1;
  a.exclude_kernel = 1;
  a.exclude_hv = 1;
  a.disabled = 1;
  const int fd = int(syscall(SYS_perf_event_open, &a, 0, -1, -1, PERF_FLAG_FD_CLOEXEC));
  if (fd < 0) return -1;
  f_owner_ex owner{F_OWNER_TID, pid_t(syscall(SYS_gettid))};
  if (fcntl(fd, F_SETFL, O_ASYNC | O_NONBLOCK) != 0 || fcntl(fd, F_SETSIG, SIGPROF) != 0 ||
      fcntl(fd, F_SETOWN_EX, &owner) != 0 || ioctl(fd, PERF_EVENT_IOC_RESET, 0) != 0 ||
      ioctl(fd, PERF_EVENT_IOC_ENABLE, 0) != 0) {
    close(fd);
    return -1;
  }
  return fd;
}

bool start(const std::string& path, int hz) {
  if (g_on.load() || hz <= 0) return false;
  g_path = path;
  g_period_ns = 1000000000L / hz;
  if (const char* e = getenv("HOLA_CPUPROF_EVENT");
      e && (strcmp(e, "user-cycles") == 0 || strcmp(e, "user-instructions") == 0)) {
    g_user_cycles = true;
    if (strcmp(e, "user-instructions") == 0) g_event_config = PERF_COUNT_HW_INSTRUCTIONS;
    if (const char* p = getenv("HOLA_CPUPROF_PERIOD"); p && atoll(p) > 0) g_cycles_period = uint64_t(atoll(p));
  }
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
  if (g_user_cycles) {
    // t_index first: an overflow may arrive as soon as the counter is enabled
    {
      std::lock_guard<std::mutex> g(g_mu);
      t_index = int(g_names.size());
      g_names.push_back(name);
    }
    t_event_fd = open_user_cycles();
    if (t_event_fd >= 0) {
      std::lock_guard<std::mutex> g(g_mu);
      g_event_fds.push_back(t_event_fd);
      t_armed = true;
      return;
    }
    std::lock_guard<std::mutex> g(g_mu);
    g_names[size_t(t_index)] += " (CPU-time timer: no cycle counter)";
  }
  if (timer_create(CLOCK_THREAD_CPUTIME_ID, &sev, &t_timer) != 0) return;
  {
    std::lock_guard<std::mutex> g(g_mu);
    if (t_index < 0) {
      t_index = int(g_names.size());
      g_names.push_back(name);
    }
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
  if (t_event_fd >= 0) {
    ioctl(t_event_fd, PERF_EVENT_IOC_DISABLE, 0);
  } else {
    itimerspec off{};
    timer_settime(t_timer, 0, &off, nullptr);
  }
  t_armed = false;
}

bool write() {
  if (!g_on.exchange(false, std::memory_order_seq_cst)) return false;
  {
    std::lock_guard<std::mutex> g(g_mu);
    itimerspec off{};
    for (timer_t t : g_timers) timer_settime(t, 0, &off, nullptr);
    for (int fd : g_event_fds) ioctl(fd, PERF_EVENT_IOC_DISABLE, 0);
  }
  // a handler already past its g_on check finishes its sample first (it runs for microseconds)
  while (g_inflight.load(std::memory_order_acquire) != 0) sched_yield();
  const size_t n = std::min(g_next.load(), kCapacity);
  // identical (thread, stack) samples are written once with their count
  std::map<std::pair<int, std::vector<uintptr_t>>, uint64_t> stacks;
  for (size_t i = 0; i < n; ++i) {
    const Sample& s = g_samples[i];
    stacks[{s.thread, std::vector<uintptr_t>(s.pc, s.pc + s.depth)}]++;
  }
  std::ofstream f(g_path);
  if (!f) return false;
  f << "# hola cpu profile\n";
  if (g_user_cycles && !g_event_fds.empty())
    f << "event " << (g_event_config == PERF_COUNT_HW_INSTRUCTIONS ? "user-instructions" : "user-cycles")
      << "\nperiod_cycles " << g_cycles_period << "\n";
  f << "period_ns " << g_period_ns << "\nsamples " << n << "\ndropped "
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
