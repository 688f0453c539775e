// instr_count: user-space instructions and cycles of a program and all its threads.
//
//   instr_count OUT.json -- PROGRAM ARGS...
//
// A deterministic measure of a server's own code per request, next to the CPU-time A/Bs,
// whose noise (other tenants on the SMT siblings, ±0.7 % per session) is as large as the
// differences left between trees. The kernel's share (send/recv/epoll, ~93 % of the
// headline server's CPU) is the same syscall sequence for every tree and is not counted
// (exclude_kernel: allowed at perf_event_paranoid <= 2 for one's own processes); the
// program's busy-polling must be off, or its spin loop counts as work.
//
// The child is stopped on a pipe until the counters (inherit = 1: every thread it creates)
// are attached, then execs PROGRAM. SIGTERM/SIGINT to instr_count are passed on to it. At
// its exit the totals are written to OUT.json ({"instructions", "cycles", "status"});
// a counter the host does not provide is null.
#include <linux/perf_event.h>
#include <signal.h>
#include <sys/syscall.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstring>

namespace {

pid_t g_child = -1;

void forward(int sig) {
  if (g_child > 0) kill(g_child, sig);
}

int open_counter(pid_t pid, uint64_t config) {
  perf_event_attr a;
  memset(&a, 0, sizeof a);
  a.type = PERF_TYPE_HARDWARE;
  a.size = sizeof a;
  a.config = config;
  a.exclude_kernel = 1;
  a.exclude_hv = 1;
  a.inherit = 1;  // threads created after attaching are counted; their counts fold in at exit
  return int(syscall(SYS_perf_event_open, &a, pid, -1, -1, 0));
}

bool read_counter(int fd, uint64_t* v) {
  return fd >= 0 && read(fd, v, sizeof *v) == ssize_t(sizeof *v);
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4 || strcmp(argv[2], "--") != 0) {
    fprintf(stderr, "usage: instr_count OUT.json -- PROGRAM ARGS...\n");
    return 2;
  }
  int go[2];
  if (pipe(go) != 0) return 2;
  g_child = fork();
  if (g_child < 0) return 2;
  if (g_child == 0) {
    close(go[1]);
    char b;
    if (read(go[0], &b, 1) != 1) _exit(127);
    close(go[0]);
    execvp(argv[3], argv + 3);
    fprintf(stderr, "instr_count: exec %s: %s\n", argv[3], strerror(errno));
    _exit(127);
  }
  close(go[0]);
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_handler = forward;
  sigaction(SIGTERM, &sa, nullptr);
  sigaction(SIGINT, &sa, nullptr);
  const int fi = open_counter(g_child, PERF_COUNT_HW_INSTRUCTIONS);
  const int ferr = fi < 0 ? errno : 0;
  const int fc = open_counter(g_child, PERF_COUNT_HW_CPU_CYCLES);
  if (fi < 0) fprintf(stderr, "instr_count: no instruction counter: %s\n", strerror(ferr));
  if (write(go[1], "g", 1) != 1) return 2;
  close(go[1]);
  int st = 0;
  while (waitpid(g_child, &st, 0) < 0 && errno == EINTR) {
  }
  uint64_t ins = 0, cyc = 0;
  const bool hi = read_counter(fi, &ins), hc = read_counter(fc, &cyc);
  FILE* f = fopen(argv[1], "w");
  if (!f) return 2;
  char a[32] = "null", b[32] = "null";
  if (hi) snprintf(a, sizeof a, "%llu", (unsigned long long)ins);
  if (hc) snprintf(b, sizeof b, "%llu", (unsigned long long)cyc);
  fprintf(f, "{\"instructions\": %s, \"cycles\": %s, \"status\": %d, \"error\": \"%s\"}\n", a, b,
          WIFEXITED(st) ? WEXITSTATUS(st) : -WTERMSIG(st), fi < 0 ? strerror(ferr) : "");
  fclose(f);
  return WIFEXITED(st) ? WEXITSTATUS(st) : 128 + WTERMSIG(st);
}
