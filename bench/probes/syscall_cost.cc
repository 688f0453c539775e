// Measures the round-trip cost of a trivial syscall and of epoll_wait(0) on this host, to
// decide whether syscall batching (io_uring) could matter next to the TCP work per request.
#include <sys/epoll.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>

int main() {
  const int n = 2000000;
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) syscall(SYS_getppid);
  auto t1 = std::chrono::steady_clock::now();
  int ep = epoll_create1(0);
  epoll_event ev[8];
  for (int i = 0; i < n; ++i) epoll_wait(ep, ev, 8, 0);
  auto t2 = std::chrono::steady_clock::now();
  double a = std::chrono::duration<double, std::nano>(t1 - t0).count() / n;
  double b = std::chrono::duration<double, std::nano>(t2 - t1).count() / n;
  printf("{\"getppid_ns\": %.1f, \"epoll_wait0_ns\": %.1f}\n", a, b);
  return 0;
}
