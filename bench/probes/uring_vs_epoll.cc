// Probe: how much of a loopback request/response server's CPU could io_uring save over the
// edge-triggered epoll + recv/send loop the hola workers use? (profiles/README.md, "Why
// there is no io_uring backend".)
//
// One server thread pinned to --server-cpu answers fixed-size requests (the 45-byte wrk-style
// GET) with a fixed 160-byte response on K keep-alive loopback connections. Client threads
// (always epoll, pinned to --client-cpus, one request in flight per connection) saturate it,
// so req/s is set by the server thread's cost per request. Server modes, run interleaved:
//   epoll : epoll_wait + recv + send per ready socket (the hola worker's pattern)
//   uring : io_uring (raw syscalls, no liburing), one IORING_OP_RECV re-armed per connection
//           and one IORING_OP_SEND per response; one io_uring_enter per batch submits and
//           reaps. SINGLE_ISSUER + DEFER_TASKRUN when the kernel offers them.
// Prints one JSON line per run: mode, req/s, server CPU ns per request.
#include <errno.h>
#include <linux/io_uring.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <pthread.h>
#include <sched.h>
#include <sys/epoll.h>
#include <sys/ioctl.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#ifndef IORING_SETUP_SINGLE_ISSUER  // older uapi headers than the running kernel
#define IORING_SETUP_SINGLE_ISSUER (1U << 12)
#endif
#ifndef IORING_SETUP_DEFER_TASKRUN
#define IORING_SETUP_DEFER_TASKRUN (1U << 13)
#endif

namespace {

constexpr size_t kReqLen = 45, kRespLen = 160;
std::atomic<bool> g_stop{false};
std::atomic<uint64_t> g_done{0};

void pin(int cpu) {
  if (cpu < 0) return;
  cpu_set_t s;
  CPU_ZERO(&s);
  CPU_SET(cpu, &s);
  pthread_setaffinity_np(pthread_self(), sizeof s, &s);
}

int64_t thread_cpu_ns() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return int64_t(ts.tv_sec) * 1000000000 + ts.tv_nsec;
}

// ---------------------------------------------------------------- raw io_uring
struct Uring {
  int fd = -1;
  unsigned *sq_head, *sq_tail, *sq_mask, *sq_array, *cq_head, *cq_tail, *cq_mask;
  io_uring_sqe* sqes;
  io_uring_cqe* cqes;
  unsigned pending = 0;

  bool init(unsigned entries) {
    io_uring_params p{};
    p.flags = IORING_SETUP_SINGLE_ISSUER | IORING_SETUP_DEFER_TASKRUN;
    fd = int(syscall(__NR_io_uring_setup, entries, &p));
    if (fd < 0) {
      p = io_uring_params{};
      fd = int(syscall(__NR_io_uring_setup, entries, &p));
      if (fd < 0) return false;
    }
    size_t sq_sz = p.sq_off.array + p.sq_entries * sizeof(unsigned);
    size_t cq_sz = p.cq_off.cqes + p.cq_entries * sizeof(io_uring_cqe);
    if (p.features & IORING_FEAT_SINGLE_MMAP) sq_sz = cq_sz = std::max(sq_sz, cq_sz);
    auto* sq = static_cast<char*>(mmap(nullptr, sq_sz, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd,
                                       IORING_OFF_SQ_RING));
    char* cq = sq;
    if (!(p.features & IORING_FEAT_SINGLE_MMAP))
      cq = static_cast<char*>(mmap(nullptr, cq_sz, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd,
                                   IORING_OFF_CQ_RING));
    sqes = static_cast<io_uring_sqe*>(mmap(nullptr, p.sq_entries * sizeof(io_uring_sqe), PROT_READ | PROT_WRITE,
                                           MAP_SHARED | MAP_POPULATE, fd, IORING_OFF_SQES));
    if (sq == MAP_FAILED || cq == MAP_FAILED || sqes == MAP_FAILED) return false;
    sq_head = reinterpret_cast<unsigned*>(sq + p.sq_off.head);
    sq_tail = reinterpret_cast<unsigned*>(sq + p.sq_off.tail);
    sq_mask = reinterpret_cast<unsigned*>(sq + p.sq_off.ring_mask);
    sq_array = reinterpret_cast<unsigned*>(sq + p.sq_off.array);
    cq_head = reinterpret_cast<unsigned*>(cq + p.cq_off.head);
    cq_tail = reinterpret_cast<unsigned*>(cq + p.cq_off.tail);
    cq_mask = reinterpret_cast<unsigned*>(cq + p.cq_off.ring_mask);
    cqes = reinterpret_cast<io_uring_cqe*>(cq + p.cq_off.cqes);
    return true;
  }
  io_uring_sqe* get() {
    unsigned tail = *sq_tail;
    unsigned idx = tail & *sq_mask;
    io_uring_sqe* e = &sqes[idx];
    memset(e, 0, sizeof *e);
    sq_array[idx] = idx;
    __atomic_store_n(sq_tail, tail + 1, __ATOMIC_RELEASE);
    ++pending;
    return e;
  }
  int enter(unsigned min_complete) {
    int r = int(syscall(__NR_io_uring_enter, fd, pending, min_complete, IORING_ENTER_GETEVENTS, nullptr, 0));
    if (r >= 0) pending -= unsigned(r) < pending ? unsigned(r) : pending;
    return r;
  }
};

struct UConn {
  int fd;
  char in[4096];
  size_t have = 0;
  bool sending = false;
};

void serve_uring(const std::vector<int>& fds, const char* resp) {
  Uring u;
  if (!u.init(4096)) {
    fprintf(stderr, "io_uring_setup failed: %s\n", strerror(errno));
    g_stop = true;
    return;
  }
  std::vector<UConn> cs(fds.size());
  auto arm_recv = [&](size_t i) {
    io_uring_sqe* e = u.get();
    e->opcode = IORING_OP_RECV;
    e->fd = cs[i].fd;
    e->addr = reinterpret_cast<uint64_t>(cs[i].in + cs[i].have);
    e->len = unsigned(sizeof cs[i].in - cs[i].have);
    e->user_data = (uint64_t(i) << 1) | 0;
  };
  for (size_t i = 0; i < fds.size(); ++i) {
    cs[i].fd = fds[i];
    arm_recv(i);
  }
  while (!g_stop.load(std::memory_order_relaxed)) {
    if (u.enter(1) < 0 && errno != EINTR && errno != EAGAIN && errno != EBUSY) break;
    unsigned head = *u.cq_head;
    const unsigned tail = __atomic_load_n(u.cq_tail, __ATOMIC_ACQUIRE);
    for (; head != tail; ++head) {
      const io_uring_cqe& c = u.cqes[head & *u.cq_mask];
      const size_t i = size_t(c.user_data >> 1);
      const bool is_send = c.user_data & 1;
      UConn& k = cs[i];
      if (is_send) {
        k.sending = false;
        continue;
      }
      if (c.res <= 0) {
        if (c.res == -EAGAIN || c.res == -EINTR) arm_recv(i);
        continue;
      }
      k.have += size_t(c.res);
      size_t n = k.have / kReqLen;
      for (size_t r = 0; r < n; ++r) {  // the response bytes are a shared constant
        io_uring_sqe* e = u.get();
        e->opcode = IORING_OP_SEND;
        e->fd = k.fd;
        e->addr = reinterpret_cast<uint64_t>(resp);
        e->len = unsigned(kRespLen);
        e->msg_flags = MSG_NOSIGNAL;
        e->user_data = (uint64_t(i) << 1) | 1;
        k.sending = true;
      }
      k.have -= n * kReqLen;
      if (k.have) memmove(k.in, k.in + n * kReqLen, k.have);
      arm_recv(i);
    }
    __atomic_store_n(u.cq_head, head, __ATOMIC_RELEASE);
  }
  close(u.fd);
}

void serve_epoll(const std::vector<int>& fds, const char* resp) {
  int ep = epoll_create1(0);
  std::vector<UConn> cs(fds.size());
  for (size_t i = 0; i < fds.size(); ++i) {
    cs[i].fd = fds[i];
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLET;
    ev.data.u64 = i;
    epoll_ctl(ep, EPOLL_CTL_ADD, fds[i], &ev);
  }
  epoll_event evs[256];
  while (!g_stop.load(std::memory_order_relaxed)) {
    int n = epoll_wait(ep, evs, 256, 100);
    for (int j = 0; j < n; ++j) {
      UConn& k = cs[evs[j].data.u64];
      for (;;) {
        const size_t room = sizeof k.in - k.have;
        ssize_t r = recv(k.fd, k.in + k.have, room, 0);
        if (r <= 0) break;
        k.have += size_t(r);
        size_t m = k.have / kReqLen;
        for (size_t q = 0; q < m; ++q) send(k.fd, resp, kRespLen, MSG_NOSIGNAL);
        k.have -= m * kReqLen;
        if (k.have) memmove(k.in, k.in + m * kReqLen, k.have);
        if (size_t(r) < room) break;  // short read: drained
      }
    }
  }
  close(ep);
}

void client(std::vector<int> fds, int cpu, const char* req) {
  pin(cpu);
  int ep = epoll_create1(0);
  std::vector<size_t> got(fds.size(), 0);
  for (size_t i = 0; i < fds.size(); ++i) {
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLET;
    ev.data.u64 = i;
    epoll_ctl(ep, EPOLL_CTL_ADD, fds[i], &ev);
    send(fds[i], req, kReqLen, MSG_NOSIGNAL);
  }
  epoll_event evs[256];
  char buf[8192];
  uint64_t done = 0;
  while (!g_stop.load(std::memory_order_relaxed)) {
    int n = epoll_wait(ep, evs, 256, 100);
    for (int j = 0; j < n; ++j) {
      size_t i = evs[j].data.u64;
      for (;;) {
        ssize_t r = recv(fds[i], buf, sizeof buf, 0);
        if (r <= 0) break;
        got[i] += size_t(r);
        while (got[i] >= kRespLen) {
          got[i] -= kRespLen;
          ++done;
          send(fds[i], req, kReqLen, MSG_NOSIGNAL);
        }
        if (size_t(r) < sizeof buf) break;
      }
    }
    if (done >= 1024) {
      g_done.fetch_add(done, std::memory_order_relaxed);
      done = 0;
    }
  }
  close(ep);
}

}  // namespace

int main(int argc, char** argv) {
  int server_cpu = 0, conns = 16, rounds = 3;
  double secs = 3;
  std::vector<int> client_cpus = {1, 2};
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string a = argv[i];
    if (a == "--server-cpu") server_cpu = atoi(argv[i + 1]);
    else if (a == "--connections") conns = atoi(argv[i + 1]);
    else if (a == "--seconds") secs = atof(argv[i + 1]);
    else if (a == "--rounds") rounds = atoi(argv[i + 1]);
    else if (a == "--client-cpus") {
      client_cpus.clear();
      std::string s = argv[i + 1];
      size_t p = 0;
      while (p < s.size()) {
        size_t q = s.find(',', p);
        if (q == std::string::npos) q = s.size();
        client_cpus.push_back(atoi(s.substr(p, q - p).c_str()));
        p = q + 1;
      }
    }
  }
  char req[kReqLen], resp[kRespLen];
  memset(req, 'q', sizeof req);
  memset(resp, 'r', sizeof resp);
  for (int round = 0; round < rounds; ++round) {
    for (const char* mode : {"epoll", "uring"}) {
      int lfd = socket(AF_INET, SOCK_STREAM, 0);
      if (lfd < 0) {
        perror("socket");
        return 1;
      }
      int one = 1;
      setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
      sockaddr_in a{};
      a.sin_family = AF_INET;
      a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
      bind(lfd, reinterpret_cast<sockaddr*>(&a), sizeof a);
      socklen_t al = sizeof a;
      getsockname(lfd, reinterpret_cast<sockaddr*>(&a), &al);
      listen(lfd, 1024);
      std::vector<int> sfds, cfds;
      for (int i = 0; i < conns; ++i) {
        int c = socket(AF_INET, SOCK_STREAM, 0);
        if (c < 0 || connect(c, reinterpret_cast<sockaddr*>(&a), sizeof a) != 0) {
          perror("connect");
          return 1;
        }
        int s = accept(lfd, nullptr, nullptr);
        setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
        setsockopt(s, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
        int fl = 1;
        ioctl(c, FIONBIO, &fl);
        ioctl(s, FIONBIO, &fl);
        cfds.push_back(c);
        sfds.push_back(s);
      }
      g_stop = false;
      g_done = 0;
      int64_t server_cpu_ns = 0;
      std::thread srv([&] {
        pin(server_cpu);
        int64_t c0 = thread_cpu_ns();
        if (std::string(mode) == "uring") serve_uring(sfds, resp);
        else serve_epoll(sfds, resp);
        server_cpu_ns = thread_cpu_ns() - c0;
      });
      std::vector<std::thread> cl;
      const size_t nc = client_cpus.size();
      for (size_t t = 0; t < nc; ++t) {
        std::vector<int> mine;
        for (size_t i = t; i < cfds.size(); i += nc) mine.push_back(cfds[i]);
        cl.emplace_back(client, mine, client_cpus[t], req);
      }
      usleep(500000);  // warm up
      uint64_t d0 = g_done.load();
      timespec t0, t1;
      clock_gettime(CLOCK_MONOTONIC, &t0);
      usleep(useconds_t(secs * 1e6));
      uint64_t d1 = g_done.load();
      clock_gettime(CLOCK_MONOTONIC, &t1);
      g_stop = true;
      for (auto& t : cl) t.join();
      send(cfds[0], req, kReqLen, MSG_NOSIGNAL);  // a last completion wakes a server blocked in io_uring_enter
      srv.join();
      const double el = double(t1.tv_sec - t0.tv_sec) + double(t1.tv_nsec - t0.tv_nsec) / 1e9;
      const uint64_t total = g_done.load();
      printf("{\"mode\":\"%s\",\"round\":%d,\"connections\":%d,\"rps\":%.0f,\"server_cpu_ns_per_req\":%.0f}\n", mode,
             round, conns, double(d1 - d0) / el, total ? double(server_cpu_ns) / double(total) : 0.0);
      fflush(stdout);
      for (int f : sfds) close(f);
      for (int f : cfds) close(f);
      close(lfd);
    }
  }
  return 0;
}
