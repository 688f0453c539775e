// Probe: does io_uring pay on the chaining hop, where each request costs hola four socket
// syscalls instead of two? ("chaining path syscall batching"; the headline
// path's answer is r31_uring: +3.6 %, not adopted.)
//
// The measured thread plays hola A on /api/hola-chaining, reduced to its I/O: for each client
// request it (1) receives the request, (2) sends a request to the downstream service on its
// own kept-alive upstream connection, (3) receives the downstream response, (4) sends the
// response to the client. One request in flight per connection pair, as hola's unpipelined
// client pool does. Downstream ("aloha") and client threads are plain epoll and pinned apart.
// Modes, run interleaved:
//   epoll : edge-triggered epoll_wait + recv/send, four syscalls per request (hola's pattern)
//   uring : io_uring (raw syscalls), a RECV armed on every socket, SENDs queued as data
//           arrives; one io_uring_enter per loop iteration submits the batch and reaps
//           (SINGLE_ISSUER + DEFER_TASKRUN when the kernel offers them)
// One JSON line per run: mode, chained req/s, hola-A CPU ns per request.
//
//   g++ -O2 -std=c++20 -pthread bench/probes/uring_chain.cc -o /tmp/uring_chain
//   /tmp/uring_chain --hop-cpu 2 --aloha-cpu 3 --client-cpus 4,5 --connections 64 --rounds 4
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

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#ifndef IORING_SETUP_SINGLE_ISSUER
#define IORING_SETUP_SINGLE_ISSUER (1U << 12)
#endif
#ifndef IORING_SETUP_DEFER_TASKRUN
#define IORING_SETUP_DEFER_TASKRUN (1U << 13)
#endif

namespace {

// sizes of the real messages: the loadgen's GET, hola's GET to aloha with B3 headers, aloha's
// JSON answer, hola's chained JSON response
constexpr size_t kCliReq = 60, kUpReq = 260, kUpResp = 190, kCliResp = 230;
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

// One chained pair: the client's connection and hola A's upstream connection for it.
struct Pair {
  int cfd, ufd;
  char cin[4096], uin[4096];
  size_t chave = 0, uhave = 0;
};

// user_data: pair index << 2 | kind
enum Kind : uint64_t { kCliRecv = 0, kUpRecv = 1, kSend = 2 };

void hop_uring(std::vector<Pair>& ps, const char* upreq, const char* cliresp) {
  Uring u;
  if (!u.init(8192)) {
    fprintf(stderr, "io_uring_setup failed: %s\n", strerror(errno));
    g_stop = true;
    return;
  }
  auto recv_on = [&](size_t i, bool up) {
    Pair& p = ps[i];
    io_uring_sqe* e = u.get();
    e->opcode = IORING_OP_RECV;
    e->fd = up ? p.ufd : p.cfd;
    char* buf = up ? p.uin : p.cin;
    size_t have = up ? p.uhave : p.chave;
    e->addr = reinterpret_cast<uint64_t>(buf + have);
    e->len = unsigned(4096 - have);
    e->user_data = (uint64_t(i) << 2) | (up ? kUpRecv : kCliRecv);
  };
  auto send_on = [&](size_t i, int fd, const char* data, size_t len) {
    io_uring_sqe* e = u.get();
    e->opcode = IORING_OP_SEND;
    e->fd = fd;
    e->addr = reinterpret_cast<uint64_t>(data);
    e->len = unsigned(len);
    e->msg_flags = MSG_NOSIGNAL;
    e->user_data = (uint64_t(i) << 2) | kSend;
  };
  for (size_t i = 0; i < ps.size(); ++i) {
    recv_on(i, false);
    recv_on(i, true);
  }
  while (!g_stop.load(std::memory_order_relaxed)) {
    if (u.enter(1) < 0 && errno != EINTR && errno != EAGAIN && errno != EBUSY) break;
    unsigned head = *u.cq_head;
    const unsigned tail = __atomic_load_n(u.cq_tail, __ATOMIC_ACQUIRE);
    for (; head != tail; ++head) {
      const io_uring_cqe& c = u.cqes[head & *u.cq_mask];
      const size_t i = size_t(c.user_data >> 2);
      const uint64_t kind = c.user_data & 3;
      if (kind == kSend) continue;
      Pair& p = ps[i];
      const bool up = kind == kUpRecv;
      if (c.res <= 0) {
        if (c.res == -EAGAIN || c.res == -EINTR) recv_on(i, up);
        continue;
      }
      if (up) {
        p.uhave += size_t(c.res);
        for (; p.uhave >= kUpResp; p.uhave -= kUpResp) send_on(i, p.cfd, cliresp, kCliResp);
      } else {
        p.chave += size_t(c.res);
        for (; p.chave >= kCliReq; p.chave -= kCliReq) send_on(i, p.ufd, upreq, kUpReq);
      }
      recv_on(i, up);
    }
    __atomic_store_n(u.cq_head, head, __ATOMIC_RELEASE);
  }
  close(u.fd);
}

void hop_epoll(std::vector<Pair>& ps, const char* upreq, const char* cliresp) {
  int ep = epoll_create1(0);
  for (size_t i = 0; i < ps.size(); ++i) {
    for (int up = 0; up < 2; ++up) {
      epoll_event ev{};
      ev.events = EPOLLIN | EPOLLET;
      ev.data.u64 = (uint64_t(i) << 1) | uint64_t(up);
      epoll_ctl(ep, EPOLL_CTL_ADD, up ? ps[i].ufd : ps[i].cfd, &ev);
    }
  }
  epoll_event evs[256];
  while (!g_stop.load(std::memory_order_relaxed)) {
    int n = epoll_wait(ep, evs, 256, 100);
    for (int j = 0; j < n; ++j) {
      Pair& p = ps[evs[j].data.u64 >> 1];
      const bool up = evs[j].data.u64 & 1;
      char* buf = up ? p.uin : p.cin;
      size_t& have = up ? p.uhave : p.chave;
      const size_t unit = up ? kUpResp : kCliReq;
      for (;;) {
        const size_t room = 4096 - have;
        ssize_t r = recv(up ? p.ufd : p.cfd, buf + have, room, 0);
        if (r <= 0) break;
        have += size_t(r);
        for (; have >= unit; have -= unit) {
          if (up) send(p.cfd, cliresp, kCliResp, MSG_NOSIGNAL);
          else send(p.ufd, upreq, kUpReq, MSG_NOSIGNAL);
        }
        if (size_t(r) < room) break;
      }
    }
  }
  close(ep);
}

// Answers every kUpReq bytes with kUpResp bytes (the downstream service).
void aloha(std::vector<int> fds, int cpu) {
  pin(cpu);
  int ep = epoll_create1(0);
  std::vector<size_t> have(fds.size(), 0);
  for (size_t i = 0; i < fds.size(); ++i) {
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLET;
    ev.data.u64 = i;
    epoll_ctl(ep, EPOLL_CTL_ADD, fds[i], &ev);
  }
  char resp[kUpResp], buf[8192];
  memset(resp, 'a', sizeof resp);
  epoll_event evs[256];
  while (!g_stop.load(std::memory_order_relaxed)) {
    int n = epoll_wait(ep, evs, 256, 100);
    for (int j = 0; j < n; ++j) {
      const size_t i = evs[j].data.u64;
      for (;;) {
        ssize_t r = recv(fds[i], buf, sizeof buf, 0);
        if (r <= 0) break;
        have[i] += size_t(r);
        for (; have[i] >= kUpReq; have[i] -= kUpReq) send(fds[i], resp, kUpResp, MSG_NOSIGNAL);
        if (size_t(r) < sizeof buf) break;
      }
    }
  }
  close(ep);
}

void client(std::vector<int> fds, int cpu) {
  pin(cpu);
  char req[kCliReq], buf[8192];
  memset(req, 'q', sizeof req);
  int ep = epoll_create1(0);
  std::vector<size_t> got(fds.size(), 0);
  for (size_t i = 0; i < fds.size(); ++i) {
    epoll_event ev{};
    ev.events = EPOLLIN | EPOLLET;
    ev.data.u64 = i;
    epoll_ctl(ep, EPOLL_CTL_ADD, fds[i], &ev);
    send(fds[i], req, kCliReq, MSG_NOSIGNAL);
  }
  epoll_event evs[256];
  uint64_t done = 0;
  while (!g_stop.load(std::memory_order_relaxed)) {
    int n = epoll_wait(ep, evs, 256, 100);
    for (int j = 0; j < n; ++j) {
      const size_t i = evs[j].data.u64;
      for (;;) {
        ssize_t r = recv(fds[i], buf, sizeof buf, 0);
        if (r <= 0) break;
        got[i] += size_t(r);
        for (; got[i] >= kCliResp; got[i] -= kCliResp) {
          ++done;
          send(fds[i], req, kCliReq, MSG_NOSIGNAL);
        }
        if (size_t(r) < sizeof buf) break;
      }
    }
    if (done >= 256) {
      g_done.fetch_add(done, std::memory_order_relaxed);
      done = 0;
    }
  }
  close(ep);
}

// A connected loopback pair (client end, server end), non-blocking, TCP_NODELAY.
bool tcp_pair(int lfd, const sockaddr_in& a, int* c, int* s) {
  *c = socket(AF_INET, SOCK_STREAM, 0);
  if (*c < 0) return false;
  if (connect(*c, reinterpret_cast<const sockaddr*>(&a), sizeof a) != 0) return false;
  *s = accept(lfd, nullptr, nullptr);
  int one = 1;
  for (int fd : {*c, *s}) {
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
    ioctl(fd, FIONBIO, &one);
  }
  return *s >= 0;
}

std::vector<int> parse_list(const std::string& s) {
  std::vector<int> out;
  size_t p = 0;
  while (p < s.size()) {
    size_t q = s.find(',', p);
    if (q == std::string::npos) q = s.size();
    out.push_back(atoi(s.substr(p, q - p).c_str()));
    p = q + 1;
  }
  return out;
}

}  // namespace

int main(int argc, char** argv) {
  int hop_cpu = 0, aloha_cpu = 1, conns = 64, rounds = 3;
  double secs = 3;
  std::vector<int> client_cpus = {2, 3};
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string a = argv[i];
    if (a == "--hop-cpu") hop_cpu = atoi(argv[i + 1]);
    else if (a == "--aloha-cpu") aloha_cpu = atoi(argv[i + 1]);
    else if (a == "--connections") conns = atoi(argv[i + 1]);
    else if (a == "--seconds") secs = atof(argv[i + 1]);
    else if (a == "--rounds") rounds = atoi(argv[i + 1]);
    else if (a == "--client-cpus") client_cpus = parse_list(argv[i + 1]);
  }
  char upreq[kUpReq], cliresp[kCliResp];
  memset(upreq, 'u', sizeof upreq);
  memset(cliresp, 'c', sizeof cliresp);
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
      socklen_t alen = sizeof a;
      getsockname(lfd, reinterpret_cast<sockaddr*>(&a), &alen);
      listen(lfd, 4096);
      std::vector<Pair> ps(static_cast<size_t>(conns));
      std::vector<int> cli_fds, aloha_fds;
      for (auto& p : ps) {
        int c, s, u, d;
        if (!tcp_pair(lfd, a, &c, &s) || !tcp_pair(lfd, a, &u, &d)) {
          perror("connect");
          return 1;
        }
        p.cfd = s;  // hola A's end of the client connection
        p.ufd = u;  // hola A's upstream connection to aloha
        cli_fds.push_back(c);
        aloha_fds.push_back(d);
      }
      g_stop = false;
      g_done = 0;
      int64_t hop_ns = 0;
      std::thread hop([&] {
        pin(hop_cpu);
        const int64_t c0 = thread_cpu_ns();
        if (std::string(mode) == "uring") hop_uring(ps, upreq, cliresp);
        else hop_epoll(ps, upreq, cliresp);
        hop_ns = thread_cpu_ns() - c0;
      });
      std::thread al(aloha, aloha_fds, aloha_cpu);
      std::vector<std::thread> cl;
      const size_t nc = client_cpus.size();
      for (size_t t = 0; t < nc; ++t) {
        std::vector<int> mine;
        for (size_t i = t; i < cli_fds.size(); i += nc) mine.push_back(cli_fds[i]);
        cl.emplace_back(client, mine, client_cpus[t]);
      }
      usleep(500000);
      const uint64_t d0 = g_done.load();
      timespec t0, t1;
      clock_gettime(CLOCK_MONOTONIC, &t0);
      usleep(useconds_t(secs * 1e6));
      const uint64_t d1 = g_done.load();
      clock_gettime(CLOCK_MONOTONIC, &t1);
      g_stop = true;
      for (auto& t : cl) t.join();
      al.join();
      char wake[kCliReq];
      memset(wake, 'q', sizeof wake);
      send(cli_fds[0], wake, kCliReq, MSG_NOSIGNAL);  // wakes a hop blocked in io_uring_enter
      hop.join();
      const double el = double(t1.tv_sec - t0.tv_sec) + double(t1.tv_nsec - t0.tv_nsec) / 1e9;
      const uint64_t total = g_done.load();
      printf("{\"mode\":\"%s\",\"round\":%d,\"connections\":%d,\"rps\":%.0f,\"hop_cpu_ns_per_req\":%.0f}\n", mode,
             round, conns, double(d1 - d0) / el, total ? double(hop_ns) / double(total) : 0.0);
      fflush(stdout);
      for (auto& p : ps) {
        close(p.cfd);
        close(p.ufd);
      }
      for (int f : cli_fds) close(f);
      for (int f : aloha_fds) close(f);
      close(lfd);
    }
  }
  return 0;
}
