// hola_zipkin_sink — a discard Zipkin collector for benchmarking the deployed tracing
// configuration (ZIPKIN_SERVER_URL is set in the image: /root/reference/Dockerfile:6).
//
// Accepts POST /api/v1/spans and /api/v2/spans (keep-alive, Content-Length or chunked
// bodies), counts the spans in each JSON batch (one "traceId" key per span) and answers
// 202 Accepted, as a Zipkin server does; the spans themselves are discarded.
// GET /stats returns {"posts":..,"spans":..,"bytes":..,"bad":..}.
//
//   hola_zipkin_sink [--host H] [--port P] [--port-file F] [--cpu-list L]
#include <errno.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "core/affinity.h"
#include "core/net.h"
#include "http/parser.h"

using namespace hola;

namespace {

struct Stats {
  uint64_t posts = 0, spans = 0, bytes = 0, bad = 0;
};

struct Conn {
  int fd;
  std::string in;
};

uint64_t count_spans(std::string_view body) {
  uint64_t n = 0;
  for (size_t p = body.find("\"traceId\""); p != std::string_view::npos; p = body.find("\"traceId\"", p + 9)) ++n;
  return n;
}

// Returns bytes consumed by one complete request at the front of `in`, 0 if incomplete,
// -1 if malformed; fills *method, *path and *body.
long parse_one(const std::string& in, std::string* method, std::string* path, std::string* body) {
  size_t he = in.find("\r\n\r\n");
  if (he == std::string::npos) return in.size() > (64 << 10) ? -1 : 0;
  std::string_view head(in.data(), he);
  size_t sp1 = head.find(' ');
  size_t sp2 = sp1 == std::string_view::npos ? sp1 : head.find(' ', sp1 + 1);
  if (sp2 == std::string_view::npos) return -1;
  *method = std::string(head.substr(0, sp1));
  *path = std::string(head.substr(sp1 + 1, sp2 - sp1 - 1));
  long cl = 0;
  bool chunked = false;
  size_t p = head.find("\r\n");
  while (p != std::string_view::npos && p + 2 <= head.size()) {
    size_t n = head.find("\r\n", p + 2);
    std::string_view line = head.substr(p + 2, n == std::string_view::npos ? std::string_view::npos : n - p - 2);
    size_t colon = line.find(':');
    if (colon != std::string_view::npos) {
      std::string_view k = line.substr(0, colon), v = line.substr(colon + 1);
      while (!v.empty() && v.front() == ' ') v.remove_prefix(1);
      if (http::iequals(k, "content-length")) cl = atol(std::string(v).c_str());
      else if (http::iequals(k, "transfer-encoding") && v.find("chunked") != std::string_view::npos) chunked = true;
    }
    p = n;
  }
  const size_t b = he + 4;
  if (chunked) {
    size_t consumed = 0;
    body->clear();
    http::Parse q = http::decode_chunked_body(in.data() + b, in.size() - b, &consumed, body);
    if (q == http::Parse::kError) return -1;
    if (q == http::Parse::kIncomplete) return 0;
    return long(b + consumed);
  }
  if (cl < 0 || cl > (256 << 20)) return -1;
  if (in.size() < b + size_t(cl)) return 0;
  body->assign(in, b, size_t(cl));
  return long(b + size_t(cl));
}

void send_all(int fd, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    ssize_t w = ::send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR || errno == EAGAIN) continue;  // small replies: the buffer has room
      return;
    }
    off += size_t(w);
  }
}

}  // namespace

int main(int argc, char** argv) {
  std::string host = "127.0.0.1", port_file, cpu_list;
  int port = 9411;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) {
        fprintf(stderr, "zipkin_sink: %s needs a value\n", a.c_str());
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--host") host = val();
    else if (a == "--port") port = atoi(val().c_str());
    else if (a == "--port-file") port_file = val();
    else if (a == "--cpu-list") cpu_list = val();
    else {
      fprintf(stderr, "usage: hola_zipkin_sink [--host H] [--port P] [--port-file F] [--cpu-list L]\n");
      return 2;
    }
  }
  signal(SIGPIPE, SIG_IGN);
  std::vector<int> cpus;
  if (!cpu_list.empty() && parse_cpu_list(cpu_list, &cpus) && !cpus.empty()) pin_current_thread(cpus[0]);
  std::string err;
  ListenOptions lo;
  lo.host = host;
  lo.port = port;
  lo.backlog = 1024;
  int lfd = listen_tcp(lo, &err);
  if (lfd < 0) {
    fprintf(stderr, "zipkin_sink: %s\n", err.c_str());
    return 1;
  }
  const int bound = bound_port(lfd);
  if (!port_file.empty()) {
    FILE* f = fopen((port_file + ".tmp").c_str(), "w");
    if (!f) return 1;
    fprintf(f, "%d\n", bound);
    fclose(f);
    rename((port_file + ".tmp").c_str(), port_file.c_str());
  }
  int ep = epoll_create1(EPOLL_CLOEXEC);
  epoll_event ev{};
  ev.events = EPOLLIN;
  ev.data.fd = lfd;
  epoll_ctl(ep, EPOLL_CTL_ADD, lfd, &ev);
  std::unordered_map<int, std::unique_ptr<Conn>> conns;
  Stats st;
  std::string method, path, body;
  epoll_event evs[64];
  char buf[65536];
  for (;;) {
    int n = epoll_wait(ep, evs, 64, -1);
    if (n < 0 && errno == EINTR) continue;
    for (int i = 0; i < n; ++i) {
      const int fd = evs[i].data.fd;
      if (fd == lfd) {
        for (;;) {
          int c = accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
          if (c < 0) break;
          set_nodelay(c);
          epoll_event e{};
          e.events = EPOLLIN;
          e.data.fd = c;
          epoll_ctl(ep, EPOLL_CTL_ADD, c, &e);
          conns[c] = std::make_unique<Conn>(Conn{c, {}});
        }
        continue;
      }
      auto it = conns.find(fd);
      if (it == conns.end()) continue;
      Conn& c = *it->second;
      bool closed = false;
      for (;;) {
        ssize_t r = ::recv(fd, buf, sizeof buf, 0);
        if (r > 0) {
          c.in.append(buf, size_t(r));
          continue;
        }
        if (r < 0 && (errno == EAGAIN || errno == EINTR)) break;
        closed = true;
        break;
      }
      for (;;) {
        long used = parse_one(c.in, &method, &path, &body);
        if (used == 0) break;
        if (used < 0) {
          ++st.bad;
          send_all(fd, "HTTP/1.1 400 Bad Request\r\nContent-Length: 0\r\nConnection: close\r\n\r\n");
          closed = true;
          break;
        }
        c.in.erase(0, size_t(used));
        if (method == "POST" && (path == "/api/v1/spans" || path == "/api/v2/spans")) {
          ++st.posts;
          st.bytes += body.size();
          st.spans += count_spans(body);
          send_all(fd, "HTTP/1.1 202 Accepted\r\nContent-Length: 0\r\n\r\n");
        } else if (method == "GET" && path == "/stats") {
          char j[256];
          int m = snprintf(j, sizeof j, "{\"posts\":%llu,\"spans\":%llu,\"bytes\":%llu,\"bad\":%llu}",
                           (unsigned long long)st.posts, (unsigned long long)st.spans,
                           (unsigned long long)st.bytes, (unsigned long long)st.bad);
          send_all(fd, "HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nContent-Length: " + std::to_string(m) +
                           "\r\n\r\n" + std::string(j, size_t(m)));
        } else {
          send_all(fd, "HTTP/1.1 404 Not Found\r\nContent-Length: 0\r\n\r\n");
        }
      }
      if (closed) {
        epoll_ctl(ep, EPOLL_CTL_DEL, fd, nullptr);
        ::close(fd);
        conns.erase(it);
      }
    }
  }
}
