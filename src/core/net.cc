#include "core/net.h"

#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <ifaddrs.h>
#include <net/if.h>
#include <netdb.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <string.h>
#include <unistd.h>

namespace hola {

int listen_tcp(const ListenOptions& o, std::string* err) {
  sockaddr_storage ss{};
  socklen_t len = 0;
  if (!resolve_host(o.host, o.port, &ss, &len, err)) return -1;
  int fd = ::socket(ss.ss_family, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0) {
    if (err) *err = std::string("socket: ") + strerror(errno);
    return -1;
  }
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
  if (o.reuseport) setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof one);
  if (o.incoming_cpu >= 0) setsockopt(fd, SOL_SOCKET, SO_INCOMING_CPU, &o.incoming_cpu, sizeof o.incoming_cpu);
  // Accepted sockets inherit TCP_NODELAY from the listener on Linux; set it once here.
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  if (::bind(fd, reinterpret_cast<sockaddr*>(&ss), len) != 0) {
    if (err) *err = std::string("bind ") + o.host + ":" + std::to_string(o.port) + ": " + strerror(errno);
    ::close(fd);
    return -1;
  }
  if (::listen(fd, o.backlog) != 0) {
    if (err) *err = std::string("listen: ") + strerror(errno);
    ::close(fd);
    return -1;
  }
  return fd;
}

bool is_local_resource_error(int err) {
  return err == EMFILE || err == ENFILE || err == ENOBUFS || err == ENOMEM || err == EAGAIN || err == EADDRNOTAVAIL;
}

int bound_port(int fd) {
  sockaddr_storage ss{};
  socklen_t len = sizeof ss;
  if (getsockname(fd, reinterpret_cast<sockaddr*>(&ss), &len) != 0) return -1;
  if (ss.ss_family == AF_INET) return ntohs(reinterpret_cast<sockaddr_in*>(&ss)->sin_port);
  if (ss.ss_family == AF_INET6) return ntohs(reinterpret_cast<sockaddr_in6*>(&ss)->sin6_port);
  return -1;
}

bool resolve_host(const std::string& host_in, int port, sockaddr_storage* out, socklen_t* len,
                  std::string* err) {
  std::string host = host_in;
  if (host.size() > 2 && host.front() == '[' && host.back() == ']') host = host.substr(1, host.size() - 2);
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  hints.ai_flags = AI_NUMERICSERV;
  addrinfo* res = nullptr;
  std::string ps = std::to_string(port);
  int rc = getaddrinfo(host.empty() ? nullptr : host.c_str(), ps.c_str(), &hints, &res);
  if (rc != 0 || !res) {
    if (err) *err = "resolve " + host + ": " + gai_strerror(rc);
    return false;
  }
  // Prefer IPv4 (the demo's cluster DNS and loopback are v4).
  addrinfo* pick = res;
  for (addrinfo* p = res; p; p = p->ai_next)
    if (p->ai_family == AF_INET) { pick = p; break; }
  memcpy(out, pick->ai_addr, pick->ai_addrlen);
  *len = pick->ai_addrlen;
  freeaddrinfo(res);
  return true;
}

void set_nodelay(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
}

void set_nonblocking(int fd, bool on) {
  int fl = fcntl(fd, F_GETFL, 0);
  fcntl(fd, F_SETFL, on ? (fl | O_NONBLOCK) : (fl & ~O_NONBLOCK));
}

int connect_nonblocking(const sockaddr_storage& addr, socklen_t len, bool* in_progress) {
  int fd = ::socket(addr.ss_family, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  if (fd < 0) return -1;
  set_nodelay(fd);
  int rc = ::connect(fd, reinterpret_cast<const sockaddr*>(&addr), len);
  if (rc == 0) {
    *in_progress = false;
    return fd;
  }
  if (errno == EINPROGRESS) {
    *in_progress = true;
    return fd;
  }
  int e = errno;
  ::close(fd);
  errno = e;
  return -1;
}

int connect_blocking(const sockaddr_storage& addr, socklen_t len, int timeout_ms) {
  bool inprog = false;
  int fd = connect_nonblocking(addr, len, &inprog);
  if (fd < 0) return -1;
  if (inprog) {
    pollfd p{fd, POLLOUT, 0};
    int rc = ::poll(&p, 1, timeout_ms);
    int soerr = 0;
    socklen_t sl = sizeof soerr;
    if (rc <= 0 || getsockopt(fd, SOL_SOCKET, SO_ERROR, &soerr, &sl) != 0 || soerr != 0) {
      ::close(fd);
      errno = rc == 0 ? ETIMEDOUT : (soerr ? soerr : errno);
      return -1;
    }
  }
  set_nonblocking(fd, false);
  return fd;
}

bool write_all(int fd, const char* p, size_t n) {
  while (n) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= size_t(w);
  }
  return true;
}

std::string sockaddr_to_string(const sockaddr_storage& a) {
  char buf[INET6_ADDRSTRLEN + 16] = {0};
  if (a.ss_family == AF_INET) {
    auto* s = reinterpret_cast<const sockaddr_in*>(&a);
    inet_ntop(AF_INET, &s->sin_addr, buf, sizeof buf);
    return std::string(buf) + ":" + std::to_string(ntohs(s->sin_port));
  }
  if (a.ss_family == AF_INET6) {
    auto* s = reinterpret_cast<const sockaddr_in6*>(&a);
    inet_ntop(AF_INET6, &s->sin6_addr, buf, sizeof buf);
    return "[" + std::string(buf) + "]:" + std::to_string(ntohs(s->sin6_port));
  }
  return "?";
}

uint32_t local_ipv4() {
  ifaddrs* ifa = nullptr;
  if (getifaddrs(&ifa) != 0) return 0;
  uint32_t found = 0;
  for (ifaddrs* p = ifa; p; p = p->ifa_next) {
    if (!p->ifa_addr || p->ifa_addr->sa_family != AF_INET) continue;
    if (p->ifa_flags & IFF_LOOPBACK) continue;
    found = reinterpret_cast<sockaddr_in*>(p->ifa_addr)->sin_addr.s_addr;
    break;
  }
  freeifaddrs(ifa);
  if (!found) found = htonl(INADDR_LOOPBACK);
  return found;
}

}  // namespace hola
