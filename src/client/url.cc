#include "client/url.h"

#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>

#include "core/net.h"
#include "http/parser.h"

namespace hola::client {

bool parse_url(std::string_view s, Url* out) {
  if (s.substr(0, 7) != "http://") return false;
  s.remove_prefix(7);
  size_t slash = s.find('/');
  std::string_view auth = s.substr(0, slash);
  std::string_view path = slash == std::string_view::npos ? std::string_view("/") : s.substr(slash);
  if (auth.empty()) return false;
  size_t at = auth.rfind('@');
  if (at != std::string_view::npos) auth.remove_prefix(at + 1);
  int port = 80;
  std::string_view host = auth;
  if (!auth.empty() && auth[0] == '[') {
    size_t rb = auth.find(']');
    if (rb == std::string_view::npos) return false;
    host = auth.substr(0, rb + 1);
    if (rb + 1 < auth.size()) {
      if (auth[rb + 1] != ':') return false;
      port = atoi(std::string(auth.substr(rb + 2)).c_str());
    }
  } else {
    size_t colon = auth.rfind(':');
    if (colon != std::string_view::npos) {
      host = auth.substr(0, colon);
      std::string ps(auth.substr(colon + 1));
      if (ps.empty()) return false;
      for (char c : ps)
        if (c < '0' || c > '9') return false;
      port = atoi(ps.c_str());
    }
  }
  if (host.empty() || port <= 0 || port > 65535) return false;
  out->host = std::string(host);
  out->port = port;
  std::string p(path);
  size_t q = p.find_first_of("?#");
  if (q != std::string::npos) p.resize(q);
  if (p.empty() || p[0] != '/') p = "/" + p;
  if (p.back() != '/') p += '/';
  out->base_path = p;
  return true;
}

namespace {
bool recv_some(int fd, std::string* buf) {
  char tmp[16384];
  ssize_t n = ::recv(fd, tmp, sizeof tmp, 0);
  if (n <= 0) return false;
  buf->append(tmp, size_t(n));
  return true;
}
}  // namespace

bool read_response(int fd, BlockingResponse* out, bool* close_delimited) {
  std::string buf;
  size_t head_end;
  for (;;) {
    head_end = buf.find("\r\n\r\n");
    if (head_end != std::string::npos) break;
    if (buf.size() > 64 * 1024 || !recv_some(fd, &buf)) return false;
  }
  std::string_view head(buf.data(), head_end);
  if (head.size() < 12 || head.substr(0, 5) != "HTTP/") return false;
  out->status = atoi(std::string(head.substr(9, 3)).c_str());
  out->headers = std::string(head);
  int64_t cl = -1;
  bool chunked = false, conn_close = false;
  size_t pos = head.find("\r\n");
  while (pos != std::string_view::npos && pos < head.size()) {
    size_t next = head.find("\r\n", pos + 2);
    std::string_view line = head.substr(pos + 2, next == std::string_view::npos ? std::string_view::npos : next - pos - 2);
    size_t colon = line.find(':');
    if (colon != std::string_view::npos) {
      std::string_view name = line.substr(0, colon), val = line.substr(colon + 1);
      while (!val.empty() && val.front() == ' ') val.remove_prefix(1);
      if (http::iequals(name, "content-length")) cl = atoll(std::string(val).c_str());
      else if (http::iequals(name, "transfer-encoding") && val.find("chunked") != std::string_view::npos) chunked = true;
      else if (http::iequals(name, "connection") && http::iequals(val, "close")) conn_close = true;
    }
    pos = next;
  }
  size_t body_start = head_end + 4;
  *close_delimited = conn_close;
  if (chunked) {
    std::string body;
    for (;;) {
      size_t consumed = 0;
      body.clear();
      http::Parse p = http::decode_chunked_body(buf.data() + body_start, buf.size() - body_start, &consumed, &body);
      if (p == http::Parse::kError) return false;
      if (p == http::Parse::kOk) break;
      if (buf.size() > (1 << 20) || !recv_some(fd, &buf)) return false;
    }
    out->body = std::move(body);
    return true;
  }
  if (cl >= 0) {
    if (cl > (1 << 20)) return false;
    while (buf.size() - body_start < size_t(cl))
      if (!recv_some(fd, &buf)) return false;
    out->body = buf.substr(body_start, size_t(cl));
    return true;
  }
  // close-delimited
  *close_delimited = true;
  while (recv_some(fd, &buf)) {
  }
  out->body = buf.substr(body_start);
  return true;
}

namespace {
bool request_on(const Url& u, const sockaddr_storage* addr, socklen_t addr_len, int* fd, std::string_view method,
                std::string_view path, std::string_view extra_headers, std::string_view body, int timeout_ms,
                BlockingResponse* out) {
  for (int attempt = 0; attempt < 2; ++attempt) {
    bool reused = *fd >= 0;
    if (*fd < 0) {
      sockaddr_storage ss{};
      socklen_t len = 0;
      if (addr) {
        if (addr_len == 0) return false;  // no address known: only a kept-alive socket will do
        ss = *addr;
        len = addr_len;
      } else if (!resolve_host(u.host, u.port, &ss, &len, nullptr)) {
        return false;
      }
      *fd = connect_blocking(ss, len, timeout_ms);
      if (*fd < 0) return false;
      timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
      setsockopt(*fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
      setsockopt(*fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
    }
    std::string req;
    req.reserve(256 + body.size());
    req.append(method).append(" ").append(path).append(" HTTP/1.1\r\nHost: ").append(u.host);
    if (u.port != 80) req.append(":").append(std::to_string(u.port));
    req.append("\r\n").append(extra_headers);
    if (!body.empty() || method == "POST" || method == "PUT")
      req.append("Content-Length: ").append(std::to_string(body.size())).append("\r\n");
    req.append("\r\n").append(body);
    bool closed = false;
    if (write_all(*fd, req.data(), req.size()) && read_response(*fd, out, &closed)) {
      if (closed) {
        ::close(*fd);
        *fd = -1;
      }
      return true;
    }
    ::close(*fd);
    *fd = -1;
    if (!reused) return false;  // a stale kept-alive socket gets one retry
  }
  return false;
}
}  // namespace

bool blocking_request(const Url& u, int* fd, std::string_view method, std::string_view path,
                      std::string_view extra_headers, std::string_view body, int timeout_ms,
                      BlockingResponse* out) {
  return request_on(u, nullptr, 0, fd, method, path, extra_headers, body, timeout_ms, out);
}

bool blocking_request(const Url& u, const sockaddr_storage& addr, socklen_t addr_len, int* fd,
                      std::string_view method, std::string_view path, std::string_view extra_headers,
                      std::string_view body, int timeout_ms, BlockingResponse* out) {
  return request_on(u, &addr, addr_len, fd, method, path, extra_headers, body, timeout_ms, out);
}

}  // namespace hola::client
