#include "client/url.h"

#include <arpa/inet.h>
#include <openssl/err.h>
#include <openssl/ssl.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>

#include "core/net.h"
#include "http/parser.h"

namespace hola::client {

bool parse_url(std::string_view s, Url* out) {
  bool tls = false;
  if (s.substr(0, 8) == "https://") {
    tls = true;
    s.remove_prefix(8);
  } else if (s.substr(0, 7) == "http://") {
    s.remove_prefix(7);
  } else {
    return false;
  }
  size_t slash = s.find('/');
  std::string_view auth = s.substr(0, slash);
  std::string_view path = slash == std::string_view::npos ? std::string_view("/") : s.substr(slash);
  if (auth.empty()) return false;
  size_t at = auth.rfind('@');
  if (at != std::string_view::npos) auth.remove_prefix(at + 1);
  int port = tls ? 443 : 80;
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
  out->tls = tls;
  std::string p(path);
  size_t q = p.find_first_of("?#");
  if (q != std::string::npos) p.resize(q);
  if (p.empty() || p[0] != '/') p = "/" + p;
  if (p.back() != '/') p += '/';
  out->base_path = p;
  return true;
}

namespace {
SSL_CTX* tls_context() {
  // One client context for the process (thread-safe static init): system CA store, honouring
  // $SSL_CERT_FILE / $SSL_CERT_DIR, peer verification on, TLS 1.2 or later.
  static SSL_CTX* ctx = [] {
    SSL_CTX* c = SSL_CTX_new(TLS_client_method());
    if (c) {
      SSL_CTX_set_min_proto_version(c, TLS1_2_VERSION);
      SSL_CTX_set_default_verify_paths(c);
      SSL_CTX_set_verify(c, SSL_VERIFY_PEER, nullptr);
    }
    return c;
  }();
  return ctx;
}

bool is_ip_literal(const std::string& h) {
  unsigned char buf[16];
  return inet_pton(AF_INET, h.c_str(), buf) == 1 || inet_pton(AF_INET6, h.c_str(), buf) == 1;
}

// TLS client handshake on a connected blocking socket (its SO_RCVTIMEO/SO_SNDTIMEO bound it).
bool start_tls(BlockingConn* c, const std::string& host_in) {
  SSL_CTX* ctx = tls_context();
  if (!ctx) return false;
  SSL* ssl = SSL_new(ctx);
  if (!ssl) return false;
  c->ssl = ssl;
  std::string host = host_in;
  if (host.size() > 2 && host.front() == '[') host = host.substr(1, host.size() - 2);
  if (is_ip_literal(host)) {
    X509_VERIFY_PARAM_set1_ip_asc(SSL_get0_param(ssl), host.c_str());
  } else {
    SSL_set_tlsext_host_name(ssl, host.c_str());
    SSL_set1_host(ssl, host.c_str());
  }
  SSL_set_fd(ssl, c->fd);
  if (SSL_connect(ssl) != 1) {
    ERR_clear_error();
    return false;
  }
  return true;
}

ssize_t io_read(BlockingConn* c, char* p, size_t n) {
  if (c->ssl) {
    int r = SSL_read(static_cast<SSL*>(c->ssl), p, int(n));
    if (r <= 0) ERR_clear_error();
    return r;
  }
  return ::recv(c->fd, p, n, 0);
}

bool io_write_all(BlockingConn* c, const char* p, size_t n) {
  if (!c->ssl) return write_all(c->fd, p, n);
  while (n) {
    int w = SSL_write(static_cast<SSL*>(c->ssl), p, int(n));
    if (w <= 0) {
      ERR_clear_error();
      return false;
    }
    p += w;
    n -= size_t(w);
  }
  return true;
}

bool recv_some(BlockingConn* c, std::string* buf) {
  char tmp[16384];
  ssize_t n = io_read(c, tmp, sizeof tmp);
  if (n <= 0) return false;
  buf->append(tmp, size_t(n));
  return true;
}
}  // namespace

void BlockingConn::close() {
  if (ssl) {
    SSL_free(static_cast<SSL*>(ssl));  // no close_notify: the socket is dropped either way
    ssl = nullptr;
  }
  if (fd >= 0) ::close(fd);
  fd = -1;
}

bool read_response(BlockingConn* c, BlockingResponse* out, bool* close_delimited, bool head_request) {
  std::string buf;
  size_t head_end, start = 0;
  for (;;) {
    for (;;) {
      head_end = buf.find("\r\n\r\n", start);
      if (head_end != std::string::npos) break;
      if (buf.size() - start > 64 * 1024 || !recv_some(c, &buf)) return false;
    }
    std::string_view head(buf.data() + start, head_end - start);
    if (head.size() < 12 || head.substr(0, 5) != "HTTP/") return false;
    out->status = atoi(std::string(head.substr(9, 3)).c_str());
    // Interim responses (100 Continue, 102, 103) come before the final one, asked for or not
    // (RFC 9110 §15.2): read past them. 101 would switch protocols; there is no upgrade here.
    if (out->status >= 100 && out->status < 200 && out->status != 101) {
      start = head_end + 4;
      continue;
    }
    break;
  }
  std::string_view head(buf.data() + start, head_end - start);
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
  // Below, bytes after the response were not asked for: the connection is out of step and is
  // dropped (*close_delimited).
  // No body whatever the headers say (RFC 9110 §6.3): a response to HEAD, 1xx, 204 and 304.
  // Reading one until the peer closes would hold the caller to its timeout (a collector that
  // answers a POST with a bare 204) and leave the connection out of step.
  if (head_request || out->status == 204 || out->status == 304 || out->status < 200) {
    out->body.clear();
    if (buf.size() > body_start) *close_delimited = true;
    return true;
  }
  if (chunked) {
    std::string body;
    size_t consumed = 0;
    for (;;) {
      consumed = 0;
      body.clear();
      http::Parse p = http::decode_chunked_body(buf.data() + body_start, buf.size() - body_start, &consumed, &body);
      if (p == http::Parse::kError) return false;
      if (p == http::Parse::kOk) break;
      if (buf.size() > (1 << 20) || !recv_some(c, &buf)) return false;
    }
    out->body = std::move(body);
    if (buf.size() > body_start + consumed) *close_delimited = true;
    return true;
  }
  if (cl >= 0) {
    if (cl > (1 << 20)) return false;
    while (buf.size() - body_start < size_t(cl))
      if (!recv_some(c, &buf)) return false;
    out->body = buf.substr(body_start, size_t(cl));
    if (buf.size() > body_start + size_t(cl)) *close_delimited = true;
    return true;
  }
  // close-delimited
  *close_delimited = true;
  while (recv_some(c, &buf)) {
  }
  out->body = buf.substr(body_start);
  return true;
}

bool blocking_request(const Url& u, BlockingConn* c, const sockaddr_storage* addr, socklen_t addr_len,
                      std::string_view method, std::string_view path, std::string_view extra_headers,
                      std::string_view body, int timeout_ms, BlockingResponse* out) {
  for (int attempt = 0; attempt < 2; ++attempt) {
    bool reused = c->open();
    if (!c->open()) {
      sockaddr_storage ss{};
      socklen_t len = 0;
      if (addr) {
        if (addr_len == 0) return false;  // no address known: only a kept-alive connection will do
        ss = *addr;
        len = addr_len;
      } else if (!resolve_host(u.host, u.port, &ss, &len, nullptr)) {
        return false;
      }
      c->fd = connect_blocking(ss, len, timeout_ms);
      if (c->fd < 0) return false;
      timeval tv{timeout_ms / 1000, (timeout_ms % 1000) * 1000};
      setsockopt(c->fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof tv);
      setsockopt(c->fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof tv);
      if (u.tls && !start_tls(c, u.host)) {
        c->close();
        return false;
      }
    }
    std::string req;
    req.reserve(256 + body.size());
    req.append(method).append(" ").append(path).append(" HTTP/1.1\r\nHost: ").append(u.host);
    if (u.port != (u.tls ? 443 : 80)) req.append(":").append(std::to_string(u.port));
    req.append("\r\n").append(extra_headers);
    if (!body.empty() || method == "POST" || method == "PUT")
      req.append("Content-Length: ").append(std::to_string(body.size())).append("\r\n");
    req.append("\r\n").append(body);
    bool closed = false;
    if (io_write_all(c, req.data(), req.size()) && read_response(c, out, &closed, method == "HEAD")) {
      if (closed) c->close();
      return true;
    }
    c->close();
    if (!reused) return false;  // a stale kept-alive connection gets one retry
  }
  return false;
}

bool blocking_request(const Url& u, int* fd, std::string_view method, std::string_view path,
                      std::string_view extra_headers, std::string_view body, int timeout_ms,
                      BlockingResponse* out) {
  BlockingConn c;
  c.fd = *fd;
  Url plain = u;
  plain.tls = false;  // this form keeps no TLS session between calls
  bool ok = blocking_request(plain, &c, nullptr, 0, method, path, extra_headers, body, timeout_ms, out);
  *fd = c.fd;
  c.fd = -1;  // ownership stays with the caller
  return ok;
}

}  // namespace hola::client
