// http:// and https:// URL parsing and a small blocking HTTP/1.1 client, over TCP or TLS
// (used off the request path: the Zipkin reporter thread and the proxy health checks).
#pragma once
#include <sys/socket.h>

#include <string>
#include <string_view>

namespace hola::client {

struct Url {
  std::string host;
  int port = 80;
  std::string base_path = "/";  // always starts and ends with '/'
  bool tls = false;             // https://
};

// Accepts "http://host[:port][/path]" and "https://..." (port 443 by default); false for other
// schemes or malformed input.
bool parse_url(std::string_view s, Url* out);

struct BlockingResponse {
  int status = 0;
  std::string headers;  // raw header block
  std::string body;
};

// A kept-alive connection of the blocking client: a TCP socket, plus the TLS session over it
// for https:// (server certificate verified against the system CA store, or $SSL_CERT_FILE /
// $SSL_CERT_DIR, and against the URL's host name).
struct BlockingConn {
  int fd = -1;
  void* ssl = nullptr;  // SSL*
  BlockingConn() = default;
  BlockingConn(const BlockingConn&) = delete;
  BlockingConn& operator=(const BlockingConn&) = delete;
  ~BlockingConn() { close(); }
  bool open() const { return fd >= 0; }
  void close();
};

// One request on `c` (connected first if needed, to `addr` when given with a non-zero length,
// else to u.host resolved here; with a zero-length `addr` only an open `c` can be used).
// Returns false on a network, TLS or protocol error or timeout, and closes `c`.
bool blocking_request(const Url& u, BlockingConn* c, const sockaddr_storage* addr, socklen_t addr_len,
                      std::string_view method, std::string_view path, std::string_view extra_headers,
                      std::string_view body, int timeout_ms, BlockingResponse* out);

// Plain-TCP form over an optionally kept-alive socket (*fd, -1 to connect).
// Returns false on network error or timeout (and closes *fd).
bool blocking_request(const Url& u, int* fd, std::string_view method, std::string_view path,
                      std::string_view extra_headers, std::string_view body, int timeout_ms,
                      BlockingResponse* out);
// Reads one HTTP/1.1 response (Content-Length / chunked / close-delimited) from a blocking
// connection.
bool read_response(BlockingConn* c, BlockingResponse* out, bool* close_delimited, bool head_request = false);

}  // namespace hola::client
