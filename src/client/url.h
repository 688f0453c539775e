// http:// URL parsing and a small blocking HTTP/1.1 client (used off the request path: the
// Zipkin reporter thread, the load generator's sanity check and the proxy health checks).
#pragma once
#include <sys/socket.h>

#include <string>
#include <string_view>

namespace hola::client {

struct Url {
  std::string host;
  int port = 80;
  std::string base_path = "/";  // always starts and ends with '/'
};

// Accepts "http://host[:port][/path]"; false for other schemes or malformed input.
bool parse_url(std::string_view s, Url* out);

struct BlockingResponse {
  int status = 0;
  std::string headers;  // raw header block
  std::string body;
};

// Minimal blocking client over an optionally kept-alive socket (*fd, -1 to connect).
// Returns false on network error or timeout (and closes *fd).
bool blocking_request(const Url& u, int* fd, std::string_view method, std::string_view path,
                      std::string_view extra_headers, std::string_view body, int timeout_ms,
                      BlockingResponse* out);
// The same, connecting to an address resolved beforehand (e.g. by an AddressCache) when a new
// connection is needed (addr_len 0: none known, so only a kept-alive *fd can be used); u.host
// still names the Host header.
bool blocking_request(const Url& u, const sockaddr_storage& addr, socklen_t addr_len, int* fd,
                      std::string_view method, std::string_view path, std::string_view extra_headers,
                      std::string_view body, int timeout_ms, BlockingResponse* out);

// Reads one HTTP/1.1 response (Content-Length / chunked / close-delimited) from a blocking fd.
bool read_response(int fd, BlockingResponse* out, bool* close_delimited);

}  // namespace hola::client
