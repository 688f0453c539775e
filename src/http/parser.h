// Incremental, pipelining-safe HTTP/1.1 request parser (the Undertow role).
//
// Zero-copy: every field is a string_view into the connection's receive buffer and is valid
// only until the buffer is compacted. Only the headers the service acts on are extracted;
// the rest are validated and skipped.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <string_view>

namespace hola::http {

constexpr size_t kMaxHeadBytes = 16 * 1024;
constexpr size_t kMaxRequestLine = 8 * 1024;

struct Request {
  std::string_view method;
  std::string_view target;  // raw request-target (path + optional ?query)
  std::string_view path;    // raw path part (no query), still percent-encoded
  std::string_view query;   // without '?'
  int version_minor = 1;    // HTTP/1.<minor>
  bool keep_alive = true;   // after applying Connection header + version default
  bool has_accept = false;
  std::string_view accept;
  std::string_view host;
  // B3 propagation headers (X-B3-*, and the single "b3" header).
  std::string_view b3_trace_id, b3_span_id, b3_parent_id, b3_sampled, b3_flags, b3_single;
  int64_t content_length = 0;
  bool chunked = false;
  bool expect_continue = false;  // "Expect: 100-continue"
  size_t head_bytes = 0;  // bytes of request-line + headers + terminating blank line
};

enum class Parse { kOk, kIncomplete, kError };

// Parses one request head from [buf, buf+len). On kError, *status holds the HTTP status to
// answer with (400, 414, 431, 501, 505).
Parse parse_request(const char* buf, size_t len, Request* req, int* status);

// For a chunked body starting at buf: on kOk sets *consumed to the full body length
// (including the last-chunk and trailers).
Parse skip_chunked_body(const char* buf, size_t len, size_t* consumed);
// Same framing rules, also appending the de-chunked payload to *body (clients). *body is
// meaningful only on kOk: pass a fresh string per attempt.
Parse decode_chunked_body(const char* buf, size_t len, size_t* consumed, std::string* body);

// Case-insensitive ASCII equality. Inline: callers compare against literals, so the length
// test and the loop fold into a few compares (an out-of-line call per header name cost 0.6 %
// of hola A's CPU on the chaining path).
inline bool iequals(std::string_view a, std::string_view b) {
  if (a.size() != b.size()) return false;
  for (size_t i = 0; i < a.size(); ++i) {
    const char x = a[i], y = b[i];
    if (x != y && ((x | 0x20) != (y | 0x20) || unsigned((x | 0x20) - 'a') > unsigned('z' - 'a'))) return false;
  }
  return true;
}
// Percent-decodes a path; false on malformed escapes. Output written to out (len <= in len).
// With keep_encoded_slash, "%2F" stays encoded (Undertow's default allow-encoded-slash=false),
// so an encoded slash never becomes a path separator.
bool percent_decode(std::string_view in, char* out, size_t* out_len, bool keep_encoded_slash = false);
// Removes "." and ".." segments from an absolute path (RFC 3986 §5.2.4), the way Undertow
// canonicalises the request path before servlet/JAX-RS matching; false unless `in` starts
// with '/'. Output written to out (len <= in len).
bool remove_dot_segments(std::string_view in, char* out, size_t* out_len);
// Drops path parameters (";name=value" up to the next '/') from every segment of a raw,
// still percent-encoded path, as Undertow does before servlet and JAX-RS matching
// ("/api/hola;jsessionid=x" -> "/api/hola"). Output written to out (len <= in len).
void strip_path_parameters(std::string_view in, char* out, size_t* out_len);

}  // namespace hola::http
