// Coverage-guided fuzzing of every parser that reads bytes from the network or from files
// (libFuzzer, with AddressSanitizer + UndefinedBehaviorSanitizer: `cmake --preset fuzz`,
// tests/test_fuzz_native.py). The reference's equivalents are JVM libraries (Undertow's
// request parser, HttpClient's response parser, java.util.Properties, Formatter, Jackson,
// Brave's B3 codec), memory-safe by construction; these are C++ and face the same input.
//
// One binary, one corpus: the first byte picks the parser, the rest is its input. Besides
// "no sanitizer report", each target checks invariants a correct parser keeps:
//   * the request parser's fields point into the buffer, and a prefix shorter than a parsed
//     head is incomplete, never an error or a different request;
//   * the chunked skipper and decoder agree on every input;
//   * the client's response parser consumes no more than it was given, and a complete
//     response's prefixes need more;
//   * path decoders never write past their input's length;
//   * a decoded JSON list re-encodes to a document that decodes to the same list.
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <optional>
#include <string>
#include <string_view>
#include <vector>

#include "client/http_client.h"
#include "client/url.h"
#include "config/jformat.h"
#include "config/properties.h"
#include "config/resolver.h"
#include "http/negotiate.h"
#include "http/parser.h"
#include "core/scan.h"
#include "json/json.h"
#include "tracing/b3.h"

using namespace hola;

namespace {

// Names the failed check by its line.
#define FUZZ_CHECK(cond)                                                           \
  do {                                                                             \
    if (!(cond)) {                                                                 \
      fprintf(stderr, "fuzz invariant failed: fuzz_parsers.cc:%d\n", __LINE__);    \
      abort();                                                                     \
    }                                                                              \
  } while (0)

// Parts of `s` split at `sep` (at most n; the last takes the rest).
std::vector<std::string_view> split(std::string_view s, char sep, size_t n) {
  std::vector<std::string_view> out;
  while (out.size() + 1 < n) {
    const size_t k = s.find(sep);
    if (k == std::string_view::npos) break;
    out.push_back(s.substr(0, k));
    s.remove_prefix(k + 1);
  }
  out.push_back(s);
  while (out.size() < n) out.emplace_back();
  return out;
}

bool inside(std::string_view v, const char* b, size_t n) {
  return v.empty() || (v.data() >= b && v.data() + v.size() <= b + n);
}

// The input in a heap block of exactly its size, so any read past it is an ASan report.
std::unique_ptr<char[]> exact_copy(std::string_view s) {
  std::unique_ptr<char[]> p(new char[s.size() ? s.size() : 1]);
  if (!s.empty()) memcpy(p.get(), s.data(), s.size());
  return p;
}

void request(std::string_view in) {
  auto buf = exact_copy(in);
  const char* b = buf.get();
  const size_t n = in.size();
  http::Request req;
  int status = 0;
  const http::Parse p = http::parse_request(b, n, &req, &status);
  if (p == http::Parse::kError) {
    FUZZ_CHECK(status >= 400 && status < 600);
    return;
  }
  if (p != http::Parse::kOk) return;
  FUZZ_CHECK(req.head_bytes > 0 && req.head_bytes <= n);
  for (std::string_view v : {req.method, req.target, req.query, req.accept, req.host, req.b3_trace_id,
                             req.b3_span_id, req.b3_parent_id, req.b3_sampled, req.b3_flags, req.b3_single})
    FUZZ_CHECK(inside(v, b, req.head_bytes));
  // an absolute-form target with an empty path ("http://h") routes as "/", a static string
  FUZZ_CHECK(inside(req.path, b, req.head_bytes) || req.path == "/");
  // a shorter prefix of a head that parses is incomplete
  for (size_t cut : {req.head_bytes - 1, req.head_bytes / 2, size_t(1)}) {
    if (cut >= req.head_bytes) continue;
    auto pre = exact_copy(in.substr(0, cut));
    http::Request r2;
    int st2 = 0;
    FUZZ_CHECK(http::parse_request(pre.get(), cut, &r2, &st2) == http::Parse::kIncomplete);
  }
  if (req.chunked) {
    size_t c1 = 0, c2 = 0;
    std::string body;
    const http::Parse a = http::skip_chunked_body(b + req.head_bytes, n - req.head_bytes, &c1);
    const http::Parse d = http::decode_chunked_body(b + req.head_bytes, n - req.head_bytes, &c2, &body);
    FUZZ_CHECK(a == d);
    if (a == http::Parse::kOk) FUZZ_CHECK(c1 == c2 && c1 <= n - req.head_bytes && body.size() <= c1);
  }
  // the path helpers on the parsed target
  std::string out(req.path.size(), '\0');
  size_t len = 0;
  if (http::percent_decode(req.path, out.data(), &len, true)) FUZZ_CHECK(len <= req.path.size());
}

void chunked(std::string_view in) {
  auto buf = exact_copy(in);
  size_t c1 = 0, c2 = 0;
  std::string body;
  const http::Parse a = http::skip_chunked_body(buf.get(), in.size(), &c1);
  const http::Parse d = http::decode_chunked_body(buf.get(), in.size(), &c2, &body);
  FUZZ_CHECK(a == d);
  if (a == http::Parse::kOk) FUZZ_CHECK(c1 == c2 && c1 <= in.size() && body.size() <= c1);
}

void response(std::string_view in, bool eof) {
  auto buf = exact_copy(in);
  std::string_view v(buf.get(), in.size());
  client::ClientResult r;
  bool close = false, head_ok = false;
  size_t consumed = 0;
  const int rc = client::parse_response_probe(v, eof, &r, &close, &consumed, &head_ok);
  FUZZ_CHECK(rc >= -1 && rc <= 1);
  if (rc != 1) return;
  FUZZ_CHECK(consumed > 0 && consumed <= in.size() && head_ok && r.status >= 100);
  FUZZ_CHECK(r.body.size() <= consumed);
  if (eof) return;
  for (size_t cut : {consumed - 1, consumed / 2}) {
    if (cut == 0 || cut >= consumed) continue;
    auto pre = exact_copy(in.substr(0, cut));
    client::ClientResult r2;
    bool c2 = false, h2 = false;
    size_t used = 0;
    FUZZ_CHECK(client::parse_response_probe(std::string_view(pre.get(), cut), false, &r2, &c2, &used, &h2) == 0);
  }
}

void paths(std::string_view in) {
  auto buf = exact_copy(in);
  std::string_view v(buf.get(), in.size());
  std::unique_ptr<char[]> out(new char[in.size() + 1]);
  size_t len = 0;
  for (bool keep : {false, true})
    if (http::percent_decode(v, out.get(), &len, keep)) FUZZ_CHECK(len <= in.size());
  if (http::remove_dot_segments(v, out.get(), &len)) FUZZ_CHECK(len <= in.size());
  http::strip_path_parameters(v, out.get(), &len);
  FUZZ_CHECK(len <= in.size());
}

void json_list(std::string_view in) {
  std::vector<std::optional<std::string>> list;
  std::string err;
  if (json::decode_string_list(in, &list, &err)) {
    const std::string again = json::string_array(list);
    std::vector<std::optional<std::string>> list2;
    const bool ok2 = json::decode_string_list(again, &list2, &err);
    if (!ok2) fprintf(stderr, "re-encoded list does not decode (%s): %s\n", err.c_str(), again.c_str());
    FUZZ_CHECK(ok2);
    FUZZ_CHECK(list == list2);
    // passed on as written (json::plain_string_list) exactly when re-encoding gives the input
    // back, with the element count it reports
    size_t count = 0;
    const bool plain = json::plain_string_list(in, &count);
    // (an element that needed escaping was escaped in the input: that input is not plain even
    // when it re-encodes to itself)
    const bool all_plain = std::all_of(list.begin(), list.end(), [](const auto& e) {
      return e && json_plain_prefix(e->data(), e->size()) == e->size();
    });
    FUZZ_CHECK(plain == (again == in && all_plain));
    if (plain) FUZZ_CHECK(count == list.size());
  } else {
    size_t count = 0;
    FUZZ_CHECK(!json::plain_string_list(in, &count));  // what fails to decode is never passed on
  }
  {
    // the plain-prefix scan against its byte loop, and the encoder's size against its output
    size_t want = 0;
    while (want < in.size() && (unsigned char)in[want] >= 0x20 && in[want] != '"' && in[want] != '\\') ++want;
    FUZZ_CHECK(json_plain_prefix(in.data(), in.size()) == want);
    std::string q;
    json::append_string(&q, in);
    FUZZ_CHECK(json::quoted_size(in) == q.size());
  }
  json::Value val;
  (void)json::parse(in, &val, &err);
}

void text_formats(std::string_view in) {
  (void)config::parse_properties(in);
  const auto parts = split(in, '\0', 3);
  (void)config::java_format(parts[0], {std::string(parts[1]), std::string(parts[2])});
  (void)config::java_format(parts[0], {});
  (void)config::parse_java_options(std::string(in));
  (void)config::java_string_hash(in);
}

void headers_misc(std::string_view in) {
  const auto f = split(in, '\n', 6);
  tracing::SpanContext ctx;
  if (tracing::extract(f[0], f[1], f[2], f[3], f[4], f[5], &ctx) == tracing::Extract::kContext) {
    std::string h;
    tracing::inject(ctx, &h);
    FUZZ_CHECK(!h.empty());
  }
  (void)http::accepts(in, "text", "plain");
  (void)http::accepts(in, "application", "json");
  client::Url u;
  (void)client::parse_url(in, &u);
  int64_t ms = 0;
  (void)client::parse_retry_after(in, 1700000000000, &ms);
}

}  // namespace

extern "C" int LLVMFuzzerTestOneInput(const uint8_t* data, size_t size) {
  if (size == 0) return 0;
  const std::string_view in(reinterpret_cast<const char*>(data) + 1, size - 1);
  switch (data[0] % 9) {
    case 0: request(in); break;
    case 1: chunked(in); break;
    case 2: response(in, false); break;
    case 3: response(in, true); break;
    case 4: paths(in); break;
    case 5: json_list(in); break;
    case 6: text_formats(in); break;
    case 7: headers_misc(in); break;
    case 8: request(in); response(in, false); break;  // one input, both directions
  }
  return 0;
}
