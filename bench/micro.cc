// hola_micro — nanosecond costs of the user-space pieces on the request path (no sockets):
// HTTP request parsing, Accept negotiation, B3 extraction, JSON encode/decode, and the
// config-time work (Properties parse + String.format) that the reference repeats per request.
#include <linux/perf_event.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "config/jformat.h"
#include "config/properties.h"
#include "http/negotiate.h"
#include "http/parser.h"
#include "json/json.h"
#include "tracing/b3.h"

using namespace hola;

// User-space instructions retired by this thread (hardware counter; -1 where the host has no
// PMU, e.g. a VM): deterministic, unlike the nanoseconds on a shared host.
int g_instr_fd = -2;
int64_t instructions() {
  if (g_instr_fd == -2) {
    perf_event_attr a;
    memset(&a, 0, sizeof a);
    a.type = PERF_TYPE_HARDWARE;
    a.size = sizeof a;
    a.config = PERF_COUNT_HW_INSTRUCTIONS;
    a.exclude_kernel = 1;
    a.exclude_hv = 1;
    g_instr_fd = int(syscall(SYS_perf_event_open, &a, 0, -1, -1, 0));
  }
  uint64_t v = 0;
  if (g_instr_fd < 0 || read(g_instr_fd, &v, sizeof v) != ssize_t(sizeof v)) return -1;
  return int64_t(v);
}

std::string g_instr_json;  // "name_instr": per-op instructions, appended by ns_per_op

template <class F>
double ns_per_op(const char* name, F f, int iters = 2000000) {
  for (int i = 0; i < iters / 10; ++i) f();  // warm
  const int64_t i0 = instructions();
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; ++i) f();
  auto t1 = std::chrono::steady_clock::now();
  const int64_t i1 = instructions();
  char buf[96];
  if (i0 >= 0 && i1 >= 0) snprintf(buf, sizeof buf, ", \"%s_instr\": %.1f", name, double(i1 - i0) / iters);
  else snprintf(buf, sizeof buf, ", \"%s_instr\": null", name);
  g_instr_json += buf;
  return std::chrono::duration<double, std::nano>(t1 - t0).count() / iters;
}

static volatile size_t sink;

int main() {
  const std::string wrk_req = "GET /api/hola HTTP/1.1\r\nHost: 127.0.0.1:8080\r\n\r\n";
  const std::string browser_req =
      "GET /api/hola HTTP/1.1\r\nHost: hola-msa.apps.example.com\r\nUser-Agent: Mozilla/5.0 (X11; Linux x86_64)\r\n"
      "Accept: text/html,application/xhtml+xml,application/xml;q=0.9,*/*;q=0.8\r\nAccept-Language: es-ES,es;q=0.9\r\n"
      "Accept-Encoding: gzip, deflate\r\nConnection: keep-alive\r\nX-B3-TraceId: 463ac35c9f6413ad\r\n"
      "X-B3-SpanId: a2fb4a1d1a96d312\r\nX-B3-Sampled: 1\r\n\r\n";
  const std::string props = "# comment\nhello=Hola de %s mediante el archivo de configuraciones\\n\n";
  std::vector<std::optional<std::string>> items = {std::string("Hola de h"), std::string("Aloha response (fallback)")};
  const std::string aloha_body = "[\"Aloha mai aloha-1\",\"Bonjour de bonjour-1\",\"Ola de ola-1\"]";

  double t_parse_min = ns_per_op("parse_wrk_request", [&] {
    http::Request r;
    int st;
    http::parse_request(wrk_req.data(), wrk_req.size(), &r, &st);
    sink = r.head_bytes;
  });
  // (components of the wrk-style parse, for the instruction counts: an empty request head, a
  // 32-character longer path, one more header, and the Request reset alone)
  const std::string minimal_req = "GET / HTTP/1.1\r\n\r\n";
  const std::string long_req = "GET /api/hola/0123456789abcdef0123456789abcdef HTTP/1.1\r\nHost: 127.0.0.1:8080\r\n\r\n";
  const std::string two_hdr_req = "GET /api/hola HTTP/1.1\r\nHost: 127.0.0.1:8080\r\nAccept: */*\r\n\r\n";
  http::Request kept;
  int kept_st;
  ns_per_op("parse_minimal", [&] {
    http::parse_request(minimal_req.data(), minimal_req.size(), &kept, &kept_st);
    sink = kept.head_bytes;
  });
  ns_per_op("parse_wrk_reused_request", [&] {
    http::parse_request(wrk_req.data(), wrk_req.size(), &kept, &kept_st);
    sink = kept.head_bytes;
  });
  ns_per_op("parse_path_plus_32", [&] {
    http::parse_request(long_req.data(), long_req.size(), &kept, &kept_st);
    sink = kept.head_bytes;
  });
  ns_per_op("parse_one_more_header", [&] {
    http::parse_request(two_hdr_req.data(), two_hdr_req.size(), &kept, &kept_st);
    sink = kept.head_bytes;
  });
  ns_per_op("memchr_46", [&] {
    sink = size_t(static_cast<const char*>(memchr(wrk_req.data() + sink % 2, '\n', wrk_req.size() - 2)) - wrk_req.data());
  });
  double t_parse_browser = ns_per_op("parse_browser_request", [&] {
    http::Request r;
    int st;
    http::parse_request(browser_req.data(), browser_req.size(), &r, &st);
    sink = r.head_bytes;
  });
  double t_accept = ns_per_op("accept_negotiation", [&] {
    sink = http::accepts("text/html,application/xhtml+xml,application/xml;q=0.9,*/*;q=0.8", "text", "plain");
  });
  double t_b3 = ns_per_op("b3_extract", [&] {
    tracing::SpanContext c;
    sink = size_t(tracing::extract("463ac35c9f6413ad", "a2fb4a1d1a96d312", "", "1", "", "", &c));
  });
  double t_json_out = ns_per_op("json_encode_chaining_body", [&] { sink = json::string_array(items).size(); }, 500000);
  double t_json_in = ns_per_op("json_decode_aloha_list", [&] {
    std::vector<std::optional<std::string>> out;
    std::string err;
    json::decode_string_list(aloha_body, &out, &err);
    sink = out.size();
  }, 500000);
  double t_props = ns_per_op("properties_parse", [&] { sink = config::parse_properties(props).map.size(); }, 500000);
  double t_format = ns_per_op("java_format", [&] { sink = config::java_format("Hola de %s", {"hola-1-abcde"}).value.size(); }, 500000);
  printf("{\"parse_wrk_request_ns\": %.1f, \"parse_browser_request_ns\": %.1f, \"accept_negotiation_ns\": %.1f, "
         "\"b3_extract_ns\": %.1f, \"json_encode_chaining_body_ns\": %.1f, \"json_decode_aloha_list_ns\": %.1f, "
         "\"properties_parse_ns\": %.1f, \"java_format_ns\": %.1f%s}\n",
         t_parse_min, t_parse_browser, t_accept, t_b3, t_json_out, t_json_in, t_props, t_format, g_instr_json.c_str());
  return 0;
}
