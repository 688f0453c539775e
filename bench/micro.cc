// hola_micro — nanosecond costs of the user-space pieces on the request path (no sockets):
// HTTP request parsing, Accept negotiation, B3 extraction, JSON encode/decode, and the
// config-time work (Properties parse + String.format) that the reference repeats per request.
#include <chrono>
#include <cstdio>
#include <string>
#include <vector>

#include "config/jformat.h"
#include "config/properties.h"
#include "http/negotiate.h"
#include "http/parser.h"
#include "json/json.h"
#include "tracing/b3.h"

using namespace hola;

template <class F>
double ns_per_op(F f, int iters = 2000000) {
  for (int i = 0; i < iters / 10; ++i) f();  // warm
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; ++i) f();
  auto t1 = std::chrono::steady_clock::now();
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

  double t_parse_min = ns_per_op([&] {
    http::Request r;
    int st;
    http::parse_request(wrk_req.data(), wrk_req.size(), &r, &st);
    sink = r.head_bytes;
  });
  double t_parse_browser = ns_per_op([&] {
    http::Request r;
    int st;
    http::parse_request(browser_req.data(), browser_req.size(), &r, &st);
    sink = r.head_bytes;
  });
  double t_accept = ns_per_op([&] {
    sink = http::accepts("text/html,application/xhtml+xml,application/xml;q=0.9,*/*;q=0.8", "text", "plain");
  });
  double t_b3 = ns_per_op([&] {
    tracing::SpanContext c;
    sink = size_t(tracing::extract("463ac35c9f6413ad", "a2fb4a1d1a96d312", "", "1", "", "", &c));
  });
  double t_json_out = ns_per_op([&] { sink = json::string_array(items).size(); }, 500000);
  double t_json_in = ns_per_op([&] {
    std::vector<std::optional<std::string>> out;
    std::string err;
    json::decode_string_list(aloha_body, &out, &err);
    sink = out.size();
  }, 500000);
  double t_props = ns_per_op([&] { sink = config::parse_properties(props).map.size(); }, 500000);
  double t_format = ns_per_op([&] { sink = config::java_format("Hola de %s", {"hola-1-abcde"}).value.size(); }, 500000);
  printf("{\"parse_wrk_request_ns\": %.1f, \"parse_browser_request_ns\": %.1f, \"accept_negotiation_ns\": %.1f, "
         "\"b3_extract_ns\": %.1f, \"json_encode_chaining_body_ns\": %.1f, \"json_decode_aloha_list_ns\": %.1f, "
         "\"properties_parse_ns\": %.1f, \"java_format_ns\": %.1f}\n",
         t_parse_min, t_parse_browser, t_accept, t_b3, t_json_out, t_json_in, t_props, t_format);
  return 0;
}
