#include "app/hola_app.h"

#include <charconv>

#include <cstring>
#include <deque>

#include "app/assets.h"
#include "app/chaining.h"
#include "config/jformat.h"
#include "core/clock.h"
#include "core/log.h"
#include "http/negotiate.h"
#include "json/json.h"
#include "metrics/hystrix_stream.h"
#include "metrics/prometheus.h"
#include "tracing/tracer.h"

namespace hola::app {

using http::build_response;
using http::Prepared;
using http::ResponseSpec;

namespace {
constexpr std::string_view kTextPlain = "text/plain";
constexpr std::string_view kJson = "application/json";
constexpr std::string_view kHtml = "text/html";
constexpr std::string_view kAllowApi = "Allow: HEAD, GET, OPTIONS\r\n";
// Undertow's default error pages (the servlet container answers outside JAX-RS).
constexpr std::string_view kUndertowNotFound = "<html><head><title>Error</title></head><body>Not Found</body></html>";
constexpr std::string_view kUndertowError =
    "<html><head><title>Error</title></head><body>Internal Server Error</body></html>";
constexpr std::string_view kUndertowMethodNotAllowed =
    "<html><head><title>Error</title></head><body>Method Not Allowed</body></html>";
}  // namespace

// Everything a worker needs to answer without touching shared state.
struct HolaApp::WorkerCache {
  uint64_t gen = ~0ull;
  uint64_t date_version = ~0ull;
  std::shared_ptr<const Content> content;
  // The contents of the last configuration generations, by generation, kept so that a
  // chaining call parked across a reload can still answer with the greeting of its own
  // request. The call holds the generation number, not the content (a shared_ptr copy per call
  // was two locked reference-count operations) and not its address: once a content is retired
  // past kRetired and freed, the allocator may hand the same address to the next one.
  std::deque<std::pair<uint64_t, std::shared_ptr<const Content>>> retired;
  static constexpr size_t kRetired = 8;
  // The content of generation `g`, if still kept; null once it was retired that long ago.
  const Content* alive(uint64_t g) const {
    if (g == gen) return content.get();
    for (const auto& r : retired)
      if (r.first == g) return r.second.get();
    return nullptr;
  }
  // [keep_alive][head]
  Prepared hola[2][2], health[2][2], health_unready[2][2], swagger[2][2], swagger_yaml[2][2], index[2][2], viewer[2][2];
  Prepared chaining_fallback[2][2];
  Prepared api_not_found[2], not_found[2][2], api_not_allowed[2], not_allowed[2], not_acceptable[2],
      api_options[2], static_options[2], server_error[2][2];
  std::vector<Prepared*> all;
  // Dynamic /api/hola-chaining success responses: the head up to and including
  // "Content-Length: " per keep-alive mode, and the body's `["<greeting>"` prefix.
  std::string chain_head[2];
  std::string chain_json_prefix;
};

const char* HolaApp::route_name(int r) {
  static const char* kNames[] = {"/api/hola", "/api/hola-chaining", "/api/health", "/api/swagger.json",
                                 "/", "/webjars/swagger-ui", "/hystrix.stream", "/metrics",
                                 "/api/*(404)", "*(404)", "/api/swagger.yaml"};
  return (r >= 0 && r < kNumRoutes) ? kNames[r] : "?";
}

std::shared_ptr<Content> compute_content(const config::Snapshot& snap, const AppOptions& o) {
  auto c = std::make_shared<Content>();
  c->generation = snap.generation;
  config::Resolved r = snap.resolver->resolve(o.greeting_key, o.greeting_default);
  c->translation = r.value;
  c->source = r.source;
  config::FormatResult f = config::java_format(r.value, {o.hostname});
  c->ok = f.ok;
  if (f.ok) c->greeting = std::move(f.value);
  else c->error = f.error + ": " + f.detail;
  return c;
}

HolaApp::HolaApp(AppOptions o) : o_(std::move(o)) {}
HolaApp::~HolaApp() = default;

void HolaApp::publish(std::shared_ptr<const Content> c) {
  {
    std::lock_guard<std::mutex> g(mu_);
    content_ = std::move(c);
  }
  gen_.fetch_add(1, std::memory_order_release);
}

std::shared_ptr<const Content> HolaApp::content() const {
  std::lock_guard<std::mutex> g(mu_);
  return content_;
}

void HolaApp::on_config(const config::Snapshot& snap) {
  auto c = compute_content(snap, o_);
  if (o_.log_changes && (!logged_once_ || c->translation != last_translation_)) {
    // DeltaSpike TypedResolver.logChanges(true): one INFO line per value change.
    LOG_INFO("New value %s for key %s (source %s).", c->translation.c_str(), o_.greeting_key.c_str(),
             c->source.c_str());
    last_translation_ = c->translation;
    logged_once_ = true;
  }
  if (!c->ok) LOG_WARN("greeting format failed: %s", c->error.c_str());
  publish(std::move(c));
}

HolaApp::WorkerCache& HolaApp::cache(http::Worker& w) { return *static_cast<WorkerCache*>(w.app_data); }

void HolaApp::on_worker_start(http::Worker& w) {
  auto* wc = new WorkerCache();
  w.app_data = wc;
  refresh(w, *wc);
}

void HolaApp::on_worker_stop(http::Worker& w) {
  delete static_cast<WorkerCache*>(w.app_data);
  w.app_data = nullptr;
}

void HolaApp::refresh(http::Worker& w, WorkerCache& wc) {
  uint64_t g = gen_.load(std::memory_order_acquire);
  if (g != wc.gen) {
    // A private copy per worker: one control block shared by all workers would bounce its
    // reference count between their cores on every reload.
    if (wc.content) {
      wc.retired.emplace_back(wc.gen, std::move(wc.content));
      if (wc.retired.size() > WorkerCache::kRetired) wc.retired.pop_front();
    }
    wc.gen = g;
    if (auto shared = content()) wc.content = std::make_shared<const Content>(*shared);
    else wc.content = nullptr;
    const Content* c = wc.content.get();
    const char* date = w.date();
    wc.all.clear();
    const assets::Asset* swagger = assets::find("swagger.json");
    const assets::Asset* swagger_yaml = assets::find("swagger.yaml");
    const assets::Asset* index = assets::find("index.html");
    const assets::Asset* viewer = assets::find("swagger-ui.html");
    std::string fallback_body;
    wc.chain_json_prefix.clear();
    if (c && c->ok) {
      fallback_body = json::string_array({c->greeting, std::string(kFallbackGreeting)});
      wc.chain_json_prefix = "[";
      json::append_string(&wc.chain_json_prefix, c->greeting);
      for (int ka = 0; ka < 2; ++ka) {
        ResponseSpec js;  // same spec as the generic path below, cut before the length
        js.keep_alive = ka;
        js.cors = true;
        js.content_type = kJson;
        std::string full = build_response(js, date).bytes;
        constexpr std::string_view kLen = "Content-Length: ";
        wc.chain_head[ka] = full.substr(0, full.find(kLen) + kLen.size());
      }
    }
    for (int ka = 0; ka < 2; ++ka) {
      for (int head = 0; head < 2; ++head) {
        ResponseSpec s;
        s.keep_alive = ka;
        s.head = head;
        if (c && c->ok) {
          s.status = 200;
          s.cors = true;
          s.content_type = kTextPlain;
          s.body = c->greeting;
        } else {
          s.status = 500;
          s.content_type = kHtml;
          s.body = kUndertowError;
        }
        wc.hola[ka][head] = build_response(s, date);
        ResponseSpec e = s;
        e.status = 500;
        e.cors = false;
        e.content_type = kHtml;
        e.body = kUndertowError;
        wc.server_error[ka][head] = build_response(e, date);
        if (c && c->ok) {
          ResponseSpec f = s;
          f.content_type = kJson;
          f.body = fallback_body;
          wc.chaining_fallback[ka][head] = build_response(f, date);
        } else {
          wc.chaining_fallback[ka][head] = wc.server_error[ka][head];
        }
        ResponseSpec h;
        h.keep_alive = ka;
        h.head = head;
        h.cors = true;
        h.content_type = kTextPlain;
        h.body = "I'm ok";  // HolaResource.java:85
        wc.health[ka][head] = build_response(h, date);
        ResponseSpec hu = h;  // readiness failing while the replica terminates
        hu.status = 503;
        hu.body = "shutting down";
        wc.health_unready[ka][head] = build_response(hu, date);
        ResponseSpec sw = h;
        sw.content_type = kJson;
        sw.body = swagger ? swagger->view() : std::string_view("{}");
        wc.swagger[ka][head] = build_response(sw, date);
        sw.content_type = "application/yaml";
        sw.body = swagger_yaml ? swagger_yaml->view() : std::string_view();
        wc.swagger_yaml[ka][head] = build_response(sw, date);
        ResponseSpec ix = h;
        ix.cors = false;
        ix.content_type = "text/html;charset=UTF-8";
        ix.body = index ? index->view() : std::string_view();
        wc.index[ka][head] = build_response(ix, date);
        ix.body = viewer ? viewer->view() : std::string_view();
        wc.viewer[ka][head] = build_response(ix, date);
        ResponseSpec nf;
        nf.keep_alive = ka;
        nf.head = head;
        nf.status = 404;
        nf.content_type = kHtml;
        nf.body = kUndertowNotFound;
        wc.not_found[ka][head] = build_response(nf, date);
        for (auto* p : {&wc.hola[ka][head], &wc.server_error[ka][head], &wc.chaining_fallback[ka][head],
                        &wc.health[ka][head], &wc.health_unready[ka][head], &wc.swagger[ka][head], &wc.swagger_yaml[ka][head], &wc.index[ka][head],
                        &wc.viewer[ka][head],
                        &wc.not_found[ka][head]})
          wc.all.push_back(p);
      }
      ResponseSpec s;
      s.keep_alive = ka;
      s.cors = true;
      s.status = 404;
      wc.api_not_found[ka] = build_response(s, date);
      s.status = 405;
      s.extra_headers = std::string(kAllowApi);
      wc.api_not_allowed[ka] = build_response(s, date);
      s.status = 406;
      s.extra_headers.clear();
      wc.not_acceptable[ka] = build_response(s, date);
      s.status = 200;
      s.extra_headers = std::string(kAllowApi);
      wc.api_options[ka] = build_response(s, date);
      ResponseSpec so;
      so.keep_alive = ka;
      so.status = 200;
      so.extra_headers = "Allow: GET, HEAD, OPTIONS\r\n";
      wc.static_options[ka] = build_response(so, date);
      so.status = 405;
      so.content_type = kHtml;
      so.body = kUndertowMethodNotAllowed;
      so.extra_headers = "Allow: GET, HEAD, OPTIONS\r\n";
      wc.not_allowed[ka] = build_response(so, date);
      for (auto* p : {&wc.api_not_found[ka], &wc.api_not_allowed[ka], &wc.not_acceptable[ka], &wc.api_options[ka],
                      &wc.static_options[ka], &wc.not_allowed[ka]})
        wc.all.push_back(p);
    }
    wc.date_version = w.date_version();
    return;
  }
  if (wc.date_version != w.date_version()) {
    wc.date_version = w.date_version();
    const char* d = w.date();
    for (Prepared* p : wc.all) p->set_date(d);
  }
}

std::string HolaApp::error_response(int status) {
  ResponseSpec s;
  s.status = status;
  s.keep_alive = false;
  char date[29];
  format_http_date(wall_sec_coarse(), date);
  return build_response(s, date).bytes;
}

namespace {

enum class Method { kGet, kHead, kOptions, kOther };

inline Method method_of(std::string_view m) {
  if (m.size() == 3 && m == "GET") return Method::kGet;
  if (m.size() == 4 && m == "HEAD") return Method::kHead;
  if (m.size() == 7 && m == "OPTIONS") return Method::kOptions;
  return Method::kOther;
}

inline bool path_is(std::string_view p, std::string_view route) {
  // JAX-RS matching tolerates one trailing slash.
  if (p.size() == route.size()) return p == route;
  return p.size() == route.size() + 1 && p.back() == '/' && p.substr(0, route.size()) == route;
}

int route_of(std::string_view p) {
  if (p.size() >= 4 && p.substr(0, 4) == "/api" && (p.size() == 4 || p[4] == '/')) {
    std::string_view rest = p.substr(4);
    if (path_is(rest, "/hola")) return HolaApp::kHola;
    if (path_is(rest, "/hola-chaining")) return HolaApp::kChaining;
    if (path_is(rest, "/health")) return HolaApp::kHealth;
    if (rest == "/swagger.json") return HolaApp::kSwagger;
    if (rest == "/swagger.yaml") return HolaApp::kSwaggerYaml;
    return HolaApp::kApiNotFound;
  }
  if (p == "/" || p == "/index.html") return HolaApp::kIndex;
  if (p == "/hystrix.stream") return HolaApp::kHystrix;
  if (p == "/metrics") return HolaApp::kMetrics;
  if (p == "/webjars/swagger-ui/2.1.4/" || p == "/webjars/swagger-ui/2.1.4/index.html" ||
      p == "/webjars/swagger-ui/2.1.4")
    return HolaApp::kViewer;
  return HolaApp::kNotFound;
}

// The path as Undertow and RESTEasy match it: path parameters dropped (before decoding, so
// %3B is not a delimiter), escapes decoded except %2F, dot segments removed. Each step's
// output is no longer than its input. Only paths containing ';', '%' or "/." get here.
std::string_view canonical_path(std::string_view path, std::string* storage) {
  std::string a(path.size(), '\0'), b;
  size_t n = 0;
  http::strip_path_parameters(path, a.data(), &n);
  a.resize(n);
  b.resize(a.size());
  if (http::percent_decode(a, b.data(), &n, /*keep_encoded_slash=*/true)) {
    b.resize(n);
    a.swap(b);
  }
  b.resize(a.size());
  if (http::remove_dot_segments(a, b.data(), &n)) {
    b.resize(n);
    a.swap(b);
  }
  *storage = std::move(a);
  return *storage;
}

// Whether the path needs canonical_path: one pass for ';', '%' or "/.". (A find_first_of(";%")
// plus a find("/.") cost about 195 instructions per request for "/api/hola" in libstdc++, a
// memchr call per path character: +12 % of the headline server's user-space instructions,
// found by bench/instr_ab.py over every commit since round 1, profiles/round4/11_instr.)
inline bool needs_canonical(std::string_view p) {
  // Eight bytes at a time for any ';', '%' or '.' (a word has a byte equal to c when
  // (x - 0x01..) & ~x & 0x80.. is non-zero for x = word ^ c*0x01..); only a path holding a '.'
  // takes the exact "/." pass. The byte loop was a quarter of on_request's user cycles.
  constexpr uint64_t k1 = 0x0101010101010101ull, k80 = 0x8080808080808080ull;
  auto has = [](uint64_t w, unsigned char c) {
    const uint64_t x = w ^ (k1 * c);
    return ((x - k1) & ~x & k80) != 0;
  };
  size_t i = 0;
  bool dot = false;
  for (; i + 8 <= p.size() && !dot; i += 8) {
    uint64_t w;
    memcpy(&w, p.data() + i, 8);
    if (has(w, ';') || has(w, '%')) return true;
    dot = has(w, '.');
  }
  for (; i < p.size() && !dot; ++i) {
    if (p[i] == ';' || p[i] == '%') return true;
    dot = p[i] == '.';
  }
  if (!dot) return false;
  char prev = 0;
  for (const char c : p) {
    if (c == ';' || c == '%' || (c == '.' && prev == '/')) return true;
    prev = c;
  }
  return false;
}

}  // namespace

void HolaApp::on_request(http::Connection& c, const http::Request& r) {
  http::Worker& w = c.worker();
  WorkerCache& wc = cache(w);
  if (__builtin_expect(wc.gen != gen_.load(std::memory_order_relaxed) || wc.date_version != w.date_version(), 0))
    refresh(w, wc);
  // While the server terminates or drains, every response closes its connection
  // (`Connection: close`), so kept-alive clients reconnect elsewhere between requests.
  const int ka = r.keep_alive && !w.server().closing() ? 1 : 0;
  if (!ka) c.close_after_response();

  std::string_view path = r.path;
  std::string canonical;  // stays empty (no allocation) for plain paths
  if (__builtin_expect(needs_canonical(path), 0)) path = canonical_path(path, &canonical);
  const int route = route_of(path);
  const Method m = method_of(r.method);
  const int head = m == Method::kHead ? 1 : 0;
  if (prom_) prom_->count(w.index(), route);

  switch (route) {
    case kHola:
    case kHealth:
    case kChaining:
    case kSwagger:
    case kSwaggerYaml: {
      // ZipKinFilter maps BraveServletFilter to exactly /api/hola and /api/hola-chaining for
      // every method (ZipKinFilter.java:43): OPTIONS, 405 and 406 answers get a server span,
      // while /api/hola/ (which JAX-RS still serves) does not match the servlet pattern.
      const bool traced = (route == kHola || route == kChaining) && path.back() != '/' && tracer_ &&
                          tracer_->enabled();
      auto send_traced = [&](std::string_view resp, int status) {
        if (!traced) {
          c.send_stable(resp);
          return;
        }
        tracing::ServerSpan span = tracer_->begin_server(w.index(), r);
        c.send_stable(resp);
        tracer_->end_server(w.index(), span, status);
      };
      if (m == Method::kOptions) {
        send_traced(wc.api_options[ka].view(), 200);
        return;
      }
      if (m == Method::kOther) {
        send_traced(wc.api_not_allowed[ka].view(), 405);
        return;
      }
      std::string_view subtype = route == kSwaggerYaml ? "yaml"
                                 : (route == kChaining || route == kSwagger) ? "json" : "plain";
      std::string_view type = (route == kChaining || route == kSwagger || route == kSwaggerYaml) ? "application" : "text";
      if (r.has_accept && !http::accepts(r.accept, type, subtype)) {
        send_traced(wc.not_acceptable[ka].view(), 406);
        return;
      }
      if (route == kHola) {
        if (traced) {
          tracing::ServerSpan span = tracer_->begin_server(w.index(), r);
          c.send_stable(wc.hola[ka][head].view());
          tracer_->end_server(w.index(), span, wc.content && wc.content->ok ? 200 : 500);
        } else {
          c.send_stable(wc.hola[ka][head].view());
        }
      } else if (route == kHealth) {
        // Readiness fails from the first termination signal on (--shutdown-delay-ms): the
        // Service stops routing new connections here while this replica still serves.
        c.send_stable((w.server().terminating() ? wc.health_unready : wc.health)[ka][head].view());
      } else if (route == kSwagger) {
        c.send_stable(wc.swagger[ka][head].view());
      } else if (route == kSwaggerYaml) {
        c.send_stable(wc.swagger_yaml[ka][head].view());
      } else {
        handle_chaining(c, r, wc, traced);
      }
      return;
    }
    case kApiNotFound:
      c.send_stable(wc.api_not_found[ka].view());
      return;
    case kIndex:
    case kViewer:
      if (m == Method::kOptions) c.send_stable(wc.static_options[ka].view());
      else if (m == Method::kOther) c.send_stable(wc.not_allowed[ka].view());
      else c.send_stable((route == kIndex ? wc.index : wc.viewer)[ka][head].view());
      return;
    case kHystrix:
      if (hystrix_ && m == Method::kGet) {
        hystrix_->subscribe(c, r);
      } else if (m == Method::kOther || m == Method::kOptions || !hystrix_) {
        c.send_stable(hystrix_ ? wc.not_allowed[ka].view() : wc.not_found[ka][head].view());
      } else {
        c.send_stable(wc.not_found[ka][head].view());  // HEAD on a stream: nothing to describe
      }
      return;
    case kMetrics:
      if (prom_ && o_.enable_metrics_endpoint && (m == Method::kGet || m == Method::kHead)) {
        std::string body = prom_->render(server_);
        ResponseSpec s;
        s.keep_alive = ka;
        s.head = head;
        s.content_type = "text/plain; version=0.0.4";
        s.body = body;
        c.send(build_response(s, w.date()).view());
      } else {
        c.send_stable(wc.not_found[ka][head].view());
      }
      return;
    default:
      c.send_stable(wc.not_found[ka][head].view());
      return;
  }
}

void HolaApp::handle_chaining(http::Connection& c, const http::Request& r, WorkerCache& wc, bool traced) {
  const int ka = r.keep_alive && !c.worker().server().closing() ? 1 : 0;
  const int head = r.method == "HEAD" ? 1 : 0;
  // constructed in place (no copy of its ~200 bytes)
  const tracing::ServerSpan span = traced ? tracer_->begin_server(c.worker().index(), r) : tracing::ServerSpan();
  if (!wc.content || !wc.content->ok) {
    // hola() throws before the downstream call is made (HolaResource.java:75)
    c.send_stable(wc.server_error[ka][head].view());
    if (traced) tracer_->end_server(c.worker().index(), span, 500);
    return;
  }
  // The request's latency for /metrics: from this pass's time to the time of the pass that
  // answers it (loop_now_ns(): no clock read of its own; an answer in this same pass, as a
  // short-circuit is, counts the pass's own handling time as 0)
  const int64_t t0 = loop_now_ns();
  if (!chainer_) {
    c.send_stable(wc.chaining_fallback[ka][head].view());
    if (traced) tracer_->end_server(c.worker().index(), span, 200);
    if (prom_) prom_->observe_chaining_us(c.worker().index(), uint64_t(loop_now_ns() - t0) / 1000);
    return;
  }
  // Async: the connection is parked until aloha answers, times out or is short-circuited.
  c.park();
  http::ConnRef conn(&c);  // held until the callback is gone, run or not
  const uint64_t cgen = wc.gen;  // the request's configuration (see WorkerCache::retired)
  // The continuation captures the server span only when it is recorded (a collector is
  // configured): without one end_server() does nothing, and the ~200-byte span would be
  // copied into the callback and moved into the call's slot for nothing.
  if (span.record) {
    chainer_->call(c.worker(), &span.ctx,
                   [this, conn = std::move(conn), cgen, ka, head, span, t0](const ChainResult& res) {
                     finish_chaining(conn, cgen, ka, head, &span, t0, res);
                   });
  } else {
    chainer_->call(c.worker(), traced ? &span.ctx : nullptr,
                   [this, conn = std::move(conn), cgen, ka, head, t0](const ChainResult& res) {
                     finish_chaining(conn, cgen, ka, head, nullptr, t0, res);
                   });
  }
}

// The answer to a parked /api/hola-chaining request, once aloha answered, timed out or was
// short-circuited. `conn` names the request's configuration by its generation `cgen` (a
// shared_ptr copy is two locked read-modify-writes per request, each draining the store
// buffer); `span` is the recorded server span, if any.
void HolaApp::finish_chaining(const http::ConnRef& conn, uint64_t cgen, int ka_req, int head,
                              const tracing::ServerSpan* span, int64_t t0, const ChainResult& res) {
  http::Worker& w = conn->worker();
  // termination may have begun while the call was parked
  const int ka = ka_req && !w.server().closing() ? 1 : 0;
  WorkerCache& wc = cache(w);
  bool answered = false;
  if (!conn->closed() && (res.null_list || res.error)) {
    // greetings.addAll(null) throws after a successful command, and with
    // fallbacks disabled HystrixRuntimeException escapes aloha(): a 500.
    if (wc.gen != gen_.load(std::memory_order_relaxed) || wc.date_version != w.date_version())
      refresh(w, wc);
    conn->complete(wc.server_error[ka][head].view(), ka);
    if (span) tracer_->end_server(w.index(), *span, 500);
    if (prom_) prom_->observe_chaining_us(w.index(), uint64_t(loop_now_ns() - t0) / 1000);
    return;
  }
  if (!conn->closed() && res.fallback) {
    // The prepared ["<greeting>","Aloha response (fallback)"] response, if the
    // configuration has not changed since the request arrived.
    if (wc.gen != gen_.load(std::memory_order_relaxed) || wc.date_version != w.date_version())
      refresh(w, wc);
    if (wc.gen == cgen) {
      conn->complete(wc.chaining_fallback[ka][head].view(), ka);
      answered = true;
    }
  }
  if (!answered && !conn->closed() && wc.gen == cgen && !wc.chain_json_prefix.empty()) {
    // [greeting, ...aloha] written straight into the connection's output
    // buffer, its exact length first (no intermediate copy, no insert)
    if (wc.gen != gen_.load(std::memory_order_relaxed) || wc.date_version != w.date_version())
      refresh(w, wc);
    if (wc.gen == cgen) {
      size_t body_len = wc.chain_json_prefix.size() + 1;
      if (res.raw) body_len += res.raw_count ? res.raw_list.size() - 1 : 0;  // ","+elements
      else
        for (auto& it : res.items) body_len += 1 + (it ? json::quoted_size(*it) : 4);
      char len[24];
      const size_t len_n = size_t(std::to_chars(len, len + sizeof len, body_len).ptr - len);
      std::string& out = conn->response_buffer();
      out.reserve(out.size() + wc.chain_head[ka].size() + len_n + 39 + (head ? 0 : body_len));
      out += wc.chain_head[ka];
      out.append(len, len_n);
      out += "\r\nDate: ";
      out.append(w.date(), 29);
      out += "\r\n\r\n";
      if (!head) {
        out += wc.chain_json_prefix;
        if (res.raw) {
          // aloha's elements as it wrote them: "[a,b]" goes in as ",a,b]"
          if (res.raw_count) {
            out += ',';
            out.append(res.raw_list.data() + 1, res.raw_list.size() - 1);
          } else {
            out += ']';
          }
        } else {
          for (auto& it : res.items) {
            out += ',';
            if (it) json::append_string(&out, *it);
            else out += "null";
          }
          out += ']';
        }
      }
      conn->complete_appended(ka);
      answered = true;
    }
  }
  if (!answered && !conn->closed()) {
    // the configuration changed while the call was parked: the greeting of the
    // request's own configuration (the current one if that was retired long ago)
    const Content* own = wc.alive(cgen);
    if (!own) own = wc.content.get();
    std::vector<std::optional<std::string>> items;
    items.reserve(1 + res.items.size());
    if (own) items.push_back(own->greeting);
    else items.push_back(std::nullopt);
    if (res.raw) {
      std::vector<std::optional<std::string>> aloha;
      std::string err;
      json::decode_string_list(res.raw_list, &aloha, &err);  // plain_string_list: cannot fail
      for (auto& s : aloha) items.push_back(std::move(s));
    } else {
      for (auto& s : res.items) items.push_back(s);
    }
    std::string body = json::string_array(items);
    ResponseSpec s;
    s.keep_alive = ka;
    s.head = head;
    s.cors = true;
    s.content_type = kJson;
    s.body = body;
    conn->complete(build_response(s, w.date()).view(), ka);
  }
  if (span) tracer_->end_server(w.index(), *span, 200);
  if (prom_) prom_->observe_chaining_us(w.index(), uint64_t(loop_now_ns() - t0) / 1000);
}

}  // namespace hola::app
