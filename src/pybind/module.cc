// hola_amd._native — Python bindings to the C++ core, used by the unit tests so they exercise
// the exact code the server runs (properties parser, String.format subset, B3 codec, Accept
// negotiation, HTTP parser, JSON codec, Hystrix state machine on a fake clock, span encoding).
#include <pybind11/pybind11.h>

#include <pybind11/stl.h>

#include <algorithm>
#include <atomic>
#include <thread>


#include "app/aloha_chainer.h"
#include "client/http_client.h"
#include "client/url.h"
#include "config/jformat.h"
#include "core/net.h"
#include "config/properties.h"
#include "config/resolver.h"
#include "http/negotiate.h"
#include "core/build_info.h"
#include "core/isa.h"
#include "http/parser.h"
#include "json/json.h"
#include "resilience/hystrix.h"
#include "tracing/b3.h"
#include "tracing/tracer.h"
#include "metrics/hystrix_stream.h"
#include "core/histogram.h"
#include "core/loop.h"
#include "core/clock.h"
#include "core/log.h"
#include "core/cpuprof.h"
#include "core/inline_function.h"
#include "core/scan.h"
#include "http/server.h"

#include <sys/socket.h>
#include <unistd.h>

namespace py = pybind11;
using namespace hola;

namespace {

py::dict parse_properties_py(py::bytes data) {
  std::string s = data;
  config::PropertiesResult r = config::parse_properties(s);
  py::dict out;
  out["ok"] = r.ok;
  out["error"] = r.error;
  py::dict m;
  for (auto& [k, v] : r.map) m[py::bytes(k)] = py::bytes(v);
  out["map"] = m;
  return out;
}

py::object java_format_py(const std::string& fmt, const std::vector<std::string>& args) {
  config::FormatResult r = config::java_format(fmt, args);
  if (r.ok) return py::bytes(r.value);
  return py::make_tuple(r.error, r.detail);
}

py::object parse_request_py(py::bytes data) {
  std::string s = data;
  http::Request r;
  int status = 0;
  http::Parse p = http::parse_request(s.data(), s.size(), &r, &status);
  if (p == http::Parse::kIncomplete) return py::str("incomplete");
  if (p == http::Parse::kError) return py::int_(status);
  py::dict d;
  d["method"] = std::string(r.method);
  d["target"] = std::string(r.target);
  d["path"] = std::string(r.path);
  d["query"] = std::string(r.query);
  d["version_minor"] = r.version_minor;
  d["keep_alive"] = r.keep_alive;
  d["has_accept"] = r.has_accept;
  d["accept"] = std::string(r.accept);
  d["host"] = std::string(r.host);
  d["content_length"] = r.content_length;
  d["chunked"] = r.chunked;
  d["head_bytes"] = r.head_bytes;
  d["b3_trace_id"] = std::string(r.b3_trace_id);
  d["b3_span_id"] = std::string(r.b3_span_id);
  d["b3_parent_id"] = std::string(r.b3_parent_id);
  d["b3_sampled"] = std::string(r.b3_sampled);
  d["b3_flags"] = std::string(r.b3_flags);
  d["b3_single"] = std::string(r.b3_single);
  return d;
}

py::object skip_chunked_py(py::bytes data) {
  std::string s = data;
  size_t n = 0;
  http::Parse p = http::skip_chunked_body(s.data(), s.size(), &n);
  if (p == http::Parse::kIncomplete) return py::str("incomplete");
  if (p == http::Parse::kError) return py::str("error");
  return py::int_(n);
}

py::object decode_chunked_py(py::bytes data) {
  std::string s = data, body;
  size_t n = 0;
  http::Parse p = http::decode_chunked_body(s.data(), s.size(), &n, &body);
  if (p == http::Parse::kIncomplete) return py::str("incomplete");
  if (p == http::Parse::kError) return py::str("error");
  return py::make_tuple(n, py::bytes(body));
}

py::object b3_extract_py(const std::string& t, const std::string& s, const std::string& p, const std::string& smp,
                         const std::string& flags, const std::string& single) {
  tracing::SpanContext c;
  tracing::Extract e = tracing::extract(t, s, p, smp, flags, single, &c);
  if (e == tracing::Extract::kNone) return py::str("none");
  if (e == tracing::Extract::kNotSampled) return py::str("not_sampled");
  py::dict d;
  d["trace_id"] = tracing::trace_id_hex(c.trace_hi, c.trace_id);
  d["span_id"] = tracing::hex64(c.span_id);
  d["parent_id"] = c.has_parent ? py::object(py::str(tracing::hex64(c.parent_id))) : py::object(py::none());
  d["sampled"] = c.sampled;
  d["debug"] = c.debug;
  return d;
}

std::string b3_inject_py(const std::string& trace_id, const std::string& span_id, py::object parent, bool sampled,
                         bool debug) {
  tracing::SpanContext c;
  tracing::parse_trace_id(trace_id, &c.trace_hi, &c.trace_id);
  tracing::parse_hex64(span_id, &c.span_id);
  if (!parent.is_none()) {
    c.has_parent = true;
    tracing::parse_hex64(parent.cast<std::string>(), &c.parent_id);
  }
  c.sampled = sampled;
  c.debug = debug;
  std::string h;
  tracing::inject(c, &h);
  return h;
}

py::object decode_string_list_py(py::bytes data) {
  std::string s = data;
  std::vector<std::optional<std::string>> out;
  std::string err;
  if (!json::decode_string_list(s, &out, &err)) return py::make_tuple("error", err);
  py::list l;
  for (auto& o : out) l.append(o ? py::object(py::bytes(*o)) : py::object(py::none()));
  return l;
}

// Decodes each document into the same vector, as the chainer does per worker; returns the
// last result (a list) or ("error", message).
py::object decode_string_list_reusing_py(const std::vector<std::string>& docs) {
  std::vector<std::optional<std::string>> out;
  std::string err;
  bool ok = true;
  for (const auto& d : docs) ok = json::decode_string_list(d, &out, &err);
  if (!ok) return py::make_tuple("error", err);
  py::list l;
  for (auto& o : out) l.append(o ? py::object(py::bytes(*o)) : py::object(py::none()));
  return l;
}

py::bytes string_array_py(const std::vector<std::optional<std::string>>& items) {
  return py::bytes(json::string_array(items));
}

// Fake-clock Hystrix command for state-machine tests.
struct PyCommand {
  FakeClock clock;
  std::unique_ptr<resilience::Command> cmd;
  PyCommand(const std::map<std::string, std::string>& props) : clock(1000000) {
    resilience::Settings s = resilience::settings_from(props, "AlohaService#aloha()", "aloha");
    cmd = std::make_unique<resilience::Command>("AlohaService#aloha()", "aloha", "aloha", s, clock);
  }
  // `ticket` >= 0 offers the call to the pool queue under that id (maxQueueSize > 0).
  std::string try_start(int64_t ticket) {
    resilience::Command::Queued q{uint64_t(ticket), 0};
    switch (cmd->try_start(ticket >= 0 ? &q : nullptr)) {
      case resilience::Command::Admit::kRun: return "run";
      case resilience::Command::Admit::kQueued: return "queued";
      case resilience::Command::Admit::kShortCircuited: return "short_circuited";
      default: return "rejected";
    }
  }
  // The ticket of the queued call that takes a released slot, or None.
  py::object next_queued() {
    resilience::Command::Queued q;
    if (!cmd->next_queued(&q)) return py::none();
    return py::int_(int64_t(q.a));
  }
  bool cancel_queued(int64_t ticket) { return cmd->cancel_queued({uint64_t(ticket), 0}); }
  void release_slot() { cmd->release_slot(); }
  void set_per_thread_bulkhead(bool on) { cmd->set_per_thread_bulkhead(on); }
  // a configuration reload (Archaius' dynamic properties): the same keys as the constructor
  void update(const std::map<std::string, std::string>& props) {
    cmd->update_settings(resilience::settings_from(props, "AlohaService#aloha()", "aloha"));
  }
  void queued_timeout(int64_t ms) { cmd->queued_timeout(ms); }
  int64_t queue_size() { return cmd->queue_size(); }
  void finish(const std::string& outcome, int64_t ms) {
    resilience::Event e = outcome == "success" ? resilience::Event::kSuccess
                          : outcome == "timeout" ? resilience::Event::kTimeout
                          : outcome == "bad_request" ? resilience::Event::kBadRequest
                                                     : resilience::Event::kFailure;
    cmd->finish(e, ms);
    if (e != resilience::Event::kSuccess) cmd->fallback(resilience::Event::kFallbackSuccess);
  }
  void advance(int64_t ms) { clock.advance(ms); }
  bool is_open() { return cmd->circuit_open(); }
  py::dict health() {
    auto h = cmd->health();
    py::dict d;
    d["total"] = h.total;
    d["errors"] = h.errors;
    d["error_pct"] = h.error_pct;
    return d;
  }
  std::string stream_json() { return metrics::HystrixStream::command_json(cmd->snapshot()); }
  py::dict transitions() {
    auto s = cmd->snapshot();
    py::dict d;
    d["opened"] = s.circuit_opened;
    d["closed_trial"] = s.circuit_closed_trial;
    d["closed_inflight"] = s.circuit_closed_inflight;
    return d;
  }
  std::string pool_json() { return metrics::HystrixStream::threadpool_json(cmd->snapshot()); }
  py::dict settings() {
    auto s = cmd->settings();
    py::dict d;
    d["timeout_ms"] = s.timeout_ms;
    d["request_volume_threshold"] = s.request_volume_threshold;
    d["error_threshold_pct"] = s.error_threshold_pct;
    d["sleep_window_ms"] = s.sleep_window_ms;
    d["pool_core_size"] = s.pool_core_size;
    d["rolling_window_ms"] = s.rolling_window_ms;
    d["health_snapshot_ms"] = s.health_snapshot_ms;
    return d;
  }
};

// Hammers one Command from `threads` C++ threads (the server's workers share one): every
// admitted call completes (failing every `fail_every`-th, 0 = never), every other call takes
// the fallback. Returns the callers' own tallies next to the Command's merged snapshot so
// tests can check the sharded counters and the atomic bulkhead add up.
py::dict hystrix_stress(int threads, int iters, int pool, int fail_every, int volume, bool loop_clock,
                        bool per_thread) {
  resilience::Settings st;
  st.pool_core_size = pool;
  st.request_volume_threshold = volume;
  st.health_snapshot_ms = loop_clock ? 500 : 0;  // as configured (500 ms), or a refresh per call
  st.sleep_window_ms = 1;
  // loop_clock: a time that stays put, as the workers' loop clock does within a pass (no
  // clock read per call: the cost of the command itself); else the system clock
  FakeClock fake;
  SystemClock sys;
  resilience::Command cmd("stress", "g", "g", st, loop_clock ? static_cast<const Clock&>(fake) : sys);
  cmd.set_per_thread_bulkhead(per_thread);
  std::atomic<int64_t> runs{0}, fails{0}, shorts{0}, rejects{0};
  std::vector<std::thread> ts;
  {
    py::gil_scoped_release nogil;
    for (int t = 0; t < threads; ++t)
      ts.emplace_back([&, t] {
        int64_t r = 0, f = 0, sc = 0, rj = 0;
        for (int i = 0; i < iters; ++i) {
          auto a = cmd.try_start();
          if (a == resilience::Command::Admit::kRun) {
            bool fail = fail_every > 0 && (i + t) % fail_every == 0;
            cmd.complete(fail ? resilience::Event::kFailure : resilience::Event::kSuccess, 1, fail, 1);
            ++r;
            f += fail;
          } else {
            cmd.rejected(0);
            (a == resilience::Command::Admit::kShortCircuited ? sc : rj) += 1;
          }
        }
        runs += r;
        fails += f;
        shorts += sc;
        rejects += rj;
      });
    for (auto& th : ts) th.join();
  }
  auto snap = cmd.snapshot();
  py::dict d, ev;
  for (int e = 0; e < resilience::kNumEvents; ++e)
    if (snap.cumulative[size_t(e)]) ev[resilience::event_name(resilience::Event(e))] = snap.cumulative[size_t(e)];
  d["runs"] = runs.load();
  d["failures"] = fails.load();
  d["short_circuited"] = shorts.load();
  d["rejected"] = rejects.load();
  d["events"] = ev;
  d["concurrent"] = snap.concurrent;
  d["largest"] = snap.pool_largest;
  d["completed"] = snap.pool_completed;
  return d;
}

std::string encode_spans_py(bool v2, const std::string& trace_id, const std::string& span_id, py::object parent,
                            const std::string& kind, int64_t start_us, int64_t end_us, const std::string& url,
                            int status, bool shared) {
  tracing::TracerOptions o;
  o.collector_url = "";
  o.ipv4 = 0x0100007f;  // 127.0.0.1
  o.port = 8080;
  tracing::Tracer t(o, 1);
  tracing::SpanRecord r{};
  tracing::parse_trace_id(trace_id, &r.trace_hi, &r.trace_id);
  tracing::parse_hex64(span_id, &r.span_id);
  r.has_parent = !parent.is_none();
  if (r.has_parent) tracing::parse_hex64(parent.cast<std::string>(), &r.parent_id);
  r.kind = kind == "client" ? tracing::Kind::kClient : tracing::Kind::kServer;
  r.start_us = start_us;
  r.end_us = end_us;
  r.status = uint16_t(status);
  r.shared = shared;
  r.method_len = 3;
  memcpy(r.method, "GET", 3);
  r.url_len = uint16_t(std::min(url.size(), tracing::kMaxUrl));
  memcpy(r.url, url.data(), r.url_len);
  r.error_len = 0;
  return v2 ? t.encode_v2({r}) : t.encode_v1({r});
}

std::vector<uint64_t> histogram_percentiles(const std::vector<uint64_t>& values, const std::vector<double>& ps) {
  hola::Histogram h;
  for (uint64_t v : values) h.add(v);
  std::vector<uint64_t> out;
  for (double p : ps) out.push_back(h.percentile(p));
  return out;
}

// Runs an EventLoop with one timer per delay (ms) plus cancellations; returns firing order.
std::vector<int> loop_timer_order(const std::vector<int>& delays, const std::vector<int>& cancel) {
  EventLoop loop;
  std::vector<int> fired;
  std::vector<EventLoop::TimerId> ids;
  for (size_t i = 0; i < delays.size(); ++i)
    ids.push_back(loop.add_timer(delays[i], [&fired, i] { fired.push_back(int(i)); }));
  for (int c : cancel) loop.cancel_timer(ids[size_t(c)]);
  int max_delay = 0;
  for (int d : delays) max_delay = std::max(max_delay, d);
  loop.add_timer(max_delay + 20, [&loop] { loop.stop(); });
  loop.post([&fired] { fired.push_back(-1); });  // cross-thread task runs first
  loop.run();
  return fired;
}

std::pair<size_t, size_t> span_ring(size_t capacity, size_t pushes) {
  tracing::SpanRing ring(capacity);
  tracing::SpanRecord r{};
  size_t ok = 0;
  for (size_t i = 0; i < pushes; ++i) {
    r.span_id = i;
    ok += ring.push(r) ? 1 : 0;
  }
  std::vector<tracing::SpanRecord> out;
  ring.drain(&out);
  for (size_t i = 0; i < out.size(); ++i)
    if (out[i].span_id != i) return {size_t(-1), 0};
  return {ok, out.size()};
}

// Logs `lines` raw lines "<tag> <thread> <i>" from each of `threads` threads (each a new
// thread, so rings of exited threads are reused across calls), then flushes; returns the
// lines dropped meanwhile (ring full).
uint64_t log_stress(int threads, int lines, const std::string& tag, bool prebuilt) {
  py::gil_scoped_release nogil;
  Logger& l = Logger::instance();
  const uint64_t d0 = l.dropped();
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t)
    ts.emplace_back([&l, t, lines, &tag, prebuilt] {
      std::string line;
      for (int i = 0; i < lines; ++i) {
        if (!prebuilt) {
          l.raw("%s %d %d", tag.c_str(), t, i);
          continue;
        }
        line = tag + " " + std::to_string(t) + " " + std::to_string(i);  // the Feign BASIC path
        l.raw_line(line);
      }
    });
  for (auto& t : ts) t.join();
  l.flush();
  return l.dropped() - d0;
}

// A handler that never returns while `hold` is set: the state of a livelocked worker (a loop
// stuck inside one connection's handler). The spin is a named, never-inlined function so a
// captured stack can be checked for it.
std::atomic<bool> g_spinning{false};
}  // namespace
// Exported (not in the anonymous namespace) so that symbolisers find its name in the module.
extern "C" __attribute__((noinline, visibility("default"))) void hola_stall_probe_spin(const std::atomic<bool>* hold) {
  g_spinning.store(true);
  while (hold->load(std::memory_order_relaxed)) __builtin_ia32_pause();
  asm volatile("" ::: "memory");  // keep a frame of its own
}
namespace {
struct SpinHandler : http::RequestHandler {
  std::atomic<bool> hold{true};
  void on_request(http::Connection& c, const http::Request& r) override {
    if (r.path == "/spin") hola_stall_probe_spin(&hold);
    static constexpr std::string_view k = "HTTP/1.1 200 OK\r\nContent-Length: 2\r\n\r\nok";
    c.send(k);
  }
};

// Server::stall_report of a worker stuck in a handler: one worker, one connection whose
// request spins in the handler; returns (report while stuck, report after release).
std::pair<std::string, std::string> stall_report_probe() {
  py::gil_scoped_release nogil;
  cpuprof::enable_capture();
  SpinHandler h;
  http::ServerOptions so;
  so.host = "127.0.0.1";
  so.port = 0;
  so.threads = 1;
  so.idle_timeout_ms = 0;
  http::Server s(so, &h);
  std::string err;
  if (!s.bind(&err)) throw std::runtime_error(err);
  s.start();
  g_spinning.store(false);
  sockaddr_storage ss{};
  socklen_t len = 0;
  if (!resolve_host("127.0.0.1", s.port(), &ss, &len, &err)) throw std::runtime_error(err);
  int fd = connect_blocking(ss, len, 2000);
  if (fd < 0) throw std::runtime_error("connect");
  static constexpr std::string_view req = "GET /spin HTTP/1.1\r\nHost: x\r\n\r\n";
  if (!write_all(fd, req.data(), req.size())) throw std::runtime_error("send");
  while (!g_spinning.load()) std::this_thread::sleep_for(std::chrono::milliseconds(1));
  std::string stuck = s.stall_report(0, true);
  h.hold.store(false);
  char buf[256];
  (void)::recv(fd, buf, sizeof buf, 0);
  // The response leaves from inside the handler: wait for the worker to finish that pass and
  // block in epoll_wait again before watching its passes.
  for (int k = 0; k < 1000 && s.activity(0).find("phase wait") == std::string::npos; ++k)
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  std::string after = s.stall_report(0, false);
  ::close(fd);
  s.shutdown(100);
  s.join();
  return {stuck, after};
}

// An event loop whose epoll descriptor is gone (closed behind its back): run() must fail fast
// (abort with a line on stderr) instead of leaving the thread. Run it in a child process.
void loop_lost_epoll_probe() {
  auto before = [] {
    std::vector<int> fds;
    for (int fd = 3; fd < 1024; ++fd) {
      char path[64], target[128];
      snprintf(path, sizeof path, "/proc/self/fd/%d", fd);
      const ssize_t n = readlink(path, target, sizeof target - 1);
      if (n > 0 && std::string_view(target, size_t(n)) == "anon_inode:[eventpoll]") fds.push_back(fd);
    }
    return fds;
  };
  const std::vector<int> old = before();
  EventLoop loop;
  for (int fd : before())
    if (std::find(old.begin(), old.end(), fd) == old.end()) ::close(fd);  // the loop's own
  loop.run();  // does not return
}

// InlineFunction: a move-only capture is destroyed exactly once, through moves, move-assignment,
// reset and destruction; calls reach the stored callable. Returns the counters.
py::dict inline_function_selftest() {
  struct Tracker {
    int* live;
    int* destroyed;
    explicit Tracker(int* l, int* d) : live(l), destroyed(d) { ++*live; }
    Tracker(Tracker&& o) noexcept : live(o.live), destroyed(o.destroyed) { ++*live; }
    Tracker(const Tracker&) = delete;
    ~Tracker() {
      --*live;
      ++*destroyed;
    }
  };
  int live = 0, destroyed = 0, calls = 0, sum = 0;
  {
    auto owned = std::make_unique<int>(7);  // move-only capture
    InlineFunction<int(int), 64> f([t = Tracker(&live, &destroyed), p = std::move(owned), &calls](int x) {
      ++calls;
      return x + *p;
    });
    sum += f(1);
    InlineFunction<int(int), 64> g(std::move(f));
    if (f) sum += 1000;  // moved-from is empty
    sum += g(2);
    InlineFunction<int(int), 64> h;
    h = std::move(g);
    sum += h(3);
    h = nullptr;  // destroys the callable
  }
  py::dict d;
  d["live"] = live;
  d["calls"] = calls;
  d["sum"] = sum;
  d["destroyed_tracked"] = destroyed > 0;
  return d;
}

}  // namespace

namespace hola::isa {
extern char g_module_isa_error[512];  // src/pybind/isa_flag.cc
}

PYBIND11_MODULE(_native, m) {
  // The module is built at the release -march: on a CPU that lacks it, fail the import with
  // the reason instead of a SIGILL later (src/core/isa.h). The check itself ran as the
  // module's first static initialiser (src/pybind/isa_flag.cc), which printed the line.
  if (isa::g_module_isa_error[0]) throw py::import_error(isa::g_module_isa_error);
  m.doc() = "hola native core (C++20) bindings";
  m.def("isa_build_level", &isa::build_level);
  m.def("build_info", [] {
    py::dict d;
    d["version"] = build_info::version();
    d["revision"] = build_info::revision();
    d["compiler"] = build_info::compiler();
    d["build_type"] = build_info::build_type();
    d["isa"] = isa::build_level();
    return d;
  });
  m.def("isa_missing_features", &isa::missing_features);
  m.def("parse_properties", &parse_properties_py, "java.util.Properties.load semantics on UTF-8 bytes");
  m.def("java_format", &java_format_py, "java.lang.String.format subset; bytes or (exception, detail)");
  m.def("java_string_hash", [](const std::string& s) { return config::java_string_hash(s); });
  m.def("parse_java_options", &config::parse_java_options);
  m.def("resolve", [](const std::vector<std::tuple<std::string, int, std::map<std::string, std::string>>>& srcs,
                      const std::string& key, const std::string& def) {
    std::vector<config::Source> v;
    for (auto& [n, o, vals] : srcs) v.push_back({n, o, vals});
    config::Resolver r(v);
    config::Resolved x = r.resolve(key, def);
    return py::make_tuple(x.value, x.source, x.key, x.found);
  });
  m.def("accepts", [](const std::string& accept, const std::string& t, const std::string& st) {
    return http::accepts(accept, t, st);
  });
  m.def("parse_request", &parse_request_py);
  m.def("remove_dot_segments", [](const std::string& p) -> py::object {
    std::string out(p.size() + 1, '\0');
    size_t n = 0;
    if (!http::remove_dot_segments(p, out.data(), &n)) return py::none();
    return py::str(out.substr(0, n));
  });
  m.def("skip_chunked_body", &skip_chunked_py);
  m.def("decode_chunked_body", &decode_chunked_py);
  m.def("b3_extract", &b3_extract_py, py::arg("trace_id") = "", py::arg("span_id") = "", py::arg("parent_id") = "",
        py::arg("sampled") = "", py::arg("flags") = "", py::arg("single") = "");
  m.def("b3_inject", &b3_inject_py, py::arg("trace_id"), py::arg("span_id"), py::arg("parent") = py::none(),
        py::arg("sampled") = true, py::arg("debug") = false);
  m.def("decode_string_list", &decode_string_list_py);
  m.def("decode_string_list_reusing", &decode_string_list_reusing_py);
  m.def("string_array", &string_array_py);
  m.def("json_quote", [](const std::string& s) { return py::bytes(json::quote(s)); });
  m.def("json_quoted_size", [](const std::string& s) { return json::quoted_size(s); });
  m.def("json_plain_string_list", [](py::bytes b) -> py::object {
    const std::string s = b;
    size_t n = 0;
    if (!json::plain_string_list(s, &n)) return py::none();
    return py::int_(n);
  });
  m.def("json_plain_prefix", [](py::bytes b) {
    const std::string s = b;
    return json_plain_prefix(s.data(), s.size());
  });
  m.def("encode_span", &encode_spans_py, py::arg("v2"), py::arg("trace_id"), py::arg("span_id"),
        py::arg("parent") = py::none(), py::arg("kind") = "server", py::arg("start_us") = 1000,
        py::arg("end_us") = 2000, py::arg("url") = "http://localhost/api/hola", py::arg("status") = 200,
        py::arg("shared") = false);
  m.def("histogram_percentiles", &histogram_percentiles);
  m.def("is_local_resource_error", &is_local_resource_error);
  m.def("parse_url", [](const std::string& s) -> py::object {
    client::Url u;
    if (!client::parse_url(s, &u)) return py::none();
    return py::make_tuple(u.host, u.port, u.base_path, u.tls);
  });
  m.def("strip_path_parameters", [](const std::string& p) {
    std::string out(p.size(), '\0');
    size_t n = 0;
    http::strip_path_parameters(p, out.data(), &n);
    out.resize(n);
    return out;
  });
  m.def("parse_retry_after", [](const std::string& v, int64_t now_ms) -> py::object {
    int64_t ms = 0;
    if (!client::parse_retry_after(v, now_ms, &ms)) return py::none();
    return py::int_(ms);
  });
  m.def("feign_backoff_ms", [](int attempt, const std::string& policy) -> py::object {
    app::RetryPolicy p;
    if (!app::parse_retry_policy(policy, &p)) return py::none();
    return py::make_tuple(p.backoff_ms(attempt), p.max_attempts);
  }, py::arg("attempt"), py::arg("policy") = "default");
  m.def("stall_report_probe", &stall_report_probe);
  m.def("inline_function_selftest", &inline_function_selftest);
  m.def("client_parse_response", [](py::bytes data, bool eof) {
    std::string in = data;
    client::ClientResult r;
    bool close = false, head_ok = false;
    size_t consumed = 0;
    const int rc = client::parse_response_probe(in, eof, &r, &close, &consumed, &head_ok);
    return py::make_tuple(rc, r.status, py::bytes(r.body), close, consumed, head_ok);
  }, py::arg("data"), py::arg("eof") = false);
  m.def("client_next_generation", [](uint32_t g) { return client::ClientPool::next_generation(g); });
  m.def("steering_within_share", [](const std::vector<int32_t>& counts, size_t w) {
    if (w >= counts.size()) throw py::index_error("worker index");
    return http::Server::steering_within_share(counts.data(), counts.size(), w);
  });
  m.def("loop_lost_epoll_probe", &loop_lost_epoll_probe);
  m.def("loop_timer_order", &loop_timer_order, py::arg("delays"), py::arg("cancel") = std::vector<int>{});
  m.def("span_ring", &span_ring);
  m.def("log_stress", &log_stress, py::arg("threads"), py::arg("lines"), py::arg("tag") = "stress",
        py::arg("prebuilt") = false);
  m.def("log_raw_line", [](const std::string& s) { Logger::instance().raw_line(s); },
        "one raw line, no flush: it reaches stderr when the writer next drains");
  m.def("hystrix_stress", &hystrix_stress, py::arg("threads"), py::arg("iters"), py::arg("pool") = 10,
        py::arg("fail_every") = 0, py::arg("volume") = 20, py::arg("loop_clock") = false,
        py::arg("per_thread") = false);
  py::class_<PyCommand>(m, "HystrixCommand")
      .def(py::init<const std::map<std::string, std::string>&>(), py::arg("props") = std::map<std::string, std::string>{})
      .def("try_start", &PyCommand::try_start, py::arg("ticket") = -1)
      .def("next_queued", &PyCommand::next_queued)
      .def("cancel_queued", &PyCommand::cancel_queued)
      .def("release_slot", &PyCommand::release_slot)
      .def("set_per_thread_bulkhead", &PyCommand::set_per_thread_bulkhead)
      .def("update", &PyCommand::update)
      .def("queued_timeout", &PyCommand::queued_timeout)
      .def("queue_size", &PyCommand::queue_size)
      .def("finish", &PyCommand::finish)
      .def("advance", &PyCommand::advance)
      .def("is_open", &PyCommand::is_open)
      .def("health", &PyCommand::health)
      .def("stream_json", &PyCommand::stream_json)
      .def("transitions", &PyCommand::transitions)
      .def("pool_json", &PyCommand::pool_json)
      .def("settings", &PyCommand::settings);
}
