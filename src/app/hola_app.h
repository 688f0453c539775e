// The hola application: routes, handlers and the per-worker prepared-response cache.
//
// Reference parity:
//   GET  /api/hola          HolaResource.hola()          HolaResource.java:52-67  (traced)
//   GET  /api/hola-chaining HolaResource.holaChaining()  HolaResource.java:69-78  (traced)
//   GET  /api/health        HolaResource.health()        HolaResource.java:80-86  (not traced)
//   GET  /api/swagger.json  SwaggerListener              SwaggerListener.java:29-42
//   GET  /hystrix.stream    HystrixServlet               HystrixServlet.java:13-17
//   GET  /                  index.html                   src/main/webapp/index.html
// `/api` is the JAX-RS application root (JaxRsActivator.java:30); every response under it
// carries `Access-Control-Allow-Origin: *` (CorsFilter.java:29-32).
#pragma once
#include <atomic>
#include <memory>
#include <mutex>
#include <string>

#include "config/manager.h"
#include "http/response.h"
#include "http/server.h"

namespace hola::tracing {
class Tracer;
struct ServerSpan;
}
namespace hola::metrics {
class HystrixStream;
class Prometheus;
}

namespace hola::app {

class Chainer;
struct ChainResult;

struct AppOptions {
  std::string hostname = "unknown";  // $HOSTNAME (HolaResource.java:57)
  std::string greeting_key = "hello";
  std::string greeting_default = "Hola de %s";  // HolaResource.java:60
  bool log_changes = true;                      // HolaResource.java:61
  bool enable_metrics_endpoint = true;          // extra: Prometheus text at /metrics
};

// Immutable state derived from one configuration snapshot.
struct Content {
  uint64_t generation = 0;
  bool ok = true;             // greeting formatted without a Formatter exception
  std::string greeting;       // String.format(translation, hostname)
  std::string translation;    // the resolved pattern
  std::string source;         // config source that supplied it
  std::string error;          // Java exception name when !ok
};

// Computes the greeting for a snapshot (resolver walk + Java String.format).
std::shared_ptr<Content> compute_content(const config::Snapshot& snap, const AppOptions& o);

class HolaApp final : public http::RequestHandler {
 public:
  explicit HolaApp(AppOptions o);
  ~HolaApp() override;

  // Thread-safe: publish new content (called from the config watcher thread).
  void publish(std::shared_ptr<const Content> c);
  std::shared_ptr<const Content> content() const;
  // Config listener: recompute content and log the change (DeltaSpike logChanges).
  void on_config(const config::Snapshot& snap);

  void set_server(http::Server* s) { server_ = s; }
  void set_chainer(Chainer* c) { chainer_ = c; }
  void set_tracer(tracing::Tracer* t) { tracer_ = t; }
  void set_hystrix_stream(metrics::HystrixStream* h) { hystrix_ = h; }
  void set_prometheus(metrics::Prometheus* p) { prom_ = p; }
  const AppOptions& options() const { return o_; }

  void on_request(http::Connection& c, const http::Request& r) override;
  void on_worker_start(http::Worker& w) override;
  void on_worker_stop(http::Worker& w) override;
  std::string error_response(int status) override;

  // Route ids (also used for per-route metrics).
  enum Route : int {
    kHola = 0, kChaining, kHealth, kSwagger, kIndex, kViewer, kHystrix, kMetrics,
    kApiNotFound, kNotFound, kSwaggerYaml, kNumRoutes
  };
  static const char* route_name(int r);

 private:
  struct WorkerCache;
  WorkerCache& cache(http::Worker& w);
  void refresh(http::Worker& w, WorkerCache& wc);
  // `traced`: the request matched ZipKinFilter's servlet pattern (server span around it).
  void handle_chaining(http::Connection& c, const http::Request& r, WorkerCache& wc, bool traced);
  void finish_chaining(const http::ConnRef& conn, uint64_t cgen, int ka_req, int head, const tracing::ServerSpan* span,
                       int64_t t0, const ChainResult& res);

  AppOptions o_;
  http::Server* server_ = nullptr;
  Chainer* chainer_ = nullptr;
  tracing::Tracer* tracer_ = nullptr;
  metrics::HystrixStream* hystrix_ = nullptr;
  metrics::Prometheus* prom_ = nullptr;
  mutable std::mutex mu_;
  std::shared_ptr<const Content> content_;
  std::atomic<uint64_t> gen_{0};
  std::string last_translation_;
  bool logged_once_ = false;
};

}  // namespace hola::app
