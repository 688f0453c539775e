// hola — native replacement for the WildFly Swarm uber-jar.
//
// Boot sequence (the reference's contextInitialized listeners, in explicit code):
//   config sources + watcher   (Configuration.java, ConfigSource SPI, config.properties)
//   tracer                      (ZipkinResource.java, ZipKinFilter.java)
//   aloha chainer + Hystrix     (HolaResource.getNextService, config.properties:17,19)
//   /hystrix.stream             (HystrixServlet.java)
//   HTTP server on :8080        (Dockerfile:8, pom.xml:74)
// SIGTERM/SIGINT/SIGHUP: stop accepting, drain in-flight requests, flush spans, exit 0.
#include <errno.h>
#include <signal.h>
#include <atomic>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <mutex>
#include <thread>

#include "app/aloha_chainer.h"
#include "app/hola_app.h"
#include "config/manager.h"
#include "config/resolver.h"
#include "core/affinity.h"
#include "core/build_info.h"
#include "core/clock.h"
#include "core/cpuprof.h"
#include "core/isa.h"
#include "core/log.h"
#include "core/net.h"
#include "http/server.h"
#include "metrics/hystrix_stream.h"
#include "metrics/prometheus.h"
#include "tracing/tracer.h"

using namespace hola;

namespace {

void usage() {
  fprintf(stderr,
          "usage: hola [options] [-Dkey=value ...]   (hola --version: release and build)\n"
          "  --port N                 listen port (default: -Dswarm.http.port, 8080, plus\n"
          "                           -Dswarm.port.offset)\n"
          "  --host ADDR              listen address (default: -Dswarm.bind.address, 0.0.0.0)\n"
          "  --threads N              event-loop workers (default: one per allowed CPU, capped by cgroup quota)\n"
          "  --cpu-list LIST          pin workers to these CPUs, e.g. 0-3,8\n"
          "  --accept rr|reuseport    connection distribution (default rr)\n"
          "  --reuseport-cpu none|self|sibling   with --accept reuseport and pinned workers, each worker's\n"
          "                           listener names this CPU as its incoming CPU, so the kernel hands a\n"
          "                           connection to the worker expecting clients there (default none = hash)\n"
          "  --conf PATH              greeting properties file (same as -Dconf=PATH)\n"
          "  --deltaspike-properties PATH   ordinal-100 properties file\n"
          "  --hystrix-config PATH    Hystrix properties (Archaius config.properties role)\n"
          "  --hostname NAME          override $HOSTNAME for the greeting\n"
          "  --zipkin-url URL         span collector (default $ZIPKIN_SERVER_URL)\n"
          "  --zipkin-v2              POST /api/v2/spans instead of /api/v1/spans\n"
          "  --trace-sample-rate R    0..1 (default 1)\n"
          "  --no-tracing             disable tracing entirely\n"
          "  --trace-queue N          spans exported per flush interval, the rest dropped and counted\n"
          "                           (default 1000: Brave 3's collector queue; 0 = bounded by the rings)\n"
          "  --trace-ring N           per-worker span ring capacity (default 2048)\n"
          "  --aloha-url URL          downstream service (default http://aloha:8080/)\n"
          "  --aloha-path PATH        downstream path (default api/aloha-chaining)\n"
          "  --feign-log basic|none   outbound call logging (default basic)\n"
          "  --feign-retry default|off|P,MAX,N   Feign Retryer on IO errors (default: Retryer.Default\n"
          "                           = 100 ms period, 1000 ms max period, 5 attempts)\n"
          "  --feign-timeouts C,R     Feign Request.Options: connect / read timeout in ms (default\n"
          "                           10000,60000; the read timeout applies when the Hystrix timeout\n"
          "                           is disabled or longer)\n"
          "  --aloha-pipeline N       pipeline up to N concurrent aloha calls per kept-alive connection,\n"
          "                           a batch's requests in one send (default 1 = off, as HttpClient)\n"
          "  --hystrix-command-key method|configkey|KEY   Hystrix command key of the aloha call\n"
          "                           (default method = \"aloha\", feign-hystrix 8.x; configkey =\n"
          "                           \"AlohaService#aloha()\", feign-hystrix 9.x SetterFactory.Default)\n"
          "  --hystrix-stream-max N   max /hystrix.stream subscribers (default 5)\n"
          "  --hystrix-stream-stall-ms N   close a subscriber that has not read for N ms (default 30000)\n"
          "  --hystrix-timeout-ms N | --hystrix-request-volume N | --hystrix-error-pct N |\n"
          "  --hystrix-sleep-window-ms N | --hystrix-pool-size N\n"
          "                           shorthands for -Dhystrix.command.default.* / threadpool.default.*\n"
          "  --config-poll-ms N       config re-check interval (default 1000)\n"
          "  --drain-ms N             graceful shutdown drain budget (default 5000)\n"
          "  --shutdown-delay-ms N    on SIGTERM/SIGINT/SIGHUP, first keep serving and accepting for N ms\n"
          "                           with /api/health answering 503 and every response closing its\n"
          "                           connection, then drain (default 0; the manifests set it so a\n"
          "                           rolling update outlasts endpoint propagation). A second signal\n"
          "                           ends the delay early\n"
          "  --exit-deadline-ms N     a termination still running N ms after the signal exits with status 3\n"
          "                           (default: shutdown delay + drain budget + 10000; 0 = never)\n"
          "  --port-file PATH         write the bound port here once listening\n"
          "  --busy-poll-us N|auto[:N] spin up to N us in epoll before sleeping (default auto; 0 = off); auto = adaptive:\n"
          "                           spin (20 us, or N) while spinning mostly finds work (saturation),\n"
          "                           back off while it mostly waits in vain (light load)\n"
          "  --busy-poll-pause N      PAUSE instructions between empty polls (SMT-friendly spin)\n"
          "  --sched-slice-us N       ask the scheduler for an N us time slice per worker (EEVDF custom slice,\n"
          "                           Linux 6.12+; default: the kernel's)\n"
          "  --idle-timeout-ms N      close connections with nothing read or written this long\n"
          "                           (default 60000, 0 = never)\n"
          "  --max-connections N      refuse connections beyond N per replica (default unlimited)\n"
          "  --no-steer               plain round-robin accept (default: L3-domain steering when pinned)\n"
          "  --epoll-lt               level-triggered connection sockets (default: edge-triggered)\n"
          "  --no-perf-counters       do not count the workers' user-space instructions and cycles\n"
          "                           (hardware counters on /metrics, where the host allows them)\n"
          "  --no-pin                 leave workers unpinned even when the affinity mask has exactly\n"
          "                           one CPU per worker (e.g. a kubelet static-CPU-manager cpuset)\n"
          "  --profile                per-stage latency histograms (accept/recv/parse/handle/send), dumped at exit\n"
          "  --profile-out PATH       write the --profile JSON here (default: stderr)\n"
          "  --cpu-profile PATH       sample the server's threads' call stacks on their CPU time and write\n"
          "                           them here at exit (bench/cpuprof_report.py symbolises them)\n"
          "  --cpu-profile-hz N       samples per CPU-second of each thread (default 1000)\n"
          "  --log-level L            debug|info|warn|error|off (default info)\n"
          "  --no-metrics             disable the /metrics endpoint\n");
}

constexpr int kAutoBusyPollUs = 20;  // spin budget of --busy-poll-us auto

bool need(int i, int argc, const char* flag) {
  if (i + 1 >= argc) {
    fprintf(stderr, "hola: %s needs a value\n", flag);
    return false;
  }
  return true;
}

}  // namespace

// See the exit watchdog in main(): the time a termination may take beyond the shutdown delay
// and the drain budget (the reporter's last span export alone may take its 2 s timeout).
constexpr int64_t kExitMarginMs = 10000;
// What the watchdog's report may take (main's stack: 200 ms capture; each worker: a 100 ms
// pass window and a 2 s budget for the stacks): the watchdog starts that much before the
// deadline, so the process has exited with status 3 by the deadline itself and a kubelet
// SIGKILL timed to it (--exit-deadline-ms = terminationGracePeriodSeconds) cannot cut the
// report short. A deadline under twice the budget starts the report half way instead.
constexpr int64_t kExitReportBudgetMs = 2500;

namespace {
// The termination step main is in, for the exit watchdog's report (a string literal).
std::atomic<const char*> g_term_step{"serving"};
void term_step(const char* s) { g_term_step.store(s, std::memory_order_relaxed); }
// The watchdog reports while holding this; main takes it before its locals (the server the
// report reads) go away, so a watchdog that fires just as main returns either finishes its
// report and exits first or finds the termination complete.
std::mutex g_watchdog_mu;
bool g_terminated = false;
}  // namespace

int main(int argc, char** argv) {
  http::ServerOptions so;
  // Adaptive busy-polling by default: the same saturation throughput as a fixed spin, less CPU
  // than no spinning at light load, and a microsecond p99 (profiles/round3/08_busypoll);
  // `--busy-poll-us 0` turns it off.
  so.busy_poll_auto = true;
  so.busy_poll_us = kAutoBusyPollUs;
  std::map<std::string, std::string> sysprops;
  const char* jo = getenv("JAVA_OPTIONS");
  if (jo) sysprops = config::parse_java_options(jo);  // `oc env dc/hola JAVA_OPTIONS=-Dconf=...`
  config::ManagerOptions mo;
  app::AppOptions ao;
  app::AlohaOptions alo;
  tracing::TracerOptions to;
  const char* zu = getenv("ZIPKIN_SERVER_URL");
  if (zu) to.collector_url = zu;
  const char* hn = getenv("HOSTNAME");
  if (hn) ao.hostname = hn;  // HolaResource.java:57 getOrDefault("HOSTNAME", "unknown")
  int threads = 0, drain_ms = 5000, stream_max = -1, shutdown_delay_ms = 0;
  int64_t exit_deadline_ms = -1;  // -1: delay + drain + kExitMarginMs; 0: no watchdog
  int64_t stream_stall_ms = 30000;
  std::string cpu_list, port_file, profile_out, cpu_profile;
  int cpu_profile_hz = 1000;
  bool auto_pin = true;
  bool no_tracing = false;
  bool port_flag = false, host_flag = false;

  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&](const char* f) -> std::string {
      if (!need(i, argc, f)) exit(2);
      return argv[++i];
    };
    if (a.rfind("-D", 0) == 0 && a.size() > 2) {
      size_t eq = a.find('=');
      if (eq == std::string::npos) sysprops[a.substr(2)] = "";
      else sysprops[a.substr(2, eq - 2)] = a.substr(eq + 1);
    } else if (a == "--port") {
      so.port = atoi(val("--port").c_str());
      port_flag = true;
    } else if (a == "--host") {
      so.host = val("--host");
      host_flag = true;
    }
    else if (a == "--threads") threads = atoi(val("--threads").c_str());
    else if (a == "--cpu-list") cpu_list = val("--cpu-list");
    else if (a == "--accept") {
      std::string m = val("--accept");
      if (m == "reuseport") so.reuseport_accept = true;
      else if (m != "rr") { fprintf(stderr, "hola: --accept rr|reuseport\n"); return 2; }
    } else if (a == "--reuseport-cpu") {
      std::string m = val("--reuseport-cpu");
      if (m == "none") so.reuseport_cpu = http::ServerOptions::ReuseportCpu::kNone;
      else if (m == "self") so.reuseport_cpu = http::ServerOptions::ReuseportCpu::kSelf;
      else if (m == "sibling") so.reuseport_cpu = http::ServerOptions::ReuseportCpu::kSibling;
      else { fprintf(stderr, "hola: --reuseport-cpu none|self|sibling\n"); return 2; }
    } else if (a == "--conf") sysprops["conf"] = val("--conf");
    else if (a == "--deltaspike-properties") mo.deltaspike_properties = val("--deltaspike-properties");
    else if (a == "--hystrix-config") mo.hystrix_config = val("--hystrix-config");
    else if (a == "--hostname") ao.hostname = val("--hostname");
    else if (a == "--zipkin-url") to.collector_url = val("--zipkin-url");
    else if (a == "--zipkin-v2") to.v2 = true;
    else if (a == "--trace-sample-rate") to.sample_rate = atof(val("--trace-sample-rate").c_str());
    else if (a == "--no-tracing") no_tracing = true;
    else if (a == "--trace-queue") to.queue_spans = size_t(atoll(val("--trace-queue").c_str()));
    else if (a == "--trace-ring") to.ring_capacity = size_t(atoll(val("--trace-ring").c_str()));
    else if (a == "--hystrix-timeout-ms")
      sysprops["hystrix.command.default.execution.isolation.thread.timeoutInMilliseconds"] = val(a.c_str());
    else if (a == "--hystrix-request-volume")
      sysprops["hystrix.command.default.circuitBreaker.requestVolumeThreshold"] = val(a.c_str());
    else if (a == "--hystrix-error-pct")
      sysprops["hystrix.command.default.circuitBreaker.errorThresholdPercentage"] = val(a.c_str());
    else if (a == "--hystrix-sleep-window-ms")
      sysprops["hystrix.command.default.circuitBreaker.sleepWindowInMilliseconds"] = val(a.c_str());
    else if (a == "--hystrix-pool-size") sysprops["hystrix.threadpool.default.coreSize"] = val(a.c_str());
    else if (a == "--aloha-url") alo.url = val("--aloha-url");
    else if (a == "--aloha-path") {
      alo.path = val("--aloha-path");
      while (!alo.path.empty() && alo.path.front() == '/') alo.path.erase(0, 1);
    }
    else if (a == "--feign-log") alo.feign_log_basic = val("--feign-log") == "basic";
    else if (a == "--feign-retry") {
      if (!app::parse_retry_policy(val("--feign-retry"), &alo.retry)) {
        fprintf(stderr, "hola: --feign-retry default|off|PERIOD_MS,MAX_PERIOD_MS,MAX_ATTEMPTS\n");
        return 2;
      }
    } else if (a == "--feign-timeouts") {
      int c = 0, r = 0;
      char tail = 0;
      if (sscanf(val("--feign-timeouts").c_str(), "%d,%d%c", &c, &r, &tail) != 2 || c < 0 || r < 0) {
        fprintf(stderr, "hola: --feign-timeouts CONNECT_MS,READ_MS\n");
        return 2;
      }
      alo.connect_timeout_ms = c;
      alo.read_timeout_ms = r;
    } else if (a == "--aloha-pipeline") {
      alo.pipeline = atoi(val("--aloha-pipeline").c_str());
      if (alo.pipeline < 1 || alo.pipeline > 256) {
        fprintf(stderr, "hola: --aloha-pipeline takes 1..256\n");
        return 2;
      }
    } else if (a == "--hystrix-command-key") {
      std::string k = val("--hystrix-command-key");
      if (k == "method") alo.command_key = "aloha";
      else if (k == "configkey") alo.command_key = alo.config_key;
      else if (!k.empty()) alo.command_key = k;
    }
    else if (a == "--hystrix-stream-max") stream_max = atoi(val("--hystrix-stream-max").c_str());
    else if (a == "--hystrix-stream-stall-ms") stream_stall_ms = atoll(val("--hystrix-stream-stall-ms").c_str());
    else if (a == "--config-poll-ms") mo.poll_ms = atoi(val("--config-poll-ms").c_str());
    else if (a == "--drain-ms") drain_ms = atoi(val("--drain-ms").c_str());
    else if (a == "--shutdown-delay-ms") shutdown_delay_ms = std::max(0, atoi(val("--shutdown-delay-ms").c_str()));
    else if (a == "--exit-deadline-ms") exit_deadline_ms = std::max<int64_t>(0, atoll(val("--exit-deadline-ms").c_str()));
    else if (a == "--port-file") port_file = val("--port-file");
    else if (a == "--busy-poll-us") {
      const std::string v = val("--busy-poll-us");
      so.busy_poll_auto = v == "auto" || v.rfind("auto:", 0) == 0;
      so.busy_poll_us = so.busy_poll_auto ? (v.size() > 5 ? atoi(v.c_str() + 5) : kAutoBusyPollUs) : atoi(v.c_str());
    }
    else if (a == "--busy-poll-pause") so.busy_poll_pause = atoi(val("--busy-poll-pause").c_str());
    else if (a == "--sched-slice-us") so.sched_slice_us = atoi(val("--sched-slice-us").c_str());
    else if (a == "--profile") so.profile = true;
    else if (a == "--no-steer") so.steer_l3 = false;
    else if (a == "--no-perf-counters") so.perf_counters = false;
    else if (a == "--no-pin") auto_pin = false;
    else if (a == "--epoll-lt") so.edge_triggered = false;
    else if (a == "--idle-timeout-ms") so.idle_timeout_ms = atoi(val("--idle-timeout-ms").c_str());
    else if (a == "--max-connections") so.max_connections = size_t(atol(val("--max-connections").c_str()));
    else if (a == "--profile-out") profile_out = val("--profile-out");
    else if (a == "--cpu-profile") cpu_profile = val("--cpu-profile");
    else if (a == "--cpu-profile-hz") cpu_profile_hz = atoi(val("--cpu-profile-hz").c_str());
    else if (a == "--no-metrics") ao.enable_metrics_endpoint = false;
    else if (a == "--log-level") {
      LogLevel l;
      if (!parse_log_level(val("--log-level"), &l)) { fprintf(stderr, "hola: bad --log-level\n"); return 2; }
      Logger::instance().set_level(l);
    } else if (a == "-h" || a == "--help") {
      usage();
      return 0;
    } else if (a == "--version") {
      printf("hola %s (revision %s, %s, %s, %s)\n", build_info::version(), build_info::revision(), isa::build_level(),
             build_info::compiler(), build_info::build_type());
      return 0;
    } else {
      fprintf(stderr, "hola: unknown argument '%s'\n", a.c_str());
      usage();
      return 2;
    }
  }

  // ---- listen address ----
  // WildFly Swarm 1.0's socket-binding properties (on the command line or in JAVA_OPTIONS, as
  // `java -Dswarm.http.port=8081 -jar hola-swarm.jar` takes them): swarm.http.port (8080),
  // swarm.port.offset added to it, swarm.bind.address (0.0.0.0). An explicit --port / --host
  // wins and takes no offset.
  if (!port_flag) {
    auto prop_int = [&](const char* k, int dflt, int* out) {
      auto it = sysprops.find(k);
      if (it == sysprops.end() || it->second.empty()) {
        *out = dflt;
        return true;
      }
      char* end = nullptr;
      long v = strtol(it->second.c_str(), &end, 10);
      if (*end || v < -65535 || v > 65535) {
        fprintf(stderr, "hola: bad -D%s=%s\n", k, it->second.c_str());
        return false;
      }
      *out = int(v);
      return true;
    };
    int port = 0, offset = 0;
    if (!prop_int("swarm.http.port", so.port, &port) || !prop_int("swarm.port.offset", 0, &offset)) return 2;
    if (port + offset < 0 || port + offset > 65535) {
      fprintf(stderr, "hola: swarm.http.port %d + swarm.port.offset %d is not a port\n", port, offset);
      return 2;
    }
    so.port = port + offset;
  }
  if (!host_flag) {
    auto it = sysprops.find("swarm.bind.address");
    if (it != sysprops.end() && !it->second.empty()) so.host = it->second;
  }

  // ---- CPUs / workers ----
  std::vector<int> cpus;
  if (!cpu_list.empty() && !parse_cpu_list(cpu_list, &cpus)) {
    fprintf(stderr, "hola: bad --cpu-list '%s'\n", cpu_list.c_str());
    return 2;
  }
  if (threads <= 0) {
    size_t n = cpus.empty() ? allowed_cpus().size() : cpus.size();
    double quota = cgroup_cpu_quota();
    if (quota > 0 && double(n) > quota) n = size_t(quota);
    threads = n ? int(n) : 1;
  }
  if (cpus.empty() && auto_pin && threads > 1) {
    // Exclusive cpuset (Guaranteed pod with integer CPUs under the static CPU manager, or
    // taskset): one worker per allowed CPU, each pinned, which also enables accept steering.
    std::vector<int> allowed = allowed_cpus();
    if (allowed.size() == size_t(threads)) cpus = allowed;
  }
  so.threads = threads;
  so.cpus = cpus;

  // Block termination signals in every thread; main waits for them with sigwait.
  sigset_t sigs;
  sigemptyset(&sigs);
  sigaddset(&sigs, SIGTERM);
  sigaddset(&sigs, SIGINT);
  // The JVM runs its shutdown hooks on SIGHUP too, unless the signal was ignored at start-up
  // (nohup); the same here.
  struct sigaction hup {};
  if (sigaction(SIGHUP, nullptr, &hup) == 0 && hup.sa_handler != SIG_IGN) sigaddset(&sigs, SIGHUP);
  pthread_sigmask(SIG_BLOCK, &sigs, nullptr);
  signal(SIGPIPE, SIG_IGN);

  // ---- config ----
  mo.sysprops = sysprops;
  mo.env = config::environment_map();
  config::Manager cfg(mo);

  // ---- app, tracer, chainer, stream ----
  app::HolaApp app(ao);
  http::Server server(so, &app);
  std::string err;
  if (!server.bind(&err)) {
    fprintf(stderr, "hola: %s\n", err.c_str());
    return 1;
  }
  app.set_server(&server);

  to.enabled = !no_tracing;
  to.ipv4 = local_ipv4();
  to.port = server.port();
  tracing::Tracer tracer(to, threads);
  if (to.enabled) app.set_tracer(&tracer);

  // Built-in Hystrix defaults = the reference's tuned config.properties:17,19.
  std::map<std::string, std::string> hystrix_defaults = {
      {"hystrix.command.default.execution.isolation.thread.timeoutInMilliseconds", "600"},
      {"hystrix.command.default.circuitBreaker.requestVolumeThreshold", "5"}};
  auto hystrix_settings = [&](const std::map<std::string, std::string>& props) {
    std::map<std::string, std::string> merged = hystrix_defaults;
    for (auto& [k, v] : props) merged[k] = v;
    return resilience::settings_from(merged, alo.command_key, alo.url);
  };
  app::AlohaChainer chainer(alo, hystrix_settings({}), threads, to.enabled ? &tracer : nullptr);
  app.set_chainer(&chainer);
  if (stream_max < 0) {
    // HystrixMetricsStreamServlet reads the Archaius property
    // hystrix.stream.maxConcurrentConnections (default 5) [lib-default].
    auto it = sysprops.find("hystrix.stream.maxConcurrentConnections");
    stream_max = it != sysprops.end() && !it->second.empty() ? atoi(it->second.c_str()) : 5;
  }
  metrics::HystrixStream stream(stream_max);
  stream.set_stall_close_ms(stream_stall_ms);
  stream.add_command(&chainer.command());
  app.set_hystrix_stream(&stream);
  metrics::Prometheus prom(threads, app::HolaApp::kNumRoutes);
  prom.set_tracer(to.enabled ? &tracer : nullptr);
  prom.set_command(&chainer.command());
  prom.set_config_reloads([&cfg] { return cfg.reloads(); });
  prom.set_stream(&stream);
  prom.set_retries([&chainer] { return chainer.feign_retries(); }, [&chainer] { return chainer.transport_retries(); });
  app.set_prometheus(&prom);

  cfg.start([&](const config::Snapshot& s) {
    app.on_config(s);
    chainer.update_settings(hystrix_settings(s.hystrix));
  });

  if (!cpu_profile.empty() && !cpuprof::start(cpu_profile, cpu_profile_hz)) {
    fprintf(stderr, "hola: cannot start the CPU profiler\n");
    return 1;
  }
  cpuprof::enable_capture();  // stall reports capture worker stacks by signal
  cpuprof::note_thread();     // ... and main's
  chainer.start();
  tracer.start();
  server.start();

  LOG_INFO("hola listening on %s:%d (workers=%d, cpus=%s, accept=%s, tracing=%s, aloha=%s)", so.host.c_str(),
           server.port(), threads, cpus.empty() ? "unpinned" : format_cpu_list(cpus).c_str(),
           so.reuseport_accept ? (server.steering() ? "reuseport+l3-steering" : "reuseport")
                               : (server.steering() ? "rr+l3-steering" : "rr"),
           !to.enabled ? "off" : (to.collector_url.empty() ? "on (no collector: spans dropped)" : to.collector_url.c_str()),
           chainer.full_url().c_str());
  // The start-up lines are on stderr before anyone is told the port (supervisors and tests
  // read them as soon as the port file appears).
  Logger::instance().flush();
  if (!port_file.empty()) {
    std::string tmp = port_file + ".tmp";
    {
      std::ofstream f(tmp);
      f << server.port() << "\n";
    }
    rename(tmp.c_str(), port_file.c_str());
  }

  int sig = 0;
  sigwait(&sigs, &sig);
  const char* sig_name = sig == SIGTERM ? "SIGTERM" : sig == SIGINT ? "SIGINT" : "SIGHUP";
  {
    // Exit watchdog: a termination that has not finished within the delay, the drain and a
    // margin for the span flush and the helper threads ends here, with a line saying so,
    // rather than at the kubelet's SIGKILL (terminationGracePeriodSeconds 30 in the
    // manifests; the defaults sum to 20 s). The line is written straight to fd 2: the log
    // writer may be what is stuck.
    const int64_t limit_ms = exit_deadline_ms >= 0 ? exit_deadline_ms
                                                   : int64_t(shutdown_delay_ms) + std::max(0, drain_ms) + kExitMarginMs;
    const int main_tid = cpuprof::current_tid();
    const int64_t report_ms = limit_ms > 2 * kExitReportBudgetMs ? limit_ms - kExitReportBudgetMs : limit_ms / 2;
    if (limit_ms > 0) std::thread([limit_ms, report_ms, &server, main_tid] {
      std::this_thread::sleep_for(std::chrono::milliseconds(report_ms));
      std::lock_guard<std::mutex> g(g_watchdog_mu);
      if (g_terminated) return;
      char line[200];
      const int n = snprintf(line, sizeof line,
                             "hola: termination did not complete within %lld ms; exiting (exit deadline %lld ms, "
                             "less the report's budget)\n",
                             (long long)report_ms, (long long)limit_ms);
      ssize_t w = ::write(2, line, size_t(n));
      // where main is (the termination step and its stack), then every event loop, with its
      // stack (the report that names a stuck handler)
      {
        uintptr_t pcs[cpuprof::kMaxCaptureDepth];
        const int k = cpuprof::capture(main_tid, pcs, cpuprof::kMaxCaptureDepth);
        const std::string m = std::string("hola: main: ") + g_term_step.load(std::memory_order_relaxed) +
                              (k > 0 ? "; stack" + cpuprof::describe_pcs(pcs, k) : "; stack: no answer") + "\n";
        w = ::write(2, m.data(), m.size());
      }
      std::vector<size_t> all(server.num_workers());
      for (size_t i = 0; i < all.size(); ++i) all[i] = i;
      for (const std::string& r : server.stall_reports(all, true)) {
        const std::string line = "hola: " + r + "\n";
        w = ::write(2, line.data(), line.size());
      }
      (void)w;
      _exit(3);
    }).detach();
  }
  if (shutdown_delay_ms > 0) {
    // Phase 1: fail readiness, keep accepting, close connections between responses. The
    // pod's endpoint removal takes a while to reach every proxy (kube-proxy's sync); new
    // connections routed here meanwhile are still served.
    term_step("shutdown delay");
    server.begin_termination();  // before the log line: the line says it has happened
    LOG_INFO("received %s: readiness failing, still serving for %d ms", sig_name, shutdown_delay_ms);
    Logger::instance().flush();
    // sigtimedwait returns early with EINTR when the thread is stopped and resumed (SIGSTOP /
    // SIGCONT, a ptrace attach such as the executor's stack sampler): wait out the rest.
    const int64_t until = mono_ns() + int64_t(shutdown_delay_ms) * 1000000;
    for (;;) {
      const int64_t left = until - mono_ns();
      if (left <= 0) break;
      timespec ts{time_t(left / 1000000000), long(left % 1000000000)};
      siginfo_t si;
      if (sigtimedwait(&sigs, &si, &ts) > 0) {
        LOG_INFO("second termination signal: ending the delay early");
        break;
      }
      if (errno != EINTR) break;  // EAGAIN: the delay is over
    }
  }
  LOG_INFO("received %s: draining (up to %d ms)", sig_name, drain_ms);
  term_step("drain (Server::shutdown)");
  server.shutdown(drain_ms);
  term_step("joining the workers");
  server.join();
  if (so.profile) {
    std::string pj = server.profile_json();
    if (profile_out.empty()) {
      LOG_INFO("profile: %s", pj.c_str());
    } else {
      std::ofstream f(profile_out);
      f << pj << "\n";
    }
  }
  term_step("stopping the config watcher");
  cfg.stop();
  term_step("stopping the aloha client");
  chainer.stop();
  term_step("flushing spans (Tracer::stop)");
  tracer.stop();
  term_step("writing the CPU profile and the last log lines");
  if (!cpu_profile.empty() && !cpuprof::write()) LOG_WARN("could not write the CPU profile to %s", cpu_profile.c_str());
  LOG_INFO("shutdown complete (%llu requests served)", (unsigned long long)server.total_requests());
  Logger::instance().flush();
  {
    std::lock_guard<std::mutex> g(g_watchdog_mu);
    g_terminated = true;
  }
  return 0;
}
