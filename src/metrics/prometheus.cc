#include "metrics/prometheus.h"

#include "core/log.h"

#include <dirent.h>
#include <sys/resource.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "app/hola_app.h"
#include "core/build_info.h"
#include "core/isa.h"
#include "http/server.h"
#include "metrics/hystrix_stream.h"
#include "resilience/hystrix.h"
#include "tracing/tracer.h"

namespace hola::metrics {

namespace {
// The standard process_* metrics of Prometheus client libraries, from /proc/self.
void process_metrics(std::string* o) {
  const double tck = double(sysconf(_SC_CLK_TCK));
  const double page = double(sysconf(_SC_PAGESIZE));
  char buf[1024];
  char num[64];
  if (FILE* f = fopen("/proc/self/stat", "r")) {
    size_t n = fread(buf, 1, sizeof buf - 1, f);
    fclose(f);
    buf[n] = 0;
    // After the parenthesised comm: v[0] is field 3 (state), so field N is v[N - 3]:
    // utime 14, stime 15, starttime 22, vsize 23, rss 24 (pages).
    if (const char* p = strrchr(buf, ')')) {
      unsigned long long v[22] = {};
      const char* q = p + 1;
      for (int k = 0; k < 22 && *q; ++k) {
        while (*q == ' ') ++q;
        v[k] = strtoull(q, nullptr, 10);
        while (*q && *q != ' ') ++q;
      }
      snprintf(num, sizeof num, "%.2f", double(v[11] + v[12]) / tck);
      *o += "# TYPE process_cpu_seconds_total counter\nprocess_cpu_seconds_total ";
      *o += num;
      *o += "\n# TYPE process_virtual_memory_bytes gauge\nprocess_virtual_memory_bytes " + std::to_string(v[20]);
      *o += "\n# TYPE process_resident_memory_bytes gauge\nprocess_resident_memory_bytes " +
            std::to_string((unsigned long long)(double(v[21]) * page)) + "\n";
      if (FILE* st = fopen("/proc/stat", "r")) {
        unsigned long long btime = 0;
        char line[256];
        while (fgets(line, sizeof line, st))
          if (sscanf(line, "btime %llu", &btime) == 1) break;
        fclose(st);
        if (btime) {
          snprintf(num, sizeof num, "%.2f", double(btime) + double(v[19]) / tck);
          *o += "# TYPE process_start_time_seconds gauge\nprocess_start_time_seconds ";
          *o += num;
          *o += "\n";
        }
      }
    }
  }
  if (DIR* d = opendir("/proc/self/fd")) {
    long n = 0;
    while (dirent* e = readdir(d))
      if (e->d_name[0] != '.') ++n;
    closedir(d);
    // minus the descriptor the directory stream itself held
    *o += "# TYPE process_open_fds gauge\nprocess_open_fds " + std::to_string(n - 1) + "\n";
  }
  rlimit rl{};
  if (getrlimit(RLIMIT_NOFILE, &rl) == 0)
    *o += "# TYPE process_max_fds gauge\nprocess_max_fds " + std::to_string((unsigned long long)rl.rlim_cur) + "\n";
}
}  // namespace

Prometheus::Prometheus(int num_workers, int num_routes)
    : nworkers_(num_workers), nroutes_(num_routes), counts_(new Counter[size_t(num_workers) * size_t(num_routes)]),
      chain_lat_(new LatencyHist[size_t(num_workers)]) {}

std::string Prometheus::render(http::Server* server) const {
  std::string o;
  // what is running: constant 1, the labels carry the release, revision and ISA level
  o += "# HELP hola_build_info The build: release, source revision, x86-64 level, compiler.\n"
       "# TYPE hola_build_info gauge\nhola_build_info{version=\"";
  o += build_info::version();
  o += "\",revision=\"";
  o += build_info::revision();
  o += "\",isa=\"";
  o += isa::build_level();
  o += "\",compiler=\"";
  o += build_info::compiler();
  o += "\"} 1\n";
  o += "# HELP hola_requests_total Requests by route.\n# TYPE hola_requests_total counter\n";
  for (int r = 0; r < nroutes_; ++r) {
    uint64_t n = 0;
    for (int w = 0; w < nworkers_; ++w)
      n += counts_[size_t(w) * size_t(nroutes_) + size_t(r)].v.load(std::memory_order_relaxed);
    o += "hola_requests_total{route=\"";
    o += app::HolaApp::route_name(r);
    o += "\"} " + std::to_string(n) + "\n";
  }
  {
    uint64_t b[kLatencyBuckets + 1] = {}, sum_us = 0, count = 0;
    for (int w = 0; w < nworkers_; ++w) {
      const LatencyHist& h = chain_lat_[size_t(w)];
      for (int i = 0; i <= kLatencyBuckets; ++i) b[i] += h.bucket[i].load(std::memory_order_relaxed);
      sum_us += h.sum_us.load(std::memory_order_relaxed);
      count += h.count.load(std::memory_order_relaxed);
    }
    o += "# HELP hola_chaining_duration_seconds /api/hola-chaining latency (aloha call, timeout or fallback).\n"
         "# TYPE hola_chaining_duration_seconds histogram\n";
    uint64_t cum = 0;
    char num[64];
    for (int i = 0; i <= kLatencyBuckets; ++i) {
      cum += b[i];
      if (i < kLatencyBuckets) snprintf(num, sizeof num, "%g", double(kLatencyBoundsUs[i]) / 1e6);
      o += "hola_chaining_duration_seconds_bucket{le=\"";
      o += i < kLatencyBuckets ? num : "+Inf";
      o += "\"} " + std::to_string(cum) + "\n";
    }
    // Buckets are read before sum/count without a lock: under load the three may differ by
    // a few in-flight observations, which Prometheus tolerates.
    snprintf(num, sizeof num, "%.6f", double(sum_us) / 1e6);
    o += "hola_chaining_duration_seconds_sum ";
    o += num;
    o += "\nhola_chaining_duration_seconds_count " + std::to_string(count) + "\n";
  }
  if (server) {
    uint64_t acc = 0, closed = 0, perr = 0, bin = 0, bout = 0, req = 0, rej = 0;
    for (size_t i = 0; i < server->num_workers(); ++i) {
      auto& s = server->worker(i).stats();
      acc += s.accepted.load(std::memory_order_relaxed);
      closed += s.closed.load(std::memory_order_relaxed);
      perr += s.parse_errors.load(std::memory_order_relaxed);
      rej += s.rejected.load(std::memory_order_relaxed);
      bin += s.bytes_in.load(std::memory_order_relaxed);
      bout += s.bytes_out.load(std::memory_order_relaxed);
      req += s.requests.load(std::memory_order_relaxed);
    }
    o += "# TYPE hola_http_requests_total counter\nhola_http_requests_total " + std::to_string(req) + "\n";
    o += "# TYPE hola_connections_accepted_total counter\nhola_connections_accepted_total " + std::to_string(acc) + "\n";
    o += "# TYPE hola_connections_open gauge\nhola_connections_open " + std::to_string(acc - closed) + "\n";
    o += "# TYPE hola_parse_errors_total counter\nhola_parse_errors_total " + std::to_string(perr) + "\n";
    o += "# TYPE hola_connections_rejected_total counter\nhola_connections_rejected_total " + std::to_string(rej) + "\n";
    o += "# TYPE hola_bytes_in_total counter\nhola_bytes_in_total " + std::to_string(bin) + "\n";
    o += "# TYPE hola_bytes_out_total counter\nhola_bytes_out_total " + std::to_string(bout) + "\n";
    o += "# TYPE hola_workers gauge\nhola_workers " + std::to_string(server->num_workers()) + "\n";
    if (server->options().busy_poll_auto) {
      uint64_t hits = 0, misses = 0, offs = 0, off_ms = 0, resumes = 0;
      for (size_t i = 0; i < server->num_workers(); ++i) {
        const EventLoop& l = server->worker(i).loop();
        hits += l.spin_hits();
        misses += l.spin_misses();
        offs += l.spin_offs();
        off_ms += l.spin_off_ms();
        resumes += l.spin_resumes();
      }
      o += "# TYPE hola_busy_poll_spins_total counter\n";
      o += "hola_busy_poll_spins_total{result=\"hit\"} " + std::to_string(hits) + "\n";
      o += "hola_busy_poll_spins_total{result=\"miss\"} " + std::to_string(misses) + "\n";
      o += "# TYPE hola_busy_poll_backoffs_total counter\nhola_busy_poll_backoffs_total " + std::to_string(offs) + "\n";
      // milliseconds of spinning switched off, summed over workers (a worker backed off for
      // most of a saturated run serves every request through a sleep and a wake-up)
      o += "# TYPE hola_busy_poll_backoff_ms_total counter\nhola_busy_poll_backoff_ms_total " + std::to_string(off_ms) + "\n";
      // back-offs ended early because the blocking waits showed the loop busy
      o += "# TYPE hola_busy_poll_resumes_total counter\nhola_busy_poll_resumes_total " + std::to_string(resumes) + "\n";
    }
    {
      // Where the workers' time goes: CPU in polls that found nothing while spinning (process
      // CPU minus this = the CPU that served), waits that could sleep, and gaps between polls
      // (handlers + descheduling) past 100 us / 1 ms / 10 ms with the longest one
      uint64_t idle_ns = 0, sleeps = 0, gmax = 0, passes = 0, over[EventLoop::kGapBuckets] = {};
      for (size_t i = 0; i < server->num_workers(); ++i) {
        const EventLoop& l = server->worker(i).loop();
        passes += l.activity().passes.load(std::memory_order_relaxed);
        idle_ns += l.idle_spin_ns();
        sleeps += l.blocking_waits();
        gmax = std::max(gmax, l.gap_max_ns());
        for (int k = 0; k < EventLoop::kGapBuckets; ++k) over[k] += l.gaps_over(k);
      }
      char num[64];
      snprintf(num, sizeof num, "%.6f", double(idle_ns) / 1e9);
      o += "# TYPE hola_loop_idle_spin_seconds_total counter\nhola_loop_idle_spin_seconds_total ";
      o += num;
      o += "\n# TYPE hola_loop_blocking_waits_total counter\nhola_loop_blocking_waits_total " + std::to_string(sleeps) + "\n";
      o += "# TYPE hola_loop_passes_total counter\nhola_loop_passes_total " + std::to_string(passes) + "\n";
      // the workers' own user-space instructions and cycles (hardware counters), when the
      // host allows them: the CPU-independent efficiency figure of the serving code
      uint64_t ins = 0, cyc = 0;
      bool any = false;
      for (size_t i = 0; i < server->num_workers(); ++i) {
        uint64_t a = 0, b = 0;
        if (server->worker(i).counters().read(&a, &b)) {
          ins += a;
          cyc += b;
          any = true;
        }
      }
      if (any) {
        o += "# TYPE hola_worker_user_instructions_total counter\nhola_worker_user_instructions_total " +
             std::to_string(ins) + "\n";
        o += "# TYPE hola_worker_user_cycles_total counter\nhola_worker_user_cycles_total " + std::to_string(cyc) + "\n";
      }
      o += "# TYPE hola_loop_poll_gaps_total counter\n";
      static const char* const kOver[EventLoop::kGapBuckets] = {"100us", "1ms", "10ms"};
      for (int k = 0; k < EventLoop::kGapBuckets; ++k)
        o += std::string("hola_loop_poll_gaps_total{over=\"") + kOver[k] + "\"} " + std::to_string(over[k]) + "\n";
      snprintf(num, sizeof num, "%.6f", double(gmax) / 1e9);
      o += "# TYPE hola_loop_poll_gap_max_seconds gauge\nhola_loop_poll_gap_max_seconds ";
      o += num;
      o += "\n";
    }
    // the scheduler's time slice of the workers (--sched-slice-us; the kernel's default otherwise)
    if (server->num_workers() && server->worker(0).sched_slice_us() > 0) {
      char sl[32];
      snprintf(sl, sizeof sl, "%.6f", double(server->worker(0).sched_slice_us()) / 1e6);
      o += "# TYPE hola_worker_sched_slice_seconds gauge\nhola_worker_sched_slice_seconds ";
      o += sl;
      o += "\n";
    }
    // 1 from the termination signal on (readiness failing, --shutdown-delay-ms), 2 while draining
    o += "# TYPE hola_server_terminating gauge\nhola_server_terminating " +
         std::to_string(server->draining() ? 2 : server->terminating() ? 1 : 0) + "\n";
    // Loop timers armed and not yet fired: tracks the calls in flight, never the call rate.
    size_t timers = 0;
    for (size_t i = 0; i < server->num_workers(); ++i) timers += server->worker(i).loop().pending_timers();
    o += "# TYPE hola_event_loop_timers gauge\nhola_event_loop_timers " + std::to_string(timers) + "\n";
  }
#ifdef HOLA_COUNT_CLOCK_READS
  o += "# TYPE hola_clock_reads_total counter\nhola_clock_reads_total{clock=\"precise\"} " +
       std::to_string(g_clock_reads.load(std::memory_order_relaxed)) + "\nhola_clock_reads_total{clock=\"coarse\"} " +
       std::to_string(g_coarse_clock_reads.load(std::memory_order_relaxed)) + "\n";
#endif
  if (tracer_) {
    tracing::TracerStats t = tracer_->stats();
    o += "# TYPE hola_spans_recorded_total counter\nhola_spans_recorded_total " + std::to_string(t.recorded) + "\n";
    o += "# TYPE hola_spans_reported_total counter\nhola_spans_reported_total " + std::to_string(t.reported) + "\n";
    o += "# TYPE hola_spans_dropped_total counter\nhola_spans_dropped_total{reason=\"ring_full\"} " +
         std::to_string(t.dropped_ring) + "\nhola_spans_dropped_total{reason=\"collector\"} " +
         std::to_string(t.dropped_no_collector) + "\nhola_spans_dropped_total{reason=\"queue_full\"} " +
         std::to_string(t.dropped_queue) + "\n";
    o += "# TYPE hola_span_post_failures_total counter\nhola_span_post_failures_total " + std::to_string(t.post_failures) + "\n";
  }
  if (cmd_) {
    resilience::CommandSnapshot s = cmd_->snapshot();
    o += "# TYPE hola_hystrix_events_total counter\n";
    for (int e = 0; e < resilience::kNumEvents; ++e) {
      if (!s.cumulative[size_t(e)]) continue;
      o += "hola_hystrix_events_total{command=\"" + s.name + "\",event=\"" + resilience::event_name(resilience::Event(e)) +
           "\"} " + std::to_string(s.cumulative[size_t(e)]) + "\n";
    }
    o += "# TYPE hola_hystrix_circuit_open gauge\nhola_hystrix_circuit_open{command=\"" + s.name + "\"} " +
         (s.circuit_open ? "1" : "0") + "\n";
    // breaker transitions: opened, and closed by the trial call after the sleep window or
    // earlier by a call already running when it opened (Hystrix 1.5's markSuccess)
    o += "# TYPE hola_hystrix_circuit_transitions_total counter\n";
    o += "hola_hystrix_circuit_transitions_total{command=\"" + s.name + "\",to=\"open\"} " +
         std::to_string(s.circuit_opened) + "\n";
    o += "hola_hystrix_circuit_transitions_total{command=\"" + s.name + "\",to=\"closed\",by=\"trial\"} " +
         std::to_string(s.circuit_closed_trial) + "\n";
    o += "hola_hystrix_circuit_transitions_total{command=\"" + s.name + "\",to=\"closed\",by=\"inflight\"} " +
         std::to_string(s.circuit_closed_inflight) + "\n";
    // the bulkhead: calls holding a pool slot, and calls waiting in the pool queue
    o += "# TYPE hola_hystrix_pool_active gauge\nhola_hystrix_pool_active{command=\"" + s.name + "\"} " +
         std::to_string(s.pool_active) + "\n";
    o += "# TYPE hola_hystrix_pool_queued gauge\nhola_hystrix_pool_queued{command=\"" + s.name + "\"} " +
         std::to_string(s.pool_queue_size) + "\n";
  }
  process_metrics(&o);
  o += "# TYPE hola_log_lines_dropped_total counter\nhola_log_lines_dropped_total " +
       std::to_string(Logger::instance().dropped()) + "\n";
  if (reloads_) o += "# TYPE hola_config_reloads_total counter\nhola_config_reloads_total " + std::to_string(reloads_()) + "\n";
  if (feign_retries_ && transport_retries_) {
    o += "# TYPE hola_aloha_retries_total counter\nhola_aloha_retries_total{kind=\"feign\"} " +
         std::to_string(feign_retries_()) + "\nhola_aloha_retries_total{kind=\"transport\"} " +
         std::to_string(transport_retries_()) + "\n";
  }
  if (server) {
    o += "# TYPE hola_accept_locality_total counter\n";
    for (int l = 0; l < http::Server::kNumLocality; ++l)
      o += std::string("hola_accept_locality_total{relation=\"") + http::Server::locality_name(l) + "\"} " +
           std::to_string(server->locality(l)) + "\n";
  }
  if (stream_) {
    o += "# TYPE hola_hystrix_stream_subscribers gauge\nhola_hystrix_stream_subscribers " +
         std::to_string(stream_->subscribers()) + "\n";
    o += "# TYPE hola_hystrix_stream_frames_skipped_total counter\nhola_hystrix_stream_frames_skipped_total " +
         std::to_string(stream_->frames_skipped()) + "\n";
    o += "# TYPE hola_hystrix_stream_stalled_closed_total counter\nhola_hystrix_stream_stalled_closed_total " +
         std::to_string(stream_->stalled_closed()) + "\n";
  }
  return o;
}

}  // namespace hola::metrics
