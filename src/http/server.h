// HTTP/1.1 server: N pinned workers, each an EventLoop that owns its connections.
//
// Replaces the Undertow IO/worker pools of the reference's WildFly Swarm runtime
// (SURVEY.md T1, CS2). Accepted sockets are dealt round-robin to workers by the acceptor
// (loop 0) so a closed-loop benchmark with a few dozen keep-alive connections is balanced
// exactly; `reuseport` mode instead gives every worker its own SO_REUSEPORT listener.
#pragma once
#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "core/histogram.h"
#include "core/loop.h"
#include "core/perfcount.h"
#include "http/parser.h"

namespace hola::http {

class Worker;
class Server;

// EventLoop::note() handler kinds of the server's handlers (0 is the loop's own).
constexpr uint32_t kConnectionHandler = 1, kAcceptorHandler = 2;

// Per-worker request counters, readable (relaxed) from other threads for /metrics.
struct alignas(64) WorkerStats {
  std::atomic<uint64_t> requests{0};
  std::atomic<uint64_t> accepted{0};
  std::atomic<uint64_t> closed{0};
  std::atomic<uint64_t> parse_errors{0};
  std::atomic<uint64_t> rejected{0};  // refused over max_connections
  std::atomic<uint64_t> bytes_in{0};
  std::atomic<uint64_t> bytes_out{0};
  // single-writer increment without a locked RMW
  static void bump(std::atomic<uint64_t>& c, uint64_t d = 1) {
    c.store(c.load(std::memory_order_relaxed) + d, std::memory_order_relaxed);
  }
};

class Connection final : public EventLoop::Handler {
 public:
  Connection(Worker* w, int fd, uint64_t id);
  ~Connection() override;

  void on_event(uint32_t events) override;

  Worker& worker() { return *worker_; }
  int fd() const { return fd_; }
  uint64_t id() const { return id_; }
  bool closed() const { return closed_; }

  // Queue response bytes (copied unless the socket takes them immediately). Order preserved.
  void send(const char* p, size_t n);
  void send(std::string_view s) { send(s.data(), s.size()); }
  // The same for bytes in a buffer that stays unchanged until this connection's next handler
  // runs (the worker's prepared responses): written to the socket from there, without the
  // copy into the output buffer, when nothing else is queued before them. Whatever the socket
  // does not take at once is copied, as are bytes queued behind other output.
  void send_stable(std::string_view s);
  // After the current response: close the connection once all queued bytes are written.
  void close_after_response() { close_after_flush_ = true; }

  // Async requests: park() from inside on_request; later call complete() (on the worker
  // thread) with the full response. Input processing resumes after completion. keep_alive is
  // what the response announces (false once the server is closing(); the caller decides).
  void park() { parked_ = true; }
  void complete(std::string_view response, bool keep_alive);
  // complete() for a response written straight into the output buffer: append it to
  // response_buffer() (nothing else may be queued in between), then call complete_appended().
  std::string& response_buffer() {
    materialize();
    return out_;
  }
  void complete_appended(bool keep_alive);

  // Long-lived streaming responses (SSE): no further request parsing; `on_close` fires when
  // the peer goes away or close() is called.
  void start_streaming(std::function<void()> on_close);
  bool streaming() const { return streaming_; }

  // Keeps the object alive across async callbacks even if the socket closes meanwhile
  // (prefer ConnRef, which cannot forget the release).
  void hold() { ++holds_; }
  void release();

  void close();
  // close() without running the on_close callback: for tearing a worker down after the
  // objects such callbacks point at may already be gone.
  void close_silently() {
    on_close_ = nullptr;
    close();
  }

  // Remote address (for tracing / logs).
  std::string peer() const;
  // Idle = no request in progress and nothing buffered either way.
  bool idle() const { return !parked_ && in_.empty() && unsent() == 0; }
  // No response owed and nothing queued to send (a partial request may be buffered).
  bool quiet() const { return !parked_ && unsent() == 0; }
  int64_t last_active_ms() const { return last_active_ms_; }
  // Bytes queued for this connection that the socket has not taken yet.
  size_t unsent() const { return out_.size() - out_off_ + stable_len_; }
  // Bytes the socket has taken over the connection's life.
  uint64_t bytes_sent() const { return sent_total_; }
  // The state published in the loop's activity record: flag bits, buffered input, unsent
  // output and the current read loop's iteration count; describe_state() decodes it.
  uint64_t state_bits(uint32_t iterations) const;
  static std::string describe_state(uint64_t bits);

 private:
  void on_readable(bool peer_closed);
  void on_writable();
  // Parses and dispatches buffered requests; returns false if the connection closed.
  bool process(const char* data, size_t len, size_t* consumed);
  void flush();
  // Copies a pending send_stable() view into out_ (before anything else is queued).
  void materialize() {
    if (stable_) {
      out_.append(stable_, stable_len_);
      stable_ = nullptr;
      stable_len_ = 0;
    }
  }
  void update_interest();
  void error_response(int status);

  Worker* worker_;
  int fd_;
  uint64_t id_;
  std::string in_;   // unconsumed input carried across reads
  std::string out_;  // unsent output
  size_t out_off_ = 0;
  // a send_stable() response not copied yet (out_ is empty while it is pending)
  const char* stable_ = nullptr;
  size_t stable_len_ = 0;
  uint64_t sent_total_ = 0;
  bool closed_ = false;
  bool parked_ = false;
  bool streaming_ = false;
  bool close_after_flush_ = false;
  bool want_write_ = false;
  bool reading_ = true;
  bool in_process_ = false;  // inside process(): batch writes instead of sending eagerly
  bool continue_sent_ = false;  // "100 Continue" already sent for the pending request
  // Edge-triggered sockets stay registered for input while a request is parked (no
  // epoll_ctl per parked request): an edge that arrives meanwhile, or input left unread when
  // the request parked, is remembered here and read when the response completes.
  bool read_pending_ = false;
  bool peer_closed_pending_ = false;
  int holds_ = 0;
  int64_t last_active_ms_ = 0;
  std::function<void()> on_close_;
  // intrusive per-worker list (for draining on shutdown)
  Connection* prev_ = nullptr;
  Connection* next_ = nullptr;
  friend class Worker;
};

class RequestHandler {
 public:
  virtual ~RequestHandler() = default;
  // Runs on the worker thread. Must either send exactly one complete response with
  // c.send() (and c.close_after_response() when !r.keep_alive) or call c.park().
  virtual void on_request(Connection& c, const Request& r) = 0;
  // Per-worker setup/teardown on the worker thread.
  virtual void on_worker_start(Worker& w) {}
  virtual void on_worker_stop(Worker& w) {}
  // Response for protocol errors (400/414/431/501/505); default is a minimal empty response.
  virtual std::string error_response(int status);
};

struct ServerOptions {
  std::string host = "0.0.0.0";
  int port = 8080;
  int threads = 1;
  std::vector<int> cpus;          // pin worker i to cpus[i % size]; empty = no pinning
  bool reuseport_accept = false;  // per-worker SO_REUSEPORT listeners instead of round-robin
  // With reuseport_accept and pinned workers: the CPU each worker's listener names as its
  // incoming CPU, so the kernel's group selection sends a connection to the worker (of this
  // replica or of another one in the group) that expects clients on that CPU.
  enum class ReuseportCpu { kNone, kSelf, kSibling } reuseport_cpu = ReuseportCpu::kNone;
  int backlog = 4096;
  size_t read_chunk = 64 * 1024;
  int busy_poll_us = 0;  // see EventLoop::set_busy_poll_us
  bool busy_poll_auto = false;  // adaptive spinning, see EventLoop::set_busy_poll_auto
  int busy_poll_pause = 0;  // see EventLoop::set_busy_poll_pause
  bool edge_triggered = true;  // EPOLLET on connection sockets (--epoll-lt turns it off)
  bool profile = false;  // per-stage latency histograms (SURVEY.md §5.1 --profile)
  // Close keep-alive connections idle this long (Undertow/WildFly no-request-timeout is
  // 60 s by default); 0 disables.
  int idle_timeout_ms = 60000;
  size_t max_connections = 0;  // per replica; 0 = unlimited (bounded by RLIMIT_NOFILE)
  // Steer each accepted connection to a worker in the L3 domain where its packets arrive
  // (SO_INCOMING_CPU), when workers are pinned; otherwise plain round-robin.
  bool steer_l3 = true;
  // Each worker counts its own user-space instructions and cycles (core/perfcount.h), exported
  // on /metrics when the host allows it (--no-perf-counters turns it off).
  bool perf_counters = true;
  // Each worker asks the scheduler for this time slice (us; 0 = the kernel's default): see
  // set_current_thread_slice_us in core/affinity.h. --sched-slice-us.
  int sched_slice_us = 0;
};

// Per-worker stage timings (ns) collected with --profile; read after the workers stop.
struct StageProfile {
  // accept = accept4() until the owning worker adopts the socket (includes the cross-worker
  // hand-off); batch = requests handled per recv().
  Histogram accept, recv, parse, handle, send, batch;
};

class Worker {
 public:
  Worker(Server* s, int index);
  // Runs after the worker's thread has stopped: connections still open (a drain that timed
  // out) are closed without their callbacks and freed with the loop.
  ~Worker();
  EventLoop& loop() { return loop_; }
  const EventLoop& loop() const { return loop_; }
  int index() const { return index_; }
  Server& server() { return *server_; }
  WorkerStats& stats() { return stats_; }
  RequestHandler& handler();
  // Shared scratch receive buffer (connections copy out only leftovers).
  char* scratch() { return scratch_.data(); }
  size_t scratch_size() const { return scratch_.size(); }
  // Current Date header value (29 bytes) and a counter bumped whenever it changes.
  const char* date() const { return date_; }
  uint64_t date_version() const { return date_version_; }
  // Accepted fd handed over from the acceptor (thread-safe).
  // accepted_ns: mono_ns() taken before accept4 (0 when not profiling).
  void adopt(int fd, int64_t accepted_ns = 0);
  void adopt_here(int fd, int64_t accepted_ns = 0);
  size_t open_connections() const { return nconns_; }
  void on_connection_closed(Connection* c);
  // Shutdown drain, on the worker thread: closes streaming connections, and idle ones (no
  // request in progress, nothing buffered) with nothing read or written for grace_ms. A
  // connection used just before the drain began is likely to carry one more request, which
  // is answered with `Connection: close` instead of racing a close against it.
  void close_idle_connections(int64_t grace_ms = 0);
  // Closes keep-alive connections idle for longer than the idle timeout.
  void sweep_idle();
  // Per-worker slot for the application.
  void* app_data = nullptr;
  StageProfile* profile() { return profile_.get(); }
  // The worker thread's own user-space instructions and cycles (open once it runs).
  const ThreadCounters& counters() const { return counters_; }
  // the slice the scheduler reports for the worker's thread (us; 0 unknown)
  long sched_slice_us() const { return slice_us_.load(std::memory_order_relaxed); }

 private:
  friend class Server;
  void tick();
  ThreadCounters counters_;
  Server* server_;
  int index_;
  EventLoop loop_;
  WorkerStats stats_;
  std::vector<char> scratch_;
  char date_[29];
  int64_t date_sec_ = 0;
  int64_t next_date_check_ms_ = 0;  // loop time of the next Date refresh (Worker::tick)
  uint64_t date_version_ = 0;
  uint64_t next_conn_id_ = 1;
  size_t nconns_ = 0;
  Connection* conns_ = nullptr;
  std::unique_ptr<StageProfile> profile_;
  std::shared_ptr<std::function<void()>> sweep_;  // idle-timeout sweeper (owned here)
  std::atomic<long> slice_us_{0};
  std::atomic<int> tid_{0};  // kernel id of the worker's thread while it runs (stall reports)
};

// Counted reference to a Connection for asynchronous callbacks (aloha calls, SSE tickers):
// holds it while any copy exists, so a callback that is destroyed without running — a
// timer dropped at shutdown, say — still releases it. Copies and destruction happen on the
// connection's worker thread, or after the worker has stopped.
class ConnRef {
 public:
  ConnRef() = default;
  explicit ConnRef(Connection* c) : c_(c) {
    if (c_) c_->hold();
  }
  ConnRef(const ConnRef& o) : c_(o.c_) {
    if (c_) c_->hold();
  }
  ConnRef(ConnRef&& o) noexcept : c_(o.c_) { o.c_ = nullptr; }
  ConnRef& operator=(const ConnRef&) = delete;
  ConnRef& operator=(ConnRef&&) = delete;
  ~ConnRef() {
    if (c_) c_->release();
  }
  Connection* operator->() const { return c_; }
  Connection* get() const { return c_; }

 private:
  Connection* c_ = nullptr;
};

class Server {
 public:
  Server(ServerOptions opts, RequestHandler* handler);
  ~Server();
  // Binds listeners; false with *err on failure.
  bool bind(std::string* err);
  int port() const { return port_; }
  // Starts worker threads (returns immediately).
  void start();
  // Termination, phase 1 (hola --shutdown-delay-ms): readiness fails (the application
  // answers its health route with 503) and every response closes its connection, while the
  // listener still accepts, so a client routed here before the endpoint removal has
  // propagated is still served, and kept-alive clients reconnect elsewhere one response at
  // a time instead of racing a close.
  void begin_termination() {
    terminating_.store(true);
    closing_.store(true);
  }
  // Phase 2: stops accepting, lets workers finish in-flight responses for up to drain_ms
  // (each kept-alive connection's next response says `Connection: close`), then stops.
  void shutdown(int drain_ms);
  void join();
  size_t num_workers() const { return workers_.size(); }
  Worker& worker(size_t i) { return *workers_[i]; }
  RequestHandler& handler() { return *handler_; }
  const ServerOptions& options() const { return opts_; }
  bool draining() const { return draining_.load(std::memory_order_relaxed); }
  bool terminating() const { return terminating_.load(std::memory_order_relaxed); }
  // Responses close their connections (terminating or draining).
  bool closing() const { return closing_.load(std::memory_order_relaxed); }
  uint64_t total_requests() const;
  bool steering() const { return !domain_workers_.empty() || !core_workers_.empty(); }
  size_t open_connections() const { return open_.load(std::memory_order_relaxed); }
  // JSON summary of the --profile histograms (call after join()).
  std::string profile_json() const;
  // Worker i's activity record, decoded (any thread, any time).
  std::string activity(size_t i) const;
  // A worker that stopped answering: its activity, whether its loop passes advance over the
  // next 100 ms, and (with_stack) its stack captured by signal. Any thread but worker i's.
  std::string stall_report(size_t i, bool with_stack);
  // The same for several workers at once (one 100 ms window; stacks within a 2 s budget).
  std::vector<std::string> stall_reports(const std::vector<size_t>& which, bool with_stack);

  // Where each accepted connection's client ran (SO_INCOMING_CPU: for loopback clients the
  // CPU of the sending thread) relative to the pinned worker that serves it.
  enum Locality { kSameCore = 0, kSameL3, kSameSocket, kCrossSocket, kUnknown, kNumLocality };
  static const char* locality_name(int l);
  uint64_t locality(int l) const { return locality_[l].load(std::memory_order_relaxed); }

  // Accept steering's balance rule: may worker w (live connections counts[w]) take one more
  // steered connection? With three or more workers, unless it already holds twice its fair
  // share + 8: a bound relative to the total, so that clients of one L3 opening theirs before
  // those of another do not push the late ones off their own L3 for the whole run
  // (profiles/round5/02_chain_modes). With one or two workers that bound refuses nothing
  // (counts[w] <= total always), so there the worker may lead the least loaded one by at most
  // max(8, total / n): two workers in two L3s fed by clients of one L3 keep a 3:1 split at
  // worst instead of one worker taking every connection.
  static bool steering_within_share(const int32_t* counts, size_t n, size_t w) {
    int64_t total = 0, least = INT64_MAX;
    for (size_t i = 0; i < n; ++i) {
      total += counts[i];
      least = counts[i] < least ? counts[i] : least;
    }
    if (n >= 3) return counts[w] <= 2 * total / int64_t(n) + 8;
    const int64_t slack = total / int64_t(n) > 8 ? total / int64_t(n) : 8;
    return counts[w] - least <= slack;
  }

 private:
  struct Acceptor : EventLoop::Handler {
    Server* server;
    Worker* worker;
    int fd;
    bool paused = false;  // at the fd limit: logged once per episode, cleared by the next accept
    void on_event(uint32_t) override;
  };
  ServerOptions opts_;
  RequestHandler* handler_;
  std::vector<std::unique_ptr<Worker>> workers_;
  std::vector<std::unique_ptr<Acceptor>> acceptors_;
  std::vector<std::thread> threads_;
  std::atomic<bool> draining_{false};
  std::atomic<bool> terminating_{false};
  std::atomic<bool> closing_{false};
  std::atomic<uint64_t> rr_{0};
  std::atomic<size_t> open_{0};
  int port_ = 0;
  // L3-domain steering state (built in the constructor from opts_.cpus).
  Worker* pick_worker(int fd);
  std::vector<std::pair<int, std::vector<size_t>>> domain_workers_;  // (l3 id, worker indices)
  std::vector<std::pair<int, size_t>> core_workers_;  // (physical core, worker index), one per core
  std::unique_ptr<std::atomic<uint32_t>[]> domain_rr_;
  std::unique_ptr<std::atomic<int32_t>[]> assigned_;  // live connections per worker
  std::atomic<uint64_t> steered_core_{0}, steered_{0}, unsteered_{0};  // accept steering outcomes
  std::atomic<uint64_t> locality_[kNumLocality] = {};
  // Counts the client/worker relation of an accepted connection (client_cpu -1 = unknown).
  void note_locality(int client_cpu, size_t worker);
  static int incoming_cpu(int fd);
  friend class Worker;
};

}  // namespace hola::http
