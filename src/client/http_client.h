// Non-blocking, per-worker, keep-alive HTTP/1.1 client pool (SURVEY.md T7/T8 role).
//
// The reference builds a *new* Apache HttpClient (and leaks it) for every chaining request
// (HolaResource.java:98-102). Here every worker owns one pool of kept-alive connections to
// aloha, driven by the worker's own event loop — no extra threads, no per-request client.
#pragma once
#include <netinet/in.h>

#include <atomic>
#include <cstdint>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "client/url.h"
#include "core/loop.h"

namespace hola::client {

// Background DNS resolution so a worker never blocks in getaddrinfo.
class AddressCache {
 public:
  AddressCache(std::string host, int port, int refresh_ms = 5000);
  ~AddressCache();
  // Starts the resolver thread and waits up to first_wait_ms for its first answer: a name
  // that resolves at once (an IP literal, /etc/hosts, a healthy DNS) is ready before the
  // first call, while an unreachable DNS server delays start-up by at most that long.
  void start(int first_wait_ms = 1000);
  // Does not wait for a getaddrinfo() that is stuck: the thread is left to finish on its own
  // (it shares the state it writes, so it outlives this object safely).
  void stop();
  // false when the host has not (yet) resolved.
  bool get(sockaddr_storage* out, socklen_t* len, std::string* err) const;
  void resolve_now();  // synchronous (tests)

 private:
  struct State;
  static void resolve(State& s);
  std::shared_ptr<State> st_;
  int refresh_ms_;
  std::thread th_;
};

struct ClientResult {
  bool ok = false;      // a complete HTTP response was received
  int status = 0;
  std::string reason;   // reason phrase of the status line ("OK")
  std::string body;
  std::string error;    // "<ExceptionClass>: <message>" when !ok
  // !ok only: the failure happened before a complete response head arrived (connect, write,
  // or reading the status line/headers). Apache HttpClient throws an IOException from
  // execute() there, which Feign turns into a RetryableException (SynchronousMethodHandler
  // errorExecuting); a failure while reading the body is a non-retryable FeignException.
  bool retryable = false;
  // ok only: a parseable Retry-After header, as milliseconds from now (negative for a date
  // in the past). Feign's ErrorDecoder.Default makes any non-2xx response carrying it a
  // RetryableException.
  bool has_retry_after = false;
  int64_t retry_after_ms = 0;
  // Back to a default result, keeping the strings' capacity (the pool reuses one result for
  // every response it reads, so a body costs no allocation).
  void clear() {
    ok = retryable = has_retry_after = false;
    status = 0;
    retry_after_ms = 0;
    reason.clear();
    body.clear();
    error.clear();
  }
};

// Retry-After value (delta-seconds or RFC 1123 date) as milliseconds from now_ms (wall
// clock, negative for a date in the past); false when it cannot be parsed.
bool parse_retry_after(std::string_view v, int64_t now_ms, int64_t* out_ms);

// The pool's response parser on its own (tests): one response from the front of `in`;
// 1 = complete (*consumed bytes), 0 = need more, -1 = malformed.
int parse_response_probe(std::string_view in, bool eof, ClientResult* r, bool* close, size_t* consumed,
                         bool* head_ok);

class ClientPool {
 public:
  using Callback = std::function<void(ClientResult&&)>;
  // `transport_retries` (optional, shared by the pools of all workers) counts requests
  // re-sent on a fresh connection after an I/O error (DefaultHttpRequestRetryHandler role).
  ClientPool(EventLoop& loop, Url target, AddressCache* addr, size_t max_idle = 64,
             std::atomic<uint64_t>* transport_retries = nullptr);
  ~ClientPool();
  // Starts GET <path>; `cb` runs exactly once on the loop thread unless cancel() is called
  // first. Returns a request id.
  uint64_t get(const std::string& path, const std::string& extra_headers, Callback cb);
  // Abandons a request (e.g. on timeout): its connection is closed, its callback dropped.
  void cancel(uint64_t id);
  // Feign's Request.Options on this pool: a connect that has not completed after
  // `connect_ms` fails as ConnectTimeoutException, and, while *read_ms > 0, a request without
  // a complete response *read_ms after it started fails as SocketTimeoutException. Both are
  // IOExceptions to Feign (retried by its Retryer) but not to HttpClient's retry handler.
  void set_timeouts(int connect_ms, const std::atomic<int>* read_ms) {
    connect_timeout_ms_ = connect_ms;
    read_timeout_ms_ = read_ms;
  }
  size_t idle_connections() const { return idle_.size(); }
  uint64_t connections_opened() const { return opened_; }
  // HTTP/1.1 pipelining (opt-in; Apache HttpClient, the reference's transport, never
  // pipelines): up to `depth` requests in flight per connection, and the requests queued on a
  // connection during one event-loop batch go out in one send(). depth 1 = off.
  void set_pipeline(int depth) { pipeline_ = depth < 1 ? 1 : depth; }

 private:
  struct Conn;
  friend struct Conn;
  struct PConn;
  friend struct PConn;
  // `req` (moved in) is the request, or null when it is already in c->out.
  void start_on(Conn* c, uint64_t id, std::string* req, Callback cb, bool reused);
  void finish(Conn* c, ClientResult&& r, bool reusable);
  void destroy(Conn* c);
  std::string build_request(const std::string& path, const std::string& extra) const;
  void build_request_into(std::string* out, const std::string& path, const std::string& extra) const;
  std::string connect_error(int err) const;

  EventLoop& loop_;
  Url target_;
  AddressCache* addr_;
  size_t max_idle_;
  std::vector<Conn*> idle_;
  // Requests in flight on plain connections, by id. An id made by get() names a slot of a
  // table: (generation << 32) | slot, so finding a request is an index and a compare, with no
  // hashing and no allocation (a hash map cost 2-4 % of hola A's CPU on the chaining path,
  // profiles/round4/03_chainab). Ids of pipelined requests carry kPipeBit; the few of those
  // re-sent on plain connections after their pipelined one failed are kept in a map.
  static constexpr uint64_t kPipeBit = uint64_t(1) << 63;
  struct Slot {
    Conn* conn = nullptr;
    uint32_t gen = 1;  // 1 .. 2^31-1: no id is 0 (callers use 0 for "no request")
  };
  std::vector<Slot> slots_;
  std::vector<uint32_t> free_slots_;
  std::unordered_map<uint64_t, Conn*> resent_;
  uint64_t new_id();                        // a free slot's id (get())
 public:
  // A slot's next generation. It wraps within 31 bits (bit 63 of an id is kPipeBit) and skips
  // 0: at 200 k calls/s on one worker a slot reused LIFO wraps 2^31 in about three hours, and
  // slot 0 at generation 0 would hand out id 0.
  static uint32_t next_generation(uint32_t g) {
    g = (g + 1) & 0x7fffffffu;
    return g ? g : 1;
  }

 private:
  void set_active(uint64_t id, Conn* c);   // the connection carrying request `id`
  Conn* active(uint64_t id) const;          // null once finished or cancelled
  void release(uint64_t id);                // finished or cancelled: the id is dead
  // The result every plain connection parses its responses into (see ClientResult::clear).
  // A callback only reads it before returning, and no read runs inside a callback.
  ClientResult scratch_;
  uint64_t next_id_ = 1;
  uint64_t opened_ = 0;
  std::string host_header_;
  // "GET <path> HTTP/1.1\r\nHost: ...\r\n...keep-alive\r\n" for the last path asked for (the
  // aloha call always asks for the same one): a request is then three appends, not seven.
  mutable std::string head_path_, head_;
  std::atomic<uint64_t>* transport_retries_;
  int connect_timeout_ms_ = 0;
  const std::atomic<int>* read_timeout_ms_ = nullptr;
  uint64_t next_serial_ = 1;  // tells a Conn from a later one at the same address
  // Connect and read timeouts each have one delay, so deadlines of one kind come due in the
  // order they were armed: a FIFO per kind with one loop timer for its front replaces a timer
  // per request (which would hold rate x timeout entries, since a timer outlives the request
  // it guards). Entries of finished requests are dropped from the front as requests finish,
  // so a FIFO holds about as many entries as there are requests in flight.
  struct Deadline {
    int64_t at_ms;
    uint64_t id, serial;
  };
  struct DeadlineFifo {
    std::deque<Deadline> q;
    EventLoop::TimerId timer = 0;
    int64_t timer_at = 0;  // deadline the armed timer fires for (0 = none armed)
    bool connect = false;  // connect timeouts (else read timeouts)
  };
  DeadlineFifo connect_fifo_, read_fifo_;
  // pipelined connections (pipeline_ > 1)
  struct PRef {
    PConn* conn;
    uint64_t serial;
  };
  int pipeline_ = 1;
  std::vector<PConn*> pconns_;
  std::unordered_map<uint64_t, PRef> pactive_;  // request id -> its pipelined connection
  std::vector<PConn*> dirty_;                   // requests queued this batch, not yet sent
  bool flush_scheduled_ = false;
  bool get_pipelined(uint64_t id, std::string& req, Callback& cb);
  PConn* open_pconn();
  void flush_dirty();
  void pdestroy(PConn* c);
  void check_head_of_line(PConn* c);
  double hol_budget_ = 10.0;     // head-of-line re-sends available (kHolResendBurst at start)
  uint64_t next_cid_ = 1;
  // Ends a pipelined connection. The request `failed` (if any: timed out, or answered with a
  // malformed or truncated response) fails with `why` (`failed_retryable` = no valid response
  // head arrived, so Feign may retry it). Every other request still waiting on the connection
  // is re-sent on a fresh one (HttpClient's transport retry: nothing came back for it), or,
  // with !resend_others (the connect failed, so nothing was sent), fails with `why` too.
  void pfail(PConn* c, const std::string& why, uint64_t failed = 0, bool failed_retryable = true,
             bool resend_others = true);
  void arm_read_deadline(uint64_t id, uint64_t serial);
  void resubmit(uint64_t id, std::string req, Callback cb, int tries, const std::string& why);
  bool live(const Deadline& d) const;
  void push_deadline(DeadlineFifo& f, int ms, uint64_t id, uint64_t serial);
  void arm(DeadlineFifo& f);
  void expire(DeadlineFifo& f);
  void pop_finished(DeadlineFifo& f);
};

}  // namespace hola::client
