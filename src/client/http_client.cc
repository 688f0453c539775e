#include "client/http_client.h"

#include <errno.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <ctime>

#include "core/clock.h"

#include "core/net.h"
#include "core/scan.h"
#include "http/parser.h"

namespace hola::client {

// ---------------------------------------------------------------- AddressCache

struct AddressCache::State {
  State(std::string h, int p) : host(std::move(h)), port(p) {}
  const std::string host;
  const int port;
  std::mutex mu;
  std::condition_variable cv;
  bool ok = false;
  bool answered = false;  // the first resolution has finished (either way)
  bool stop = false;
  bool done = false;  // the thread has left its loop
  sockaddr_storage addr{};
  socklen_t len = 0;
  std::string err;
};

namespace {
// Bounded wait against the system clock: libstdc++ implements steady-clock waits with
// pthread_cond_clockwait, which the toolchain's ThreadSanitizer does not intercept (it then
// reports a false "double lock"); pthread_cond_timedwait is intercepted.
template <class Pred>
bool wait_ms(std::condition_variable& cv, std::unique_lock<std::mutex>& g, int ms, Pred p) {
  return cv.wait_until(g, std::chrono::system_clock::now() + std::chrono::milliseconds(ms), p);
}
}  // namespace

AddressCache::AddressCache(std::string host, int port, int refresh_ms)
    : st_(std::make_shared<State>(std::move(host), port)), refresh_ms_(refresh_ms) {
  // Java's UnknownHostException message is the host name.
  st_->err = "UnknownHostException: " + st_->host;
}

AddressCache::~AddressCache() { stop(); }

void AddressCache::resolve(State& s) {
  sockaddr_storage ss{};
  socklen_t len = 0;
  std::string err;
  bool ok = resolve_host(s.host, s.port, &ss, &len, &err);
  std::lock_guard<std::mutex> g(s.mu);
  s.ok = ok;
  s.answered = true;
  if (ok) {
    s.addr = ss;
    s.len = len;
    s.err.clear();
  } else {
    s.err = "UnknownHostException: " + err;
  }
  s.cv.notify_all();
}

void AddressCache::resolve_now() { resolve(*st_); }

void AddressCache::start(int first_wait_ms) {
  std::shared_ptr<State> st = st_;
  const int refresh = refresh_ms_;
  th_ = std::thread([st, refresh] {
    std::unique_lock<std::mutex> g(st->mu);
    while (!st->stop) {
      g.unlock();
      resolve(*st);
      g.lock();
      wait_ms(st->cv, g, refresh, [&] { return st->stop; });
    }
    st->done = true;
    st->cv.notify_all();
  });
  std::unique_lock<std::mutex> g(st_->mu);
  wait_ms(st_->cv, g, first_wait_ms, [&] { return st_->answered; });
}

void AddressCache::stop() {
  if (!th_.joinable()) return;
  bool done;
  {
    std::unique_lock<std::mutex> g(st_->mu);
    st_->stop = true;
    st_->cv.notify_all();
    done = wait_ms(st_->cv, g, 200, [&] { return st_->done; });
  }
  // A thread inside getaddrinfo() cannot be interrupted, and joining it would make shutdown
  // wait for a DNS timeout: it holds its own reference to the state, sees `stop` when the
  // call returns and exits.
  if (done) th_.join();
  else th_.detach();
}

bool AddressCache::get(sockaddr_storage* out, socklen_t* len, std::string* err) const {
  std::lock_guard<std::mutex> g(st_->mu);
  if (!st_->ok) {
    if (err) *err = st_->err;
    return false;
  }
  *out = st_->addr;
  *len = st_->len;
  return true;
}

// ---------------------------------------------------------------- connection

constexpr int kTransportRetries = 3;  // DefaultHttpRequestRetryHandler(3, false)
// Interim 1xx responses accepted before a call's final response: the 64 KiB a response head
// may take. Past it the answer is treated as malformed.
constexpr size_t kMaxInterimBytes = 64 * 1024;
// How long the calls queued behind an abandoned pipelined call wait for its answer before they
// are re-sent on fresh connections (see ClientPool::cancel).
constexpr int kDrainGraceMs = 50;
// Those re-sends draw on a budget (Finagle's and Envoy's retry budgets): each pipelined call
// sent earns 0.1 of a re-send, up to a burst of 10. Calls are abandoned exactly when aloha is
// slower than the Hystrix timeout, and every re-send is a second GET to a downstream that is
// probably still working on the first, so without a bound the load on aloha would grow as it
// slows. Over budget, the calls stay on their connection until their answers arrive or their
// own deadlines abandon them; at most ~10 % more requests reach aloha.
constexpr double kHolResendPerCall = 0.1, kHolResendBurst = 10.0;

struct ClientPool::Conn final : EventLoop::Handler {
  enum State { kConnecting, kWriting, kReading, kIdle, kDead };
  ClientPool* pool = nullptr;
  int fd = -1;
  State st = kDead;
  std::string out;
  size_t off = 0;
  std::string in;
  uint64_t id = 0;
  uint64_t serial = 0;
  Callback cb;
  bool reused = false;  // went out on a kept-alive socket
  int tries = 0;        // transport re-executions so far (DefaultHttpRequestRetryHandler)
  bool head_ok = false;  // a complete, well-formed final status line + header block has arrived
  size_t interim_bytes = 0;  // interim 1xx responses read (and dropped) for the call in flight
  uint32_t interest = 0;

  void set_interest(uint32_t ev) {
    if (ev == interest) return;
    interest = ev;
    pool->loop_.mod(fd, ev, this);
  }
  // io = an I/O error (not a connect failure or a protocol error).
  void fail(const std::string& why, bool io = true);
  void on_event(uint32_t ev) override;
  void do_write();
  void do_read();
  // Returns 1 complete, 0 need more, -1 malformed; sets *keep on completion.
  int try_parse(ClientResult* r, bool* keep, bool eof);
};

// A pipelined connection (ClientPool::set_pipeline): requests queue in order, responses
// complete them in order.
struct ClientPool::PConn final : EventLoop::Handler {
  struct Pending {
    uint64_t id, serial;
    std::string req;  // kept for a re-send if the connection fails before the response
    Callback cb;
    int tries = 0;
    bool abandoned = false;  // cancelled (timed out): its response is read and dropped
  };
  ClientPool* pool = nullptr;
  int fd = -1;
  bool connecting = false, dead = false, dirty = false;
  bool draining = false;  // a call on it was abandoned: no new calls; closes once none waits
  bool drain_timer = false;  // the head-of-line check (ClientPool::cancel) is armed
  uint64_t cid = 0;          // tells this connection from a later one (timers look it up)
  std::string out, in;
  size_t off = 0;
  std::deque<Pending> q;
  size_t front_interim = 0;  // interim 1xx bytes read (and dropped) for the oldest request
  uint32_t interest = 0;

  void set_interest(uint32_t ev) {
    if (ev == interest) return;
    interest = ev;
    pool->loop_.mod(fd, ev, this);
  }
  void on_event(uint32_t ev) override;
  void do_write();
  void do_read();
};

void ClientPool::Conn::fail(const std::string& why, bool io) {
  // Apache HttpClient's DefaultHttpRequestRetryHandler (the default of the HttpClientBuilder
  // in HolaResource.java:98-102): an idempotent GET that hit an I/O error before its response
  // head (a stale kept-alive socket, a reset, EOF with no response) is re-executed at once
  // on a fresh connection, up to 3 times. Connect failures and protocol errors are not.
  if (io && !head_ok && st != kConnecting && tries < kTransportRetries) {
    ClientPool* p = pool;
    uint64_t rid = id;
    Callback c = std::move(cb);
    std::string r = std::move(out);
    const int t = tries + 1;
    if (p->transport_retries_) p->transport_retries_->fetch_add(1, std::memory_order_relaxed);
    p->destroy(this);  // the id stays live: start_on points it at the fresh connection
    auto* fresh = new Conn();
    fresh->pool = p;
    fresh->tries = t;
    p->start_on(fresh, rid, &r, std::move(c), false);
    return;
  }
  ClientResult res;
  res.ok = false;
  res.error = why;
  res.retryable = !head_ok;
  pool->finish(this, std::move(res), false);
}

void ClientPool::Conn::on_event(uint32_t ev) {
  if (st == kDead) return;
  if (st == kIdle) {
    // Anything on an idle connection is a close or junk: drop it.
    pool->idle_.erase(std::remove(pool->idle_.begin(), pool->idle_.end(), this), pool->idle_.end());
    pool->destroy(this);
    return;
  }
  if (st == kConnecting) {
    int soerr = 0;
    socklen_t sl = sizeof soerr;
    getsockopt(fd, SOL_SOCKET, SO_ERROR, &soerr, &sl);
    if (soerr != 0 || (ev & (EPOLLERR | EPOLLHUP))) {
      fail(pool->connect_error(soerr ? soerr : ECONNREFUSED), false);
      return;
    }
    st = kWriting;
    pool->arm_read_deadline(id, serial);
  }
  if (st == kWriting) {
    do_write();
    return;
  }
  if (st == kReading) do_read();
}

void ClientPool::Conn::do_write() {
  while (off < out.size()) {
    ssize_t w = ::send(fd, out.data() + off, out.size() - off, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN) {
        set_interest(EPOLLOUT);
        return;
      }
      fail(std::string("SocketException: ") + strerror(errno));
      return;
    }
    off += size_t(w);
  }
  st = kReading;
  set_interest(EPOLLIN | EPOLLRDHUP);
}

namespace {
// One response from the front of `in`: 1 = complete (*consumed bytes; *close when the
// connection cannot carry another response), 0 = need more, -1 = malformed. *head_ok is set
// once a well-formed status line and header block have arrived.
// Header name (before the colon) against a lower-case literal, a word at a time: letters
// compare case-insensitively (OR 0x20 at their positions only), every other byte exactly. A
// fold of every byte would also map CR (0x0d) onto '-' and control bytes onto digits, and
// the client does not check response header names for token characters first, so
// "Content\rLength" must not read as Content-Length. The words and fold masks are built at
// compile time from the literal (the last word overlaps the one before it, as read).
template <size_t N>
struct FieldName {
  static_assert(N - 1 >= 8, "names of 8 bytes or more");
  static constexpr size_t n = N - 1;
  static constexpr size_t kWords = (n + 7) / 8;
  uint64_t word[kWords] = {}, fold[kWords] = {};
  static constexpr size_t offset(size_t w) { return w + 1 < kWords ? 8 * w : n - 8; }
  constexpr FieldName(const char (&lit)[N]) {
    for (size_t w = 0; w < kWords; ++w)
      for (size_t i = 0; i < 8; ++i) {
        const char c = lit[offset(w) + i];
        word[w] |= uint64_t((unsigned char)c) << (8 * i);
        if (c >= 'a' && c <= 'z') fold[w] |= uint64_t(0x20) << (8 * i);
      }
  }
};

template <FieldName F>
inline bool field_is(std::string_view k) {
  if (k.size() != F.n) return false;
  for (size_t w = 0; w < F.kWords; ++w) {
    uint64_t x;
    memcpy(&x, k.data() + F.offset(w), 8);
    if ((x | F.fold[w]) != F.word[w]) return false;
  }
  return true;
}

std::string_view trim_ows(std::string_view v) {
  while (!v.empty() && (v.front() == ' ' || v.front() == '\t')) v.remove_prefix(1);
  while (!v.empty() && (v.back() == ' ' || v.back() == '\t')) v.remove_suffix(1);
  return v;
}

// Content-Length as HttpClient 4.5's LaxContentLengthStrategy reads it: the last header whose
// value parses as a Java long wins (a negative one means "to the close"), one that does not
// parse is skipped, none leaves *cl at -1. Values over the body cap stay over it.
void content_length(std::string_view v, int64_t* cl) {
  v = trim_ows(v);
  bool neg = false;
  if (!v.empty() && (v.front() == '+' || v.front() == '-')) {
    neg = v.front() == '-';
    v.remove_prefix(1);
  }
  if (v.empty() || v.size() > 19) return;
  int64_t x = 0;
  for (char d : v) {
    if (d < '0' || d > '9') return;
    if (x <= (1 << 20)) x = x * 10 + (d - '0');
  }
  *cl = neg ? -1 : x;
}

// Transfer-Encoding as HttpClient 4.5 reads the first such header: chunked when its last
// coding is "chunked" (RFC 9112 §6.1: chunked must be applied last); any other value means the
// body runs to the close, Content-Length notwithstanding.
bool last_coding_is_chunked(std::string_view v) {
  const size_t comma = v.rfind(',');
  std::string_view last = comma == std::string_view::npos ? v : v.substr(comma + 1);
  if (const size_t semi = last.find(';'); semi != std::string_view::npos) last = last.substr(0, semi);
  return http::iequals(trim_ows(last), "chunked");
}

int parse_one(std::string_view in, bool eof, ClientResult* r, bool* close, size_t* consumed, bool* head_ok,
              bool* interim) {
  // One pass over the head's lines (each newline found inline when the line is short,
  // core/scan.h): a find("\r\n\r\n") followed by a find("\r\n") and a find(':') per line
  // was a memchr call per candidate, most of this function's cycles (profiles/round4/
  // 14_user_cycles). Lines end in CRLF; a bare LF is accepted as HttpClient does.
  const char* s = in.data();
  const size_t n = in.size();
  auto need_more = [&] { return n > 64 * 1024 ? -1 : 0; };
  const char* nl = find_newline(s, n);
  if (!nl) return need_more();
  std::string_view head(s, size_t(nl - s));
  if (!head.empty() && head.back() == '\r') head.remove_suffix(1);
  if (head.size() < 12 || head.substr(0, 5) != "HTTP/") {
    // a status line may only be judged once it is complete
    return -1;
  }
  int status = 0;
  for (size_t k = 9; k < 12; ++k) {
    if (head[k] < '0' || head[k] > '9') return -1;
    status = status * 10 + (head[k] - '0');
  }
  if (status < 100) return -1;
  const bool http10 = head.substr(5, 3) == "1.0";
  int64_t cl = -1;
  bool chunked = false, te_seen = false;
  bool has_retry_after = false;
  int64_t retry_after_ms = 0;
  bool conn_close = http10;
  size_t p = size_t(nl - s) + 1;
  for (;;) {
    const char* e = find_newline(s + p, n - p);
    if (!e) return need_more();
    std::string_view line(s + p, size_t(e - (s + p)));
    p = size_t(e - s) + 1;
    if (!line.empty() && line.back() == '\r') line.remove_suffix(1);
    if (line.empty()) break;  // end of head
    // the colon, with the vector compare over the buffer from the line's start (a header
    // line is short: one compare instead of a memchr call per line)
    const char* c = find_byte<':'>(line.data(), n - size_t(line.data() - s));
    if (!c || c >= line.data() + line.size()) continue;
    const size_t colon = size_t(c - line.data());
    std::string_view k = line.substr(0, colon), v = line.substr(colon + 1);
    while (!v.empty() && (v.front() == ' ' || v.front() == '\t')) v.remove_prefix(1);
    switch (k.size()) {
      case 14:
        if (field_is<"content-length">(k)) content_length(v, &cl);
        break;
      case 17:
        if (field_is<"transfer-encoding">(k) && !te_seen) {
          te_seen = true;
          chunked = last_coding_is_chunked(v);
        }
        break;
      case 10:
        if (field_is<"connection">(k)) {
          if (http::iequals(v, "close")) conn_close = true;
          else if (http::iequals(v, "keep-alive")) conn_close = false;
        }
        break;
      case 11:
        if (field_is<"retry-after">(k)) has_retry_after = parse_retry_after(v, wall_us() / 1000, &retry_after_ms);
        break;
      default:
        break;
    }
  }
  if (te_seen && !chunked) cl = -1;  // another transfer coding: the body runs to the close
  r->reason.assign(head.size() > 13 && head[12] == ' ' ? head.substr(13) : std::string_view());
  r->has_retry_after = has_retry_after;
  r->retry_after_ms = retry_after_ms;
  *close = conn_close;
  size_t body = p;
  *interim = status < 200 && status != 101;
  // A final head: the server has answered, the call is no longer safe to send again. An
  // interim 1xx is not an answer: HttpClient 4.5's HttpRequestExecutor reads past it inside
  // execute(), and a connection that closes before the final head throws
  // NoHttpResponseException there, which the retry handler re-sends for an idempotent GET.
  if (!*interim) *head_ok = true;
  if (status == 204 || status == 304 || (status >= 100 && status < 200)) {
    r->status = status;
    *consumed = body;
    return 1;
  }
  if (chunked) {
    size_t used = 0;
    std::string out;
    http::Parse q = http::decode_chunked_body(in.data() + body, in.size() - body, &used, &out);
    if (q == http::Parse::kError) return -1;
    if (q == http::Parse::kIncomplete) return in.size() > (1 << 20) ? -1 : 0;
    r->status = status;
    r->body = std::move(out);
    *consumed = body + used;
    return 1;
  }
  if (cl >= 0) {
    if (cl > (1 << 20)) return -1;
    if (in.size() - body < size_t(cl)) return 0;
    r->status = status;
    r->body.assign(in.substr(body, size_t(cl)));
    *consumed = body + size_t(cl);
    return 1;
  }
  // close-delimited body
  if (!eof) return in.size() > (1 << 20) ? -1 : 0;
  r->status = status;
  r->body.assign(in.substr(body));
  *consumed = in.size();
  *close = true;
  return 1;
}

// parse_one() past any interim 1xx responses (100 Continue, 102 Processing, 103 Early Hints):
// a client must accept them before the final response even unasked (RFC 9110 §15.2), and
// HttpClient's request executor reads past every one. 101 ends the exchange (no upgrade here).
// When the final response is still incomplete (0), *consumed is the length of the interims
// before it, so the caller can drop them and never parse them again: re-parsing every interim
// on each read of a downstream that keeps sending them was quadratic.
int parse_response(std::string_view in, bool eof, ClientResult* r, bool* close, size_t* consumed, bool* head_ok) {
  size_t off = 0;
  for (;;) {
    bool interim = false;
    size_t used = 0;
    const int rc = parse_one(in.substr(off), eof, r, close, &used, head_ok, &interim);
    if (rc != 1) {
      *consumed = rc == 0 ? off : 0;
      return rc;
    }
    off += used;
    if (!interim) {
      *consumed = off;
      return 1;
    }
    r->clear();
  }
}
}  // namespace

int parse_response_probe(std::string_view in, bool eof, ClientResult* r, bool* close, size_t* consumed,
                         bool* head_ok) {
  return parse_response(in, eof, r, close, consumed, head_ok);
}

int ClientPool::Conn::try_parse(ClientResult* r, bool* keep, bool eof) {
  bool close = false;
  size_t consumed = 0;
  const int rc = parse_response(in, eof, r, &close, &consumed, &head_ok);
  // a response followed by stray bytes leaves a connection that cannot be reused
  if (rc == 1) *keep = !close && consumed == in.size();
  if (rc == 0 && consumed) {
    // interim responses before a final one still due: dropped, and bounded per call (the
    // 64 KiB a response head may take), so a downstream that sends nothing but 1xx fails
    // the call as malformed instead of holding it until the timeout
    interim_bytes += consumed;
    in.erase(0, consumed);
    if (interim_bytes > kMaxInterimBytes) return -1;
  }
  return rc;
}

void ClientPool::Conn::do_read() {
  char buf[16384];
  for (;;) {
    ssize_t n = ::recv(fd, buf, sizeof buf, 0);
    bool eof = false;
    if (n > 0) {
      in.append(buf, size_t(n));
      reused = false;
    } else if (n == 0) {
      eof = true;
    } else {
      if (errno == EINTR) continue;
      if (errno == EAGAIN) return;
      fail(std::string("SocketException: ") + strerror(errno));
      return;
    }
    ClientResult& r = pool->scratch_;
    r.clear();
    bool keep = false;
    int rc = try_parse(&r, &keep, eof);
    if (rc < 0) {
      fail("ClientProtocolException: malformed response", false);
      return;
    }
    if (rc == 1) {
      r.ok = true;
      pool->finish(this, std::move(r), keep && !eof);
      return;
    }
    if (eof) {
      fail(in.empty() ? "NoHttpResponseException: connection closed" : "TruncatedChunkException: premature EOF");
      return;
    }
    if (size_t(n) < sizeof buf) return;  // drained for now (level-triggered)
  }
}

// ---------------------------------------------------------------- pool

bool parse_retry_after(std::string_view v, int64_t now_ms, int64_t* out_ms) {
  while (!v.empty() && (v.back() == ' ' || v.back() == '\t')) v.remove_suffix(1);
  if (v.empty()) return false;
  bool digits = true;
  int64_t secs = 0;
  for (char d : v) {
    if (d < '0' || d > '9') {
      digits = false;
      break;
    }
    secs = std::min<int64_t>(secs * 10 + (d - '0'), int64_t(1) << 40);
  }
  if (digits) {
    *out_ms = secs * 1000;
    return true;
  }
  // RFC 1123 date, e.g. "Wed, 21 Oct 2015 07:28:00 GMT" (Feign's RetryAfterDecoder format).
  std::string s(v);
  tm t{};
  const char* end = strptime(s.c_str(), "%a, %d %b %Y %H:%M:%S GMT", &t);
  if (!end || *end) return false;
  *out_ms = int64_t(timegm(&t)) * 1000 - now_ms;
  return true;
}

std::string ClientPool::connect_error(int err) const {
  // Apache HttpClient 4.5 wraps a refused/failed connect as HttpHostConnectException.
  return "HttpHostConnectException: Connect to " + target_.host + ":" + std::to_string(target_.port) + " failed: " + strerror(err);
}

ClientPool::ClientPool(EventLoop& loop, Url target, AddressCache* addr, size_t max_idle,
                       std::atomic<uint64_t>* transport_retries)
    : loop_(loop), target_(std::move(target)), addr_(addr), max_idle_(max_idle), transport_retries_(transport_retries) {
  connect_fifo_.connect = true;
  host_header_ = target_.host;
  if (target_.port != 80) host_header_ += ":" + std::to_string(target_.port);
}

ClientPool::~ClientPool() {
  for (PConn* c : pconns_) {
    if (c->fd >= 0) {
      loop_.del(c->fd);
      ::close(c->fd);
    }
    delete c;
  }
  for (DeadlineFifo* f : {&connect_fifo_, &read_fifo_})
    if (f->timer) loop_.cancel_timer(f->timer);
  for (Conn* c : idle_) {
    if (c->fd >= 0) ::close(c->fd);
    delete c;
  }
  auto drop = [this](Conn* c) {
    if (c->fd >= 0) {
      loop_.del(c->fd);
      ::close(c->fd);
    }
    delete c;
  };
  for (Slot& sl : slots_)
    if (sl.conn) drop(sl.conn);
  for (auto& [id, c] : resent_) drop(c);
}

std::string ClientPool::build_request(const std::string& path, const std::string& extra) const {
  std::string r;
  build_request_into(&r, path, extra);
  return r;
}

void ClientPool::build_request_into(std::string* out, const std::string& path, const std::string& extra) const {
  // Into a connection's own buffer: a kept-alive connection reuses its capacity, so the
  // request costs no allocation.
  if (path != head_path_ || head_.empty()) {
    head_path_ = path;
    head_ = "GET " + path + " HTTP/1.1\r\nHost: " + host_header_ + "\r\nAccept: application/json\r\nConnection: keep-alive\r\n";
  }
  std::string& r = *out;
  r.clear();
  r.reserve(head_.size() + extra.size() + 2);
  r += head_;
  r += extra;
  r += "\r\n";
}

uint64_t ClientPool::new_id() {
  uint32_t s;
  if (!free_slots_.empty()) {
    s = free_slots_.back();
    free_slots_.pop_back();
  } else {
    s = uint32_t(slots_.size());
    slots_.emplace_back();
  }
  return uint64_t(slots_[s].gen) << 32 | s;
}

void ClientPool::set_active(uint64_t id, Conn* c) {
  if (id & kPipeBit) resent_[id] = c;
  else slots_[uint32_t(id)].conn = c;
}

ClientPool::Conn* ClientPool::active(uint64_t id) const {
  if (id & kPipeBit) {
    auto it = resent_.find(id);
    return it == resent_.end() ? nullptr : it->second;
  }
  const uint32_t s = uint32_t(id);
  if (s >= slots_.size() || slots_[s].gen != uint32_t(id >> 32)) return nullptr;
  return slots_[s].conn;
}

void ClientPool::release(uint64_t id) {
  if (id & kPipeBit) {
    resent_.erase(id);
    return;
  }
  const uint32_t s = uint32_t(id);
  if (s >= slots_.size() || slots_[s].gen != uint32_t(id >> 32)) return;
  slots_[s].conn = nullptr;
  slots_[s].gen = next_generation(slots_[s].gen);  // a late timer or cancel with the old id finds nothing
  free_slots_.push_back(s);
}

uint64_t ClientPool::get(const std::string& path, const std::string& extra_headers, Callback cb) {
  if (pipeline_ > 1) {
    const uint64_t pid = kPipeBit | next_id_++;
    std::string req = build_request(path, extra_headers);
    if (get_pipelined(pid, req, cb)) return pid;
  }
  const uint64_t id = new_id();
  const bool reused = !idle_.empty();
  Conn* c;
  if (reused) {
    c = idle_.back();
    idle_.pop_back();
  } else {
    c = new Conn();
    c->pool = this;
  }
  build_request_into(&c->out, path, extra_headers);
  start_on(c, id, nullptr, std::move(cb), reused);
  return id;
}

bool ClientPool::live(const Deadline& d) const {
  if (const Conn* c = active(d.id)) return c->serial == d.serial;
  auto pt = pactive_.find(d.id);
  return pt != pactive_.end() && pt->second.serial == d.serial;
}

void ClientPool::push_deadline(DeadlineFifo& f, int ms, uint64_t id, uint64_t serial) {
  const Deadline d{mono_ms() + ms, id, serial};
  if (f.q.empty() || f.q.back().at_ms <= d.at_ms) {
    f.q.push_back(d);
  } else {
    // The timeout was shortened (a config reload): keep the FIFO in deadline order.
    auto it = std::upper_bound(f.q.begin(), f.q.end(), d.at_ms,
                               [](int64_t at, const Deadline& x) { return at < x.at_ms; });
    f.q.insert(it, d);
  }
  arm(f);
}

void ClientPool::arm(DeadlineFifo& f) {
  if (f.q.empty()) return;
  const int64_t at = f.q.front().at_ms;
  if (f.timer_at != 0 && f.timer_at <= at) return;
  if (f.timer) loop_.cancel_timer(f.timer);
  f.timer_at = at;
  DeadlineFifo* fp = &f;
  f.timer = loop_.add_timer(at - mono_ms(), [this, fp] {
    fp->timer = 0;
    fp->timer_at = 0;
    expire(*fp);
  });
}

void ClientPool::expire(DeadlineFifo& f) {
  const int64_t now = mono_ms();
  while (!f.q.empty()) {
    const Deadline d = f.q.front();
    if (!live(d)) {
      f.q.pop_front();
      continue;
    }
    if (d.at_ms > now) break;
    f.q.pop_front();
    if (auto pt = pactive_.find(d.id); pt != pactive_.end()) {
      // Pipelined: the responses behind this one cannot overtake it, so the connection ends;
      // this request fails with the timeout, the others are re-sent on fresh connections.
      PConn* pc = pt->second.conn;
      if (!f.connect)
        pfail(pc, "SocketTimeoutException: Read timed out", d.id);
      else if (pc->connecting)
        pfail(pc, "ConnectTimeoutException: Connect to " + target_.host + ":" + std::to_string(target_.port) +
                      " failed: connect timed out", 0, true, false);
      continue;
    }
    Conn* c = active(d.id);
    // fail() runs the callback, which may start (and push deadlines for) further requests
    if (f.connect) {
      if (c->st == Conn::kConnecting)
        c->fail("ConnectTimeoutException: Connect to " + target_.host + ":" + std::to_string(target_.port) +
                    " failed: connect timed out",
                false);
    } else if (c->st == Conn::kWriting || c->st == Conn::kReading) {
      c->fail("SocketTimeoutException: Read timed out", false);
    }
  }
  arm(f);
}

void ClientPool::pop_finished(DeadlineFifo& f) {
  while (!f.q.empty() && !live(f.q.front())) f.q.pop_front();
}

void ClientPool::start_on(Conn* c, uint64_t id, std::string* req, Callback cb, bool reused) {
  c->id = id;
  c->serial = next_serial_++;
  c->cb = std::move(cb);
  if (req) c->out = std::move(*req);  // else the caller built it in c->out
  c->off = 0;
  c->in.clear();
  c->reused = reused;
  c->head_ok = false;
  c->interim_bytes = 0;
  set_active(id, c);
  if (reused) {
    c->st = Conn::kWriting;
    arm_read_deadline(id, c->serial);
    c->do_write();
    return;
  }
  sockaddr_storage ss{};
  socklen_t len = 0;
  std::string err;
  if (!addr_ || !addr_->get(&ss, &len, &err)) {
    // Report asynchronously: callers expect the callback after get() returns.
    c->st = Conn::kDead;
    loop_.add_timer(0, [this, id, err] {
      Conn* c = active(id);
      if (!c) return;
      ClientResult r;
      r.error = err;
      r.retryable = true;  // UnknownHostException is an IOException
      finish(c, std::move(r), false);
    });
    return;
  }
  bool inprog = false;
  c->fd = connect_nonblocking(ss, len, &inprog);
  if (c->fd < 0) {
    std::string e = connect_error(errno);
    c->st = Conn::kDead;
    loop_.add_timer(0, [this, id, e] {
      Conn* c = active(id);
      if (!c) return;
      ClientResult r;
      r.error = e;
      r.retryable = true;
      finish(c, std::move(r), false);
    });
    return;
  }
  ++opened_;
  c->interest = EPOLLOUT;
  loop_.add(c->fd, EPOLLOUT, c);
  c->st = inprog ? Conn::kConnecting : Conn::kWriting;
  if (inprog && connect_timeout_ms_ > 0) push_deadline(connect_fifo_, connect_timeout_ms_, id, c->serial);
  if (!inprog) {
    arm_read_deadline(id, c->serial);
    c->do_write();
  }
}

void ClientPool::arm_read_deadline(uint64_t id, uint64_t serial) {
  // Feign's read timeout runs once the socket is connected (a connect has its own timeout):
  // armed when the request starts going out, never while the connect is still pending, so a
  // slow connect cannot leave the request unguarded afterwards.
  if (!read_timeout_ms_) return;
  const int rt = read_timeout_ms_->load(std::memory_order_relaxed);
  if (rt > 0) push_deadline(read_fifo_, rt, id, serial);
}

void ClientPool::finish(Conn* c, ClientResult&& r, bool reusable) {
  release(c->id);
  if (!read_fifo_.q.empty()) pop_finished(read_fifo_);
  if (!connect_fifo_.q.empty()) pop_finished(connect_fifo_);
  Callback cb = std::move(c->cb);
  c->cb = nullptr;
  // With pipelining on, new requests never take plain idle connections (only re-sends use
  // plain ones), so keeping them would only hold sockets open.
  if (reusable && c->fd >= 0 && idle_.size() < max_idle_ && pipeline_ <= 1) {
    c->st = Conn::kIdle;
    c->in.clear();
    c->set_interest(EPOLLIN | EPOLLRDHUP);
    idle_.push_back(c);
  } else {
    destroy(c);
  }
  if (cb) cb(std::move(r));
}

void ClientPool::destroy(Conn* c) {
  if (c->fd >= 0) {
    loop_.del(c->fd);
    ::close(c->fd);
    c->fd = -1;
  }
  c->st = Conn::kDead;
  c->cb = nullptr;
  loop_.retire(c);
}

void ClientPool::cancel(uint64_t id) {
  if (auto pt = pactive_.find(id); pt != pactive_.end()) {
    // Abandoned (its Hystrix timeout fired) on a shared connection. Aloha already has the
    // calls queued behind it, so re-sending them would duplicate work exactly when aloha is
    // slow, and spend their transport retries. Instead the connection takes no new calls; the
    // calls already on it complete as their answers arrive (this one's is read and dropped)
    // or at their own deadlines, and it closes once no call on it is waited for.
    PConn* c = pt->second.conn;
    for (auto& p : c->q)
      if (p.id == id) {
        p.abandoned = true;
        p.cb = nullptr;
      }
    pactive_.erase(pt);
    c->draining = true;
    if (std::all_of(c->q.begin(), c->q.end(), [](const PConn::Pending& p) { return p.abandoned; })) pdestroy(c);
    else check_head_of_line(c);
    if (!read_fifo_.q.empty()) pop_finished(read_fifo_);
    if (!connect_fifo_.q.empty()) pop_finished(connect_fifo_);
    return;
  }
  Conn* c = active(id);
  if (!c) return;
  release(id);
  destroy(c);
  if (!read_fifo_.q.empty()) pop_finished(read_fifo_);
  if (!connect_fifo_.q.empty()) pop_finished(connect_fifo_);
}

// ---------------------------------------------------------------- pipelined connections

void ClientPool::check_head_of_line(PConn* c) {
  // The wait for an abandoned call's answer is bounded: responses come back in order, so a
  // slow answer at the head would hold every call queued behind it until each hits its own
  // timeout (a Hystrix TIMEOUT that counts against the breaker). If the abandoned call is
  // still at the head after kDrainGraceMs, the calls behind it are re-sent on fresh
  // connections (a transport re-send, as when the connection fails); while an abandoned call
  // still waits further back, the check runs again.
  if (c->dead || c->drain_timer) return;
  if (std::none_of(c->q.begin(), c->q.end(), [](const PConn::Pending& p) { return p.abandoned; })) return;
  c->drain_timer = true;
  const uint64_t cid = c->cid;
  loop_.add_timer(kDrainGraceMs, [this, cid] {
    auto it = std::find_if(pconns_.begin(), pconns_.end(), [cid](const PConn* p) { return p->cid == cid; });
    if (it == pconns_.end()) return;  // closed meanwhile
    PConn* pc = *it;
    pc->drain_timer = false;
    if (pc->dead || pc->q.empty()) return;
    if (!pc->q.front().abandoned) {
      check_head_of_line(pc);
      return;
    }
    const double behind = double(std::count_if(pc->q.begin(), pc->q.end(), [](const PConn::Pending& p) {
      return !p.abandoned && p.cb;
    }));
    if (behind > hol_budget_) {  // over the re-send budget: keep waiting on this connection
      check_head_of_line(pc);
      return;
    }
    hol_budget_ -= behind;
    pfail(pc, "NoHttpResponseException: the answer ahead on a pipelined connection did not come");
  });
}


ClientPool::PConn* ClientPool::open_pconn() {
  sockaddr_storage ss{};
  socklen_t len = 0;
  if (!addr_ || !addr_->get(&ss, &len, nullptr)) return nullptr;  // the plain path reports it
  bool inprog = false;
  const int fd = connect_nonblocking(ss, len, &inprog);
  if (fd < 0) return nullptr;
  auto* c = new PConn();
  c->pool = this;
  c->cid = next_cid_++;
  c->fd = fd;
  c->connecting = inprog;
  c->interest = inprog ? uint32_t(EPOLLOUT) : uint32_t(EPOLLIN | EPOLLRDHUP);
  loop_.add(fd, c->interest, c);
  pconns_.push_back(c);
  ++opened_;
  return c;
}

bool ClientPool::get_pipelined(uint64_t id, std::string& req, Callback& cb) {
  // Fill the connection this batch already writes to, then any other with room, then a new
  // one: requests of one batch share a send() and a TCP segment.
  const size_t depth = size_t(pipeline_);
  PConn* c = nullptr;
  for (PConn* p : dirty_)
    if (!p->dead && !p->draining && p->q.size() < depth) {
      c = p;
      break;
    }
  if (!c)
    for (PConn* p : pconns_)
      if (!p->dead && !p->draining && p->q.size() < depth) {
        c = p;
        break;
      }
  if (!c && !(c = open_pconn())) return false;
  const uint64_t serial = next_serial_++;
  hol_budget_ = std::min(kHolResendBurst, hol_budget_ + kHolResendPerCall);
  c->out += req;
  c->q.push_back({id, serial, std::move(req), std::move(cb)});
  pactive_[id] = {c, serial};
  if (!c->connecting) arm_read_deadline(id, serial);
  if (c->connecting && connect_timeout_ms_ > 0) push_deadline(connect_fifo_, connect_timeout_ms_, id, serial);
  if (!c->dirty) {
    c->dirty = true;
    dirty_.push_back(c);
  }
  if (!flush_scheduled_) {
    flush_scheduled_ = true;
    loop_.defer([this] { flush_dirty(); });
  }
  return true;
}

void ClientPool::flush_dirty() {
  flush_scheduled_ = false;
  std::vector<PConn*> batch;
  batch.swap(dirty_);
  for (PConn* c : batch) {
    c->dirty = false;
    if (!c->dead && !c->connecting) c->do_write();
  }
}

void ClientPool::PConn::on_event(uint32_t ev) {
  if (dead) return;
  if (connecting) {
    int soerr = 0;
    socklen_t sl = sizeof soerr;
    getsockopt(fd, SOL_SOCKET, SO_ERROR, &soerr, &sl);
    if (soerr != 0 || (ev & (EPOLLERR | EPOLLHUP))) {
      // Nothing was sent: every call fails with the connect error, as each would on its own
      // connection (HttpHostConnectException: no transport retry; Feign may retry it).
      pool->pfail(this, pool->connect_error(soerr ? soerr : ECONNREFUSED), 0, true, false);
      return;
    }
    connecting = false;
    for (const Pending& p : q) pool->arm_read_deadline(p.id, p.serial);
    set_interest(EPOLLIN | EPOLLRDHUP);
    do_write();
    return;
  }
  if (ev & EPOLLOUT) {
    do_write();
    if (dead) return;
  }
  if (ev & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) do_read();
}

void ClientPool::PConn::do_write() {
  while (off < out.size()) {
    ssize_t w = ::send(fd, out.data() + off, out.size() - off, MSG_NOSIGNAL);
    if (w < 0) {
      if (errno == EINTR) continue;
      if (errno == EAGAIN) {
        set_interest(EPOLLIN | EPOLLRDHUP | EPOLLOUT);
        return;
      }
      pool->pfail(this, std::string("SocketException: ") + strerror(errno));
      return;
    }
    off += size_t(w);
  }
  out.clear();
  off = 0;
  set_interest(EPOLLIN | EPOLLRDHUP);
}

void ClientPool::PConn::do_read() {
  char buf[16384];
  for (;;) {
    ssize_t n = ::recv(fd, buf, sizeof buf, 0);
    bool eof = false;
    if (n > 0) {
      in.append(buf, size_t(n));
    } else if (n == 0) {
      eof = true;
    } else {
      if (errno == EINTR) continue;
      if (errno == EAGAIN) return;
      pool->pfail(this, std::string("SocketException: ") + strerror(errno));
      return;
    }
    // Responses arrive in request order: each completes the oldest request.
    size_t used = 0;
    bool front_head = false;  // the oldest request's response head has arrived (body pending)
    while (!q.empty()) {
      ClientResult r;
      bool close = false, head_ok = false;
      size_t consumed = 0;
      const int rc = parse_response(std::string_view(in).substr(used), eof, &r, &close, &consumed, &head_ok);
      if (rc < 0) {
        // The oldest call got a bad answer: it fails alone, as on the plain path (a protocol
        // error is never re-sent; Feign may retry it only if no valid head arrived). The calls
        // behind it got no answer at all, so they are re-sent.
        pool->pfail(this, "ClientProtocolException: malformed response", q.front().id, !head_ok);
        return;
      }
      if (rc == 0) {
        front_head = head_ok;
        used += consumed;  // the front's interim responses: dropped (parse_response)
        front_interim += consumed;
        if (front_interim > kMaxInterimBytes) {
          pool->pfail(this, "ClientProtocolException: malformed response", q.front().id, !head_ok);
          return;
        }
        break;
      }
      front_interim = 0;
      used += consumed;
      Pending p = std::move(q.front());
      q.pop_front();
      pool->pactive_.erase(p.id);
      r.ok = true;
      if (!p.abandoned && p.cb) p.cb(std::move(r));
      if (dead) return;  // the callback's work ended this connection
      if (close) {
        in.clear();
        pool->pfail(this, "NoHttpResponseException: connection closed");
        return;
      }
    }
    if (used) {
      in.erase(0, used);
      // answered requests leave the deadline FIFOs (as ClientPool::finish does for plain ones)
      if (!pool->read_fifo_.q.empty()) pool->pop_finished(pool->read_fifo_);
      if (!pool->connect_fifo_.q.empty()) pool->pop_finished(pool->connect_fifo_);
    }
    if (eof || (q.empty() && !in.empty())) {
      // The peer closed, or sent bytes nobody asked for: the connection is done. A call whose
      // response head had arrived fails for good (HttpClient re-sends only before a response);
      // the calls with nothing received yet are re-sent.
      if (eof && front_head && !q.empty()) {
        pool->pfail(this, "TruncatedChunkException: premature EOF", q.front().id, false);
        return;
      }
      pool->pfail(this, in.empty() || q.empty() ? "NoHttpResponseException: connection closed"
                                                : "TruncatedChunkException: premature EOF");
      return;
    }
    if (draining && std::all_of(q.begin(), q.end(), [](const Pending& p) { return p.abandoned; })) {
      pool->pdestroy(this);  // nothing on it is waited for any more
      return;
    }
    if (size_t(n) < sizeof buf) return;
  }
}

void ClientPool::pdestroy(PConn* c) {
  if (c->dead) return;
  c->dead = true;
  loop_.del(c->fd);
  ::close(c->fd);
  c->fd = -1;
  pconns_.erase(std::remove(pconns_.begin(), pconns_.end(), c), pconns_.end());
  dirty_.erase(std::remove(dirty_.begin(), dirty_.end(), c), dirty_.end());
  loop_.retire(c);
}

void ClientPool::pfail(PConn* c, const std::string& why, uint64_t failed, bool failed_retryable, bool resend_others) {
  std::deque<PConn::Pending> q;
  q.swap(c->q);
  pdestroy(c);
  for (auto& p : q) {
    pactive_.erase(p.id);
    if (p.abandoned || !p.cb) continue;
    if (p.id == failed || !resend_others) {
      ClientResult r;
      r.error = why;
      // retryable = an IOException before a response head (Feign's RetryableException)
      r.retryable = p.id == failed ? failed_retryable : true;
      p.cb(std::move(r));
    } else {
      resubmit(p.id, std::move(p.req), std::move(p.cb), p.tries + 1, why);
    }
  }
  if (!read_fifo_.q.empty()) pop_finished(read_fifo_);
  if (!connect_fifo_.q.empty()) pop_finished(connect_fifo_);
}

void ClientPool::resubmit(uint64_t id, std::string req, Callback cb, int tries, const std::string& why) {
  if (tries > kTransportRetries) {
    ClientResult r;
    r.error = why;
    r.retryable = true;
    cb(std::move(r));
    return;
  }
  if (transport_retries_) transport_retries_->fetch_add(1, std::memory_order_relaxed);
  // DefaultHttpRequestRetryHandler: the idempotent GET goes out again on a fresh connection
  auto* fresh = new Conn();
  fresh->pool = this;
  fresh->tries = tries;
  start_on(fresh, id, &req, std::move(cb), false);
}

}  // namespace hola::client
