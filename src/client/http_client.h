// Non-blocking, per-worker, keep-alive HTTP/1.1 client pool (SURVEY.md T7/T8 role).
//
// The reference builds a *new* Apache HttpClient (and leaks it) for every chaining request
// (HolaResource.java:98-102). Here every worker owns one pool of kept-alive connections to
// aloha, driven by the worker's own event loop — no extra threads, no per-request client.
#pragma once
#include <netinet/in.h>

#include <atomic>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
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
  void start();
  void stop();
  // false when the host has not (yet) resolved.
  bool get(sockaddr_storage* out, socklen_t* len, std::string* err) const;
  void resolve_now();  // synchronous (tests / startup)

 private:
  std::string host_;
  int port_;
  int refresh_ms_;
  mutable std::mutex mu_;
  bool ok_ = false;
  sockaddr_storage addr_{};
  socklen_t len_ = 0;
  std::string err_ = "not resolved yet";
  std::thread th_;
  std::atomic<bool> stop_{false};
};

struct ClientResult {
  bool ok = false;      // a complete HTTP response was received
  int status = 0;
  std::string body;
  std::string error;    // network error description when !ok
};

class ClientPool {
 public:
  using Callback = std::function<void(ClientResult&&)>;
  ClientPool(EventLoop& loop, Url target, AddressCache* addr, size_t max_idle = 64);
  ~ClientPool();
  // Starts GET <path>; `cb` runs exactly once on the loop thread unless cancel() is called
  // first. Returns a request id.
  uint64_t get(const std::string& path, const std::string& extra_headers, Callback cb);
  // Abandons a request (e.g. on timeout): its connection is closed, its callback dropped.
  void cancel(uint64_t id);
  size_t idle_connections() const { return idle_.size(); }
  uint64_t connections_opened() const { return opened_; }

 private:
  struct Conn;
  friend struct Conn;
  void start_on(Conn* c, uint64_t id, std::string req, Callback cb, bool reused);
  void finish(Conn* c, ClientResult&& r, bool reusable);
  void destroy(Conn* c);
  std::string build_request(const std::string& path, const std::string& extra) const;

  EventLoop& loop_;
  Url target_;
  AddressCache* addr_;
  size_t max_idle_;
  std::vector<Conn*> idle_;
  std::unordered_map<uint64_t, Conn*> active_;
  uint64_t next_id_ = 1;
  uint64_t opened_ = 0;
  std::string host_header_;
};

}  // namespace hola::client
