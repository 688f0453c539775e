// Socket helpers shared by the server, the outbound client, the load generator and the
// round-robin proxy.
#pragma once
#include <netinet/in.h>
#include <sys/socket.h>

#include <cstdint>
#include <string>
#include <vector>

namespace hola {

struct ListenOptions {
  std::string host = "0.0.0.0";
  int port = 8080;
  int backlog = 4096;
  bool reuseport = false;
  // SO_INCOMING_CPU on the listener (-1 = unset): in an SO_REUSEPORT group, Linux 6.1+ hands
  // a new connection to the listener whose incoming CPU is the CPU its SYN was processed on
  // (the client's CPU for loopback clients), and hashes only when none matches.
  int incoming_cpu = -1;
};

// Creates a non-blocking listening TCP socket; returns fd or -1 (errno set, message in *err).
int listen_tcp(const ListenOptions& o, std::string* err);
// Port actually bound (useful with port 0).
int bound_port(int fd);

// Parses "host:port" / "[v6]:port"; resolves with getaddrinfo (blocking).
bool resolve_host(const std::string& host, int port, sockaddr_storage* out, socklen_t* len,
                  std::string* err);

// Non-blocking connect; returns fd (connect may be in progress) or -1.
int connect_nonblocking(const sockaddr_storage& addr, socklen_t len, bool* in_progress);
// Blocking connect with a timeout in ms; returns fd or -1.
int connect_blocking(const sockaddr_storage& addr, socklen_t len, int timeout_ms);

// A connect/socket errno caused by this host running out of something (fds, memory,
// ephemeral ports), not by the peer: it must never mark a backend DOWN.
bool is_local_resource_error(int err);

void set_nodelay(int fd);
void set_nonblocking(int fd, bool on = true);

// Writes all bytes (blocking fd); false on error.
bool write_all(int fd, const char* p, size_t n);

std::string sockaddr_to_string(const sockaddr_storage& a);
// First non-loopback IPv4 address of this host in network order (0 when none): used as the
// Zipkin endpoint ipv4 (Brave reports the local address of the servlet container).
uint32_t local_ipv4();

}  // namespace hola
