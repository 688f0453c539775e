"""In-process fake downstream services for integration tests.

* :class:`FakeAloha`  — the `aloha` service hola chains to (AlohaService.java:25). Its mode can
  be switched at runtime: ``ok`` / ``slow`` / ``error`` (HTTP 500) / ``garbage`` (invalid
  JSON) / ``chunked`` / ``chunked_lf`` (chunk lines ended by a bare LF) / ``close`` (drop the
  connection) / ``unavailable`` (HTTP 503 with ``Retry-After: <retry_after>``) / ``empty``
  (200, empty body) / ``json_null`` (200, ``null``) / ``no_content`` (204) /
  ``close_delimited`` (no Content-Length, body ends at EOF) / ``drop_idle`` (keep-alive
  response, then the socket closes while idle) / ``bad_status`` (an invalid HTTP status line:
  no valid response head) / ``bad_chunk`` (a valid 200 head, then a malformed chunk size).
  Records every request's headers so tests can check B3 propagation.
* :class:`FakeZipkin` — a span collector recording POST /api/v1/spans and /api/v2/spans.
"""
from __future__ import annotations

import json
import socket
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer


class _Server(ThreadingHTTPServer):
    daemon_threads = True
    allow_reuse_address = True

    def handle_error(self, request, client_address):
        # Clients (hola) legitimately abandon slow calls at their timeout: a broken pipe here
        # is expected, not a test failure worth a traceback on stderr.
        pass


class _Base:
    def __init__(self, handler_cls):
        self.server = _Server(("127.0.0.1", 0), handler_cls)
        self.server.owner = self  # type: ignore[attr-defined]
        self.port = self.server.server_address[1]
        self.thread = threading.Thread(target=self.server.serve_forever, daemon=True)

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self.port}/"

    def start(self):
        self.thread.start()
        return self

    def stop(self):
        self.server.shutdown()
        self.server.server_close()

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()


class _AlohaHandler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"

    def log_message(self, *a):  # silence
        pass

    def do_GET(self):
        owner: FakeAloha = self.server.owner  # type: ignore[attr-defined]
        with owner.lock:
            owner.requests.append({"path": self.path, "headers": {k.lower(): v for k, v in self.headers.items()},
                                   "peer_port": self.client_address[1]})
            mode, delay, payload = owner.mode, owner.delay_s, owner.payload
            if mode == "slow_once":  # this request is slow, the ones after it are not
                owner.mode = "ok"
        if mode in ("slow", "slow_once"):
            time.sleep(delay)
        if mode == "close":
            self.close_connection = True
            self.connection.shutdown(socket.SHUT_RDWR)
            return
        if mode == "bad_status":  # HTTP-level fault: no parseable status line
            self.wfile.write(b"HTTP/1.1 2x0 Broken\r\nContent-Length: 2\r\n\r\n[]")
            self.wfile.flush()
            return
        if mode == "bad_chunk":  # a valid head, then framing no HTTP/1.1 parser accepts
            self.wfile.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\n"
                             b"Transfer-Encoding: chunked\r\n\r\nzz\r\n[]\r\n0\r\n\r\n")
            self.wfile.flush()
            return
        if mode == "cr_in_name":  # a CR inside a header name: not Transfer-Encoding, must not chunk
            body = json.dumps(payload).encode()
            self.wfile.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nTransfer\rEncoding: chunked\r\n"
                             b"Content-Length: %d\r\n\r\n%s" % (len(body), body))
            self.wfile.flush()
            return
        if mode == "cl_unparseable":  # HttpClient's lax strategy: the last parseable Content-Length wins
            body = json.dumps(payload).encode()
            self.wfile.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nContent-Length: %d\r\n"
                             b"Content-Length: 12abc\r\n\r\n%s" % (len(body), body))
            self.wfile.flush()
            return
        if mode == "te_not_chunked":  # a transfer coding other than chunked: the body runs to the close
            body = json.dumps(payload).encode()
            self.close_connection = True
            self.wfile.write(b"HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nTransfer-Encoding: identity\r\n"
                             b"Content-Length: 2\r\n\r\n%s" % body)
            self.wfile.flush()
            self.connection.shutdown(socket.SHUT_WR)
            return
        if mode == "interim_close_once":  # a 100 Continue, then the connection closes; next ones ok
            with owner.lock:
                owner.mode = "ok"
            self.wfile.write(b"HTTP/1.1 100 Continue\r\n\r\n")
            self.wfile.flush()
            self.close_connection = True
            self.connection.shutdown(socket.SHUT_RDWR)
            return
        if mode == "interim_flood":  # 96 KiB of interim responses before the final one
            self.wfile.write(b"HTTP/1.1 100 Continue\r\n\r\n" * (96 * 1024 // 25))
        if mode == "interim":  # unasked-for 1xx responses before the final one (RFC 9110 §15.2)
            self.wfile.write(b"HTTP/1.1 100 Continue\r\n\r\n"
                             b"HTTP/1.1 103 Early Hints\r\nLink: </aloha.css>; rel=preload\r\n\r\n")
        if self.path != "/api/aloha-chaining":
            body, status = b"not found", 404
        elif mode == "error":
            body, status = b"boom", 500
        elif mode == "unavailable":  # 503 + Retry-After: Feign's ErrorDecoder makes it retryable
            body, status = b"busy", 503
        elif mode == "empty":
            body, status = b"", 200
        elif mode == "json_null":
            body, status = b"null", 200
        elif mode == "no_content":
            body, status = b"", 204
        elif mode == "garbage":
            body, status = b"{not json", 200
        elif mode == "compact" or owner.compact:  # as Jackson writes a List<String>: no whitespace
            body, status = json.dumps(payload, separators=(",", ":"), ensure_ascii=False).encode(), 200
        else:
            body, status = json.dumps(payload).encode(), 200
        self.send_response(status)
        self.send_header("Content-Type", "application/json")
        if mode == "unavailable":
            self.send_header("Retry-After", owner.retry_after)
        if mode == "close_delimited":  # no Content-Length: the body ends with the connection
            self.close_connection = True
            self.end_headers()
            self.wfile.write(body)
            self.wfile.flush()
            self.connection.shutdown(socket.SHUT_WR)
            return
        if mode in ("chunked", "chunked_lf"):
            eol = b"\r\n" if mode == "chunked" else b"\n"  # bare LF: tolerated framing (RFC 9112 §2.2)
            self.send_header("Transfer-Encoding", "chunked")
            self.end_headers()
            half = len(body) // 2
            for part in (body[:half], body[half:]):
                self.wfile.write(b"%x%s%s%s" % (len(part), eol, part, eol))
            self.wfile.write(b"0" + eol + eol)
        else:
            if status != 204:
                self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)
            if mode == "drop_idle":  # a kept-alive response, then the socket closes while idle
                self.wfile.flush()
                self.close_connection = True


class FakeAloha(_Base):
    def __init__(self, payload=None, mode: str = "ok", delay_s: float = 1.0):
        self.lock = threading.Lock()
        self.requests: list[dict] = []
        self.mode = mode
        self.delay_s = delay_s
        self.retry_after = "0"  # Retry-After value sent in mode "unavailable"
        self.payload = payload if payload is not None else ["Aloha mai aloha-1", "Bonjour de bonjour-1"]
        self.compact = False  # every list written without whitespace (modes that write a list)
        super().__init__(_AlohaHandler)

    def set_mode(self, mode: str, delay_s: float | None = None):
        with self.lock:
            self.mode = mode
            if delay_s is not None:
                self.delay_s = delay_s


class _ZipkinHandler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"

    def log_message(self, *a):
        pass

    def do_POST(self):
        owner: FakeZipkin = self.server.owner  # type: ignore[attr-defined]
        n = int(self.headers.get("Content-Length", "0"))
        body = self.rfile.read(n)
        with owner.lock:
            owner.posts.append({"path": self.path, "content_type": self.headers.get("Content-Type"),
                                "spans": json.loads(body), "peer_port": self.client_address[1]})
            status, interim = owner.status, owner.interim
        if interim:  # a 100 Continue nobody asked for, as some fronts send (RFC 9110 §15.2)
            self.wfile.write(b"HTTP/1.1 100 Continue\r\n\r\n")
        self.send_response(status)
        if status != 204:  # a 204 carries no Content-Length (RFC 9110 §8.6)
            self.send_header("Content-Length", "0")
        self.end_headers()


class FakeZipkin(_Base):
    """Zipkin collector stand-in. With ``tls=(certfile, keyfile)`` it serves HTTPS (the URL
    becomes https://127.0.0.1:PORT/)."""

    def __init__(self, status: int = 202, tls: tuple[str, str] | None = None, interim: bool = False):
        self.lock = threading.Lock()
        self.posts: list[dict] = []
        self.status = status
        self.interim = interim
        super().__init__(_ZipkinHandler)
        self.tls = tls
        if tls:
            import ssl

            ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
            ctx.load_cert_chain(*tls)
            self.server.socket = ctx.wrap_socket(self.server.socket, server_side=True)

    @property
    def url(self) -> str:
        return f"{'https' if self.tls else 'http'}://127.0.0.1:{self.port}/"

    def spans(self) -> list[dict]:
        with self.lock:
            return [s for p in self.posts for s in p["spans"]]

    def wait_for(self, pred, timeout: float = 10.0) -> list[dict]:
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            sp = self.spans()
            if pred(sp):
                return sp
            time.sleep(0.05)
        return self.spans()


def closed_port() -> int:
    """A localhost port with nothing listening (connection refused)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port
