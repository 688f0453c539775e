"""Small networking helpers for tests and harnesses (stdlib only)."""
from __future__ import annotations

import http.client
import socket
import time


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def http_get(host: str, port: int, path: str, headers: dict | None = None, method: str = "GET",
             timeout: float = 5.0, body: bytes | None = None):
    """Returns (status, headers_dict_lowercase, body_bytes) over a fresh connection."""
    conn = http.client.HTTPConnection(host, port, timeout=timeout)
    try:
        conn.request(method, path, body=body, headers=headers or {})
        r = conn.getresponse()
        data = r.read()
        return r.status, {k.lower(): v for k, v in r.getheaders()}, data
    finally:
        conn.close()


def wait_http(host: str, port: int, path: str = "/api/health", timeout: float = 20.0) -> bool:
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        try:
            st, _, _ = http_get(host, port, path, timeout=1.0)
            if st == 200:
                return True
        except OSError:
            pass
        time.sleep(0.02)
    return False
