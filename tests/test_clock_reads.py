"""Clock reads per chained request: hola A's request path for GET
/api/hola-chaining reads no clock of its own. Millisecond bookkeeping (the Hystrix windows
and the execution timeout's deadline) and the /metrics latency histogram use the time the
event loop read when the pass found its events (src/core/clock.h loop_now_ms/ns). Wall-clock
span timestamps are read only when a collector records them.

The `clockcount` build counts every clock read (hola_clock_reads_total). A is run with
busy-polling off and driven one request at a time. Each pass of its loop then reads the clock
exactly twice: before the blocking wait and after it. So everything above 2 x passes is the
request path's own."""
from __future__ import annotations

import json
import socket

import pytest

from hola_amd import native
from hola_amd.server import HolaProcess


def _metrics(s) -> dict:
    _, _, body = s.get("/metrics")
    out = {}
    for ln in body.decode().splitlines():
        if ln.startswith("hola_clock_reads_total{"):
            out["clock_" + ln.split('"')[1]] = float(ln.rsplit(" ", 1)[1])
        elif ln.startswith(("hola_loop_passes_total ", "hola_http_requests_total ")):
            k, v = ln.split()
            out[k] = float(v)
    return out


def _get(sock, path: str) -> bytes:
    sock.sendall(f"GET {path} HTTP/1.1\r\nHost: a\r\n\r\n".encode())
    buf = b""
    while b"\r\n\r\n" not in buf:
        buf += sock.recv(65536)
    head, _, body = buf.partition(b"\r\n\r\n")
    n = int([ln.split(b":")[1] for ln in head.split(b"\r\n") if ln.lower().startswith(b"content-length")][0])
    while len(body) < n:
        body += sock.recv(65536)
    return body


@pytest.mark.parametrize("collector", [False, True])
def test_chained_request_path_reads_no_clock(collector, tmp_path):
    exe = native.build("clockcount") / "hola"
    with HolaProcess(args=["--aloha-url", "http://127.0.0.1:1/", "--no-tracing", "--feign-log", "none",
                           "--feign-retry", "off", "--log-level", "warn"], env={"HOSTNAME": "B"}, threads=1) as b:
        args = ["--aloha-url", f"http://127.0.0.1:{b.port}/", "--aloha-path", "api/hola-chaining",
                "--feign-log", "none", "--busy-poll-us", "0", "--log-level", "warn"]
        if collector:  # spans recorded: their timestamps are wall-clock reads (2 per span)
            args += ["--zipkin-url", "http://127.0.0.1:1/"]
        with HolaProcess(args=args, env={"HOSTNAME": "A"}, threads=1, exe=exe) as a:
            with socket.create_connection(("127.0.0.1", a.port), timeout=10) as sk:
                assert json.loads(_get(sk, "/api/hola-chaining")) == ["Hola de A", "Hola de B",
                                                                       "Aloha response (fallback)"]
                m0 = _metrics(a)
                n = 300
                for _ in range(n):
                    _get(sk, "/api/hola-chaining")
                m1 = _metrics(a)
    reads = m1["clock_precise"] - m0["clock_precise"]
    passes = m1["hola_loop_passes_total"] - m0["hola_loop_passes_total"]
    # the /metrics scrape between the two snapshots is one request (and pass) of its own
    own = (reads - 2 * passes) / n
    if collector:
        # server span start/end and client span start/end: four wall-clock reads per request
        assert 3.9 <= own <= 4.1, (reads, passes)
    else:
        # the timeout timer re-arms once per expiry (two reads per 600 ms): nothing per request
        assert own <= 0.05, (reads, passes, own)
    print(f"\nclock reads per chained request: {reads / n:.3f} (loop {2 * passes / n:.3f}, request path {own:.3f})")
    assert passes / n <= 2.2  # a request readable, then aloha's answer readable
