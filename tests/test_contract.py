"""The behavioural contract of the reference service, end to end against the
native server binary."""
import json
import re
import os
import shutil
import socket
import time
from pathlib import Path

import pytest


def test_hola_default_greeting(hola):
    s = hola(env={"HOSTNAME": "h"})
    st, h, body = s.get("/api/hola")
    assert st == 200
    assert body == b"Hola de h"
    assert h["content-type"].split(";")[0] == "text/plain"
    assert h["access-control-allow-origin"] == "*"  # CorsFilter.java:31


def test_hola_hostname_unset(hola_bin):
    from hola_amd.server import HolaProcess

    with HolaProcess(env={}) as s:  # HOSTNAME absent -> "unknown" (HolaResource.java:57)
        st, _, body = s.get("/api/hola")
    assert (st, body) == (200, b"Hola de unknown")


def test_hola_with_translation_file(hola):
    from pathlib import Path

    conf = Path(__file__).resolve().parent.parent / "translation.properties"
    s = hola(args=[f"-Dconf={conf}"], env={"HOSTNAME": "h"})
    st, _, body = s.get("/api/hola")
    # translation.properties ends in a literal backslash-n escape -> a real newline
    assert (st, body) == (200, b"Hola de h mediante el archivo de configuraciones\n")


def test_chaining_fallback_when_aloha_down(hola):
    s = hola(args=["--aloha-url", "http://127.0.0.1:1/", "--feign-log", "none"], env={"HOSTNAME": "h"})
    st, h, body = s.get("/api/hola-chaining")
    assert st == 200
    assert h["content-type"].split(";")[0] == "application/json"
    assert h["access-control-allow-origin"] == "*"
    assert json.loads(body) == ["Hola de h", "Aloha response (fallback)"]


def test_health(hola):
    s = hola()
    st, h, body = s.get("/api/health")
    assert (st, body) == (200, b"I'm ok")
    assert h["content-type"].split(";")[0] == "text/plain"
    assert h["access-control-allow-origin"] == "*"


def test_head(hola):
    s = hola(env={"HOSTNAME": "h"})
    st, h, body = s.get("/api/hola", method="HEAD")
    assert st == 200 and body == b""
    assert h["content-length"] == str(len("Hola de h"))
    assert h["access-control-allow-origin"] == "*"


def test_options(hola):
    s = hola()
    st, h, body = s.get("/api/hola", method="OPTIONS")
    assert st == 200
    assert set(x.strip() for x in h["allow"].split(",")) == {"GET", "HEAD", "OPTIONS"}


@pytest.mark.parametrize("method", ["POST", "PUT", "DELETE", "PATCH"])
def test_method_not_allowed(hola, method):
    s = hola()
    st, h, _ = s.get("/api/hola", method=method, body=b"x" if method != "DELETE" else None)
    assert st == 405
    assert "GET" in h["allow"]


@pytest.mark.parametrize("accept,status", [
    ("application/json", 406),
    ("text/plain", 200),
    ("text/*", 200),
    ("*/*", 200),
    ("text/html, */*;q=0.1", 200),
    ("*/*, text/plain;q=0", 406),
    ("text/html, image/gif, image/jpeg, *; q=.2, */*; q=.2", 200),  # Java HttpURLConnection default
])
def test_negotiation(hola, accept, status):
    s = hola()
    st, _, _ = s.get("/api/hola", headers={"Accept": accept})
    assert st == status


def test_chaining_negotiation(hola):
    s = hola(args=["--aloha-url", "http://127.0.0.1:1/", "--feign-log", "none"])
    assert s.get("/api/hola-chaining", headers={"Accept": "text/plain"})[0] == 406
    assert s.get("/api/hola-chaining", headers={"Accept": "application/json"})[0] == 200


def test_not_found(hola):
    s = hola()
    assert s.get("/api/nope")[0] == 404
    assert s.get("/api")[0] == 404
    st, h, body = s.get("/nope")
    assert st == 404 and b"Not Found" in body


def test_index_and_swagger(hola):
    s = hola()
    st, h, body = s.get("/")
    assert st == 200 and h["content-type"].startswith("text/html")
    assert b"webjars/swagger-ui/2.1.4/?url=" in body and b"api/swagger.json" in body
    st, h, body = s.get("/api/swagger.json")
    assert st == 200 and h["content-type"].split(";")[0] == "application/json"
    doc = json.loads(body)
    assert doc["swagger"] == "2.0"
    info = doc["info"]  # SwaggerListener.java:31-40
    assert info["title"] == "Hola microservices REST API"
    assert info["version"] == "1.0.0"
    assert info["description"] == "Operations that can be invoked in the hola microservices"
    assert info["license"] == {"name": "Apache 2.0", "url": "http://www.apache.org/licenses/LICENSE-2.0.html"}
    assert info["contact"]["name"] == "developer@redhat.com"
    assert doc["basePath"] == "/api" and doc["schemes"] == ["http"]
    assert set(doc["paths"]) == {"/hola", "/hola-chaining", "/health"}
    st, h, body = s.get("/webjars/swagger-ui/2.1.4/?url=http://x/api/swagger.json")
    assert st == 200 and b"swagger" in body.lower()


def test_trailing_slash_and_percent_encoding(hola):
    s = hola(env={"HOSTNAME": "h"})
    assert s.get("/api/hola/")[2] == b"Hola de h"
    assert s.get("/api/hol%61")[2] == b"Hola de h"
    assert s.get("/api/hola?x=1&y=2")[2] == b"Hola de h"


def test_dot_segments_are_removed_before_matching(hola):
    """Undertow canonicalises the request path before servlet/JAX-RS matching (parity
    unpinned: no reference artefact covers it); RFC 3986 §5.2.4 gives the same result."""
    s = hola(env={"HOSTNAME": "h"})
    assert s.get("/api/../api/hola")[2] == b"Hola de h"
    assert s.get("/api/./hola")[2] == b"Hola de h"
    assert s.get("/../../api/health")[2] == b"I'm ok"
    assert s.get("/api/%2e%2e/api/hola")[2] == b"Hola de h"  # decoded first, then canonicalised
    assert s.get("/api/hola/x/..")[2] == b"Hola de h"       # -> /api/hola/ (one trailing slash)
    assert s.get("/api/hola/..")[0] == 404                   # -> /api/


def test_encoded_slash_is_not_a_separator(hola):
    """Undertow's default allow-encoded-slash=false leaves %2F encoded, so it never splits a
    segment: /api%2Fhola and /api/x%2F..%2Fhola are 404 (parity unpinned: no reference
    artefact covers it)."""
    s = hola(env={"HOSTNAME": "h"})
    assert s.get("/api%2Fhola")[0] == 404
    assert s.get("/api%2fhola")[0] == 404
    assert s.get("/api/x%2F..%2Fhola")[0] == 404
    assert s.get("/api/hol%61")[2] == b"Hola de h"  # other escapes still decode


def _raw(port, data: bytes, timeout=3.0) -> bytes:
    with socket.create_connection(("127.0.0.1", port), timeout=timeout) as c:
        c.sendall(data)
        c.shutdown(socket.SHUT_WR)
        out = b""
        while True:
            b = c.recv(65536)
            if not b:
                break
            out += b
    return out


def test_pipelining_keeps_order(hola):
    s = hola(env={"HOSTNAME": "h"})
    req = b"GET /api/hola HTTP/1.1\r\nHost: x\r\n\r\nGET /api/health HTTP/1.1\r\nHost: x\r\n\r\n" \
          b"GET /api/hola HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n"
    out = _raw(s.port, req)
    assert out.count(b"HTTP/1.1 200 OK") == 3
    i1, i2, i3 = out.find(b"Hola de h"), out.find(b"I'm ok"), out.rfind(b"Hola de h")
    assert 0 < i1 < i2 < i3
    assert b"Connection: close" in out


def test_http10_closes(hola):
    s = hola(env={"HOSTNAME": "h"})
    out = _raw(s.port, b"GET /api/hola HTTP/1.0\r\n\r\n")
    assert out.startswith(b"HTTP/1.1 200 OK") and b"Connection: close" in out and out.endswith(b"Hola de h")


@pytest.mark.parametrize("raw,status", [
    (b"GARBAGE\r\n\r\n", b"400"),
    (b"GET /api/hola HTTP/2.0\r\n\r\n", b"505"),
    (b"GET /api/hola HTTP/1.1\r\nBad Header\r\n\r\n", b"400"),
    (b"GET /api/hola HTTP/1.1\r\nContent-Length: 5\r\nTransfer-Encoding: chunked\r\n\r\n", b"400"),
])
def test_malformed_requests(hola, raw, status):
    s = hola()
    out = _raw(s.port, raw)
    assert out.split(b" ")[1] == status
    # the server survives
    assert s.get("/api/health")[0] == 200


def test_request_bodies_are_skipped(hola):
    s = hola(env={"HOSTNAME": "h"})
    req = (b"GET /api/hola HTTP/1.1\r\nContent-Length: 4\r\n\r\nabcd"
           b"GET /api/hola HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n3\r\nabc\r\n0\r\n\r\n"
           b"GET /api/health HTTP/1.1\r\nConnection: close\r\n\r\n")
    out = _raw(s.port, req)
    assert out.count(b"200 OK") == 3 and out.endswith(b"I'm ok")


def test_date_header(hola):
    s = hola()
    _, h, _ = s.get("/api/hola")
    assert h["date"].endswith("GMT") and len(h["date"]) == 29


def test_idle_keepalive_connections_are_closed(hola):
    s = hola(args=["--idle-timeout-ms", "200"])
    with socket.create_connection(("127.0.0.1", s.port), timeout=3) as c:
        c.sendall(b"GET /api/health HTTP/1.1\r\nHost: x\r\n\r\n")
        assert b"I'm ok" in c.recv(4096)
        time.sleep(0.8)
        assert c.recv(4096) == b""  # server closed the idle connection


def test_max_connections(hola):
    s = hola(args=["--max-connections", "2"], threads=1)
    socks = [socket.create_connection(("127.0.0.1", s.port), timeout=3) for _ in range(2)]
    try:
        for c in socks:
            c.sendall(b"GET /api/health HTTP/1.1\r\nHost: x\r\n\r\n")
            assert b"I'm ok" in c.recv(4096)
        with socket.create_connection(("127.0.0.1", s.port), timeout=3) as extra:
            extra.sendall(b"GET /api/health HTTP/1.1\r\nHost: x\r\n\r\n")
            try:
                data = extra.recv(4096)
            except ConnectionResetError:
                data = b""
            assert data == b""
    finally:
        for c in socks:
            c.close()
    time.sleep(0.1)
    assert s.get("/api/health")[0] == 200  # capacity returns once connections close


def test_many_concurrent_connections(hola):
    """1000 simultaneous keep-alive connections on 2 workers, each served in turn."""
    s = hola(threads=2, env={"HOSTNAME": "h"})
    socks = [socket.create_connection(("127.0.0.1", s.port), timeout=5) for _ in range(1000)]
    try:
        for c in socks:
            c.sendall(b"GET /api/hola HTTP/1.1\r\nHost: x\r\n\r\n")
        ok = 0
        for c in socks:
            data = b""
            while not data.endswith(b"Hola de h"):
                chunk = c.recv(4096)
                if not chunk:
                    break
                data += chunk
            ok += data.startswith(b"HTTP/1.1 200 OK")
        assert ok == 1000
        _, _, m = s.get("/metrics")
        assert b"hola_connections_open 10" in m  # 1000 + the metrics connection itself
    finally:
        for c in socks:
            c.close()


def test_metrics_process_collector(hola):
    """/metrics carries the standard process_* metrics of Prometheus client libraries."""
    import resource

    s = hola()
    t0 = time.time()
    m = {}
    for line in s.get("/metrics")[2].decode().splitlines():
        if line.startswith("process_"):
            k, v = line.split()
            m[k] = float(v)
    assert set(m) == {"process_cpu_seconds_total", "process_virtual_memory_bytes", "process_resident_memory_bytes",
                      "process_start_time_seconds", "process_open_fds", "process_max_fds"}
    assert 1 << 20 < m["process_resident_memory_bytes"] < 512 << 20
    assert m["process_virtual_memory_bytes"] > m["process_resident_memory_bytes"]
    assert abs(m["process_start_time_seconds"] - t0) < 120
    assert 3 <= m["process_open_fds"] < 200
    assert m["process_max_fds"] == resource.getrlimit(resource.RLIMIT_NOFILE)[0]
    assert m["process_cpu_seconds_total"] >= 0


def test_version_and_build_info(hola, hola_bin):
    """`hola --version` and /metrics' hola_build_info name the release (the reference's Maven
    version, pom.xml:24, which the image is tagged with), the source revision, the x86-64 level
    and the compiler; all three views agree."""
    import re
    import subprocess

    from hola_amd import native

    out = subprocess.run([str(hola_bin), "--version"], capture_output=True, text=True, timeout=10)
    assert out.returncode == 0, out.stderr
    info = native.load_native().build_info()
    m = re.fullmatch(r"hola (\S+) \(revision (\S+), (x86-64(?:-v\d)?), (.+), (\S+)\)\n", out.stdout)
    assert m, out.stdout
    assert m.group(1) == info["version"] == "0.0.1-SNAPSHOT"
    assert re.fullmatch(r"[0-9a-f]{7,40}(-dirty)?|unknown", m.group(2))
    assert m.group(3) == info["isa"]
    for tool in ("hola_rrproxy", "hola_loadgen"):  # built from the same tree: the same revision
        v = subprocess.run([str(hola_bin.parent / tool), "--version"], capture_output=True, text=True, timeout=10)
        assert v.stdout == f"{tool} {m.group(1)} (revision {m.group(2)}, {m.group(3)})\n", v.stdout
    line = next(ln for ln in hola().get("/metrics")[2].decode().splitlines() if ln.startswith("hola_build_info{"))
    assert line == (f'hola_build_info{{version="{m.group(1)}",revision="{m.group(2)}",isa="{m.group(3)}",'
                    f'compiler="{m.group(4)}"}} 1')


def test_expect_100_continue(hola):
    s = hola()
    with socket.create_connection(("127.0.0.1", s.port), timeout=3) as c:
        c.sendall(b"POST /api/hola HTTP/1.1\r\nHost: x\r\nContent-Length: 4\r\nExpect: 100-continue\r\n\r\n")
        assert c.recv(4096).startswith(b"HTTP/1.1 100 Continue\r\n\r\n")
        c.sendall(b"abcd")
        data = c.recv(4096)
        assert data.startswith(b"HTTP/1.1 405")


def test_swagger_yaml_matches_json(hola):
    import yaml

    s = hola()
    st, h, body = s.get("/api/swagger.yaml")
    assert st == 200 and h["content-type"] == "application/yaml"
    assert h["access-control-allow-origin"] == "*"
    assert yaml.safe_load(body) == json.loads(s.get("/api/swagger.json")[2])


def test_slowloris_partial_request_times_out(hola):
    s = hola(args=["--idle-timeout-ms", "200"])
    with socket.create_connection(("127.0.0.1", s.port), timeout=3) as c:
        c.sendall(b"GET /api/hola HTTP/1.1\r\nHost: x\r\nX-Slow: ")  # never finished
        time.sleep(0.8)
        assert c.recv(4096) == b""


def test_peer_that_stops_reading_responses_times_out(hola):
    """A client that pipelines requests but never reads the answers fills the socket, then the
    server's bounded backlog (reading stops at 1 MiB unsent); with nothing read or written for
    --idle-timeout-ms the connection is closed, freeing its buffers, while a slow reader that
    makes progress is kept."""
    s = hola(args=["--idle-timeout-ms", "300"], threads=1)
    req = b"GET /api/hola HTTP/1.1\r\nHost: x\r\n\r\n"
    stalled = socket.socket()
    stalled.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)
    stalled.connect(("127.0.0.1", s.port))
    stalled.setblocking(False)
    sent = 0
    t0 = time.monotonic()
    while time.monotonic() - t0 < 3:  # until the server stops reading (our sends block)
        try:
            sent += stalled.send(req * 256)
        except BlockingIOError:
            time.sleep(0.05)
            try:
                sent += stalled.send(req * 256)
            except BlockingIOError:
                break
    assert sent > len(req) * 10000
    # a slow reader: one small read every 100 ms keeps its connection alive past the timeout
    slow = socket.create_connection(("127.0.0.1", s.port), timeout=3)
    slow.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)
    slow.sendall(req * 20000)
    got = 0
    for _ in range(10):
        time.sleep(0.1)
        got += len(slow.recv(65536))
    assert got > 0
    # the stalled connection is gone: its unread responses end in EOF or a reset
    stalled.setblocking(True)
    stalled.settimeout(3)
    end = None
    try:
        while True:
            chunk = stalled.recv(1 << 20)
            if not chunk:
                end = "eof"
                break
    except ConnectionResetError:
        end = "reset"
    assert end in ("eof", "reset")
    slow.settimeout(0.5)
    assert slow.recv(65536)  # still served
    stalled.close()
    slow.close()


@pytest.mark.parametrize("sig", ["SIGTERM", "SIGINT", "SIGHUP"])
def test_termination_signals_drain_and_exit_zero(hola, sig):
    """The JVM runs its shutdown hooks on SIGTERM, SIGINT and SIGHUP alike: each one drains
    and exits 0 here."""
    import signal

    s = hola()
    assert s.get("/api/hola")[0] == 200
    assert s.stop(getattr(signal, sig), timeout=10) == 0
    assert f"received {sig}: draining" in s.log()


def test_profile_stage_histograms(hola, tmp_path):
    """`--profile`: per-stage latency histograms dumped at exit."""
    import signal

    out = tmp_path / "prof.json"
    s = hola(args=["--profile", "--profile-out", str(out)], threads=2)
    for _ in range(3):
        with socket.create_connection(("127.0.0.1", s.port), timeout=5) as c:
            c.sendall(b"GET /api/hola HTTP/1.1\r\nHost: x\r\n\r\n" * 4 + b"GET /api/health HTTP/1.1\r\nConnection: close\r\n\r\n")
            while c.recv(65536):
                pass
    assert s.stop(signal.SIGTERM, timeout=10) == 0
    prof = json.loads(out.read_text())
    for stage in ("accept", "recv", "parse", "handle", "send", "batch"):
        assert stage in prof, prof
    assert prof["accept"]["count"] == 3
    assert prof["parse"]["count"] == 15 and prof["handle"]["count"] == 15
    assert prof["batch"]["max"] >= 2  # pipelined requests handled from one recv()


def test_ipv6_listener(hola):
    """`--host ::1`: the listener is address-family agnostic (getaddrinfo)."""
    try:
        probe = socket.socket(socket.AF_INET6, socket.SOCK_STREAM)
        probe.bind(("::1", 0))
        probe.close()
    except OSError:
        pytest.skip("no IPv6 loopback here")
    s = hola(args=["--host", "::1"], env={"HOSTNAME": "v6"})
    with socket.create_connection(("::1", s.port), timeout=5) as c:
        c.sendall(b"GET /api/hola HTTP/1.1\r\nHost: [::1]\r\nConnection: close\r\n\r\n")
        data = b""
        while chunk := c.recv(65536):
            data += chunk
    assert data.startswith(b"HTTP/1.1 200 OK") and data.endswith(b"\r\n\r\nHola de v6")


@pytest.mark.skipif(shutil.which("taskset") is None or len(os.sched_getaffinity(0)) < 2, reason="needs taskset, 2 CPUs")
def test_workers_pin_to_an_exclusive_cpuset(hola):
    """A cpuset with exactly one CPU per worker (kubelet static CPU manager) pins the workers
    without --cpu-list; --no-pin opts out."""
    cpus = sorted(os.sched_getaffinity(0))[:2]
    wrap = ["taskset", "-c", ",".join(map(str, cpus))]
    s = hola(wrapper=wrap, threads=2)
    assert s.get("/api/hola")[0] == 200
    assert f"cpus={cpus[0]},{cpus[1]}" in s.log() or f"cpus={cpus[0]}-{cpus[1]}" in s.log(), s.log()
    s2 = hola(wrapper=wrap, threads=2, args=["--no-pin"])
    assert "cpus=unpinned" in s2.log(), s2.log()


@pytest.mark.parametrize("mode", [[], ["--epoll-lt"]], ids=["edge", "level"])
def test_request_then_fin_is_answered_and_closed_promptly(hola, mode):
    """A FIN that arrives with the request (same epoll edge) must still be seen: the server
    answers, then closes at once instead of waiting for the idle sweep."""
    s = hola(args=["--idle-timeout-ms", "5000", *mode])
    for payload, want in ((b"GET /api/hola HTTP/1.1\r\nHost: x\r\n\r\n", b"Hola de testhost"),
                          (b"GET /api/hola HTTP/1.1\r\nHost: x\r\nX-Partial: ", b"")):
        c = socket.create_connection(("127.0.0.1", s.port), timeout=3)
        c.sendall(payload)
        c.shutdown(socket.SHUT_WR)
        t0 = time.monotonic()
        data = b""
        while True:
            chunk = c.recv(65536)
            if not chunk:
                break
            data += chunk
        c.close()
        assert time.monotonic() - t0 < 1.0
        assert want in data


def test_loadgen_pipelined_batches_counted(hola):
    """hola_loadgen --pipeline: every response of a back-to-back batch is parsed and counted
    (the server answers a batch from one recv with one send)."""
    from hola_amd.parallel.loadgen import run_duration

    s = hola()
    out = run_duration([("127.0.0.1", s.port)], 4, 1, 0.5, 0.2, pipeline=8)
    lat = out["latency"]
    assert lat["errors"] == 0 and lat["non2xx"] == 0 and lat["count"] > 8 and lat["reconnects"] == 0


def test_loadgen_wrk_style_invocation(hola):
    """`hola_loadgen -t1 -c4 -d1s --latency http://host:port/path` as a drop-in for the wrk runs
    of BASELINE configs 2-4: wrk's glued options and duration suffix, text summary."""
    import subprocess

    from hola_amd.native import binary

    s = hola()
    r = subprocess.run([str(binary("hola_loadgen")), "-t1", "-c4", "-d1s", "--latency",
                        f"http://127.0.0.1:{s.port}/api/health"], capture_output=True, text=True, timeout=30)
    assert r.returncode == 0, r.stderr
    out = r.stdout
    assert out.startswith("Running 1s test @ http://127.0.0.1:") and "1 threads and 4 connections" in out
    assert "Latency Distribution" in out and "Requests/sec:" in out
    assert "Socket errors" not in out and "Non-2xx" not in out
    assert int(out.split(" requests in ")[0].split()[-1]) > 0


def test_loadgen_url_with_ipv6_literal(hola):
    """wrk-style URL with a bracketed IPv6 literal; the Host header carries the brackets."""
    import socket
    import subprocess

    from hola_amd.native import binary

    try:
        with socket.socket(socket.AF_INET6) as sk:
            sk.bind(("::1", 0))
    except OSError:
        pytest.skip("no IPv6 loopback")
    s = hola(args=["--host", "::1"])
    r = subprocess.run([str(binary("hola_loadgen")), "-t1", "-c2", "-d1", "--json",
                        f"http://[::1]:{s.port}/api/hola"], capture_output=True, text=True, timeout=30)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    assert out["rps"] > 0 and out["latency"]["errors"] == 0 and out["latency"]["non2xx"] == 0


def test_request_body_over_limit_is_413_and_closes(hola):
    """Request bodies are read and discarded (no route takes one); beyond 1 MiB the server
    answers 413 and closes, for Content-Length and for chunked bodies. WildFly's listener
    default is a 10 MB max-post-size; the lower bound here caps buffered bytes per
    connection (docs/PARITY.md)."""
    s = hola()
    out = _raw(s.port, b"POST /api/hola HTTP/1.1\r\nHost: x\r\nContent-Length: 2000000\r\n\r\n" + b"x" * 1000)
    assert out.startswith(b"HTTP/1.1 413") and b"Connection: close" in out
    chunk = b"%x\r\n%s\r\n" % (600000, b"y" * 600000)
    out = _raw(s.port, b"POST /api/hola HTTP/1.1\r\nHost: x\r\nTransfer-Encoding: chunked\r\n\r\n" + chunk * 2 + b"0\r\n\r\n")
    assert out.startswith(b"HTTP/1.1 413")
    # under the limit the body is skipped and the connection stays usable
    small = b"POST /api/hola HTTP/1.1\r\nHost: x\r\nContent-Length: 5\r\n\r\nhello"
    out = _raw(s.port, small + b"GET /api/health HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
    assert out.startswith(b"HTTP/1.1 405") and out.count(b"HTTP/1.1 200 OK") == 1 and out.endswith(b"I'm ok")


def test_path_parameters_are_ignored_for_matching(hola, native):
    """Undertow parses ";name=value" path parameters out of every segment before servlet and
    JAX-RS matching (a ;jsessionid, a matrix parameter), so they never change the route; an
    encoded %3B is not a delimiter (parity unpinned: no reference artefact covers it)."""
    assert native.strip_path_parameters("/api/hola;jsessionid=abc") == "/api/hola"
    assert native.strip_path_parameters("/api;v=1/hola;x;y=2/") == "/api/hola/"
    assert native.strip_path_parameters("/api/hola%3Bx") == "/api/hola%3Bx"
    s = hola(env={"HOSTNAME": "h"})
    assert s.get("/api/hola;jsessionid=abc")[2] == b"Hola de h"
    assert s.get("/api;v=1/hola")[2] == b"Hola de h"
    assert s.get("/api/health;x")[2] == b"I'm ok"
    assert s.get("/api/hola%3Bx")[0] == 404


def test_long_paths_are_canonicalised_too(hola):
    """Path parameters, escapes and dot segments are handled for paths of any length the
    request line allows, not only short ones."""
    s = hola(env={"HOSTNAME": "h"})
    assert s.get("/api/hola;jsessionid=" + "x" * 1500)[2] == b"Hola de h"
    assert s.get("/api/" + "a/../" * 300 + "hola")[2] == b"Hola de h"
    assert s.get("/api/" + "%7A/../" * 200 + "hola")[2] == b"Hola de h"
    assert s.get("/api/" + "%7A" * 600)[0] == 404


def _raw_exchange(sock, path: str = "/api/hola") -> tuple[int, dict, bytes]:
    """One request on a kept-alive socket; returns (status, headers, body)."""
    sock.sendall(f"GET {path} HTTP/1.1\r\nHost: x\r\n\r\n".encode())
    data = b""
    while b"\r\n\r\n" not in data:
        chunk = sock.recv(65536)
        if not chunk:
            raise ConnectionError("EOF before a response")
        data += chunk
    head, _, body = data.partition(b"\r\n\r\n")
    lines = head.decode().split("\r\n")
    hdrs = {k.lower(): v for k, v in (l.split(": ", 1) for l in lines[1:])}
    n = int(hdrs.get("content-length", "0"))
    while len(body) < n:
        chunk = sock.recv(65536)
        if not chunk:
            raise ConnectionError("EOF inside a body")
        body += chunk
    return int(lines[0].split()[1]), hdrs, body


def test_shutdown_delay_fails_readiness_but_keeps_serving(hola):
    """--shutdown-delay-ms: after SIGTERM the replica keeps accepting and serving for the delay,
    /api/health answers 503 (the readiness probe of pom.xml:90-94 fails, so the Service stops
    routing here), and every response carries `Connection: close` so kept-alive clients move
    elsewhere between requests. Then it drains and exits 0."""
    import signal

    s = hola(args=["--shutdown-delay-ms", "1500"])
    ka = socket.create_connection(("127.0.0.1", s.port), timeout=5)
    assert _raw_exchange(ka)[0] == 200
    t0 = time.monotonic()
    s.proc.send_signal(signal.SIGTERM)
    deadline = time.monotonic() + 5
    while "readiness failing" not in s.log() and time.monotonic() < deadline:
        time.sleep(0.01)
    st, h, body = _raw_exchange(ka)  # the kept-alive connection: served once more, then closed
    assert st == 200 and body == b"Hola de testhost" and h["connection"] == "close"
    assert ka.recv(10) == b""
    st, h, body = s.get("/api/health")  # a new connection is still accepted
    assert st == 503 and body == b"shutting down"
    assert b"hola_server_terminating 1" in s.get("/metrics")[2]
    st, h, body = s.get("/api/hola")
    assert st == 200 and body == b"Hola de testhost"
    assert s.proc.poll() is None
    assert s.proc.wait(timeout=10) == 0
    assert time.monotonic() - t0 >= 1.4
    log = s.log()
    assert "received SIGTERM: readiness failing, still serving for 1500 ms" in log
    assert "received SIGTERM: draining" in log


def test_second_signal_ends_the_shutdown_delay(hola):
    import signal

    s = hola(args=["--shutdown-delay-ms", "30000"])
    s.proc.send_signal(signal.SIGTERM)
    deadline = time.monotonic() + 5
    while "readiness failing" not in s.log() and time.monotonic() < deadline:
        time.sleep(0.01)
    t0 = time.monotonic()
    s.proc.send_signal(signal.SIGTERM)
    assert s.proc.wait(timeout=10) == 0
    assert time.monotonic() - t0 < 5
    assert "ending the delay early" in s.log()


def test_stop_and_continue_do_not_cut_the_shutdown_delay(hola):
    """SIGSTOP/SIGCONT (or a ptrace attach, such as the executor's stack sampler) interrupts
    the delay's sigtimedwait with EINTR; the replica waits out the rest of the delay instead of
    draining at once (it did, before)."""
    import signal

    s = hola(args=["--shutdown-delay-ms", "1500"])
    t0 = time.monotonic()
    s.proc.send_signal(signal.SIGTERM)
    deadline = time.monotonic() + 5
    while "readiness failing" not in s.log() and time.monotonic() < deadline:
        time.sleep(0.01)
    s.proc.send_signal(signal.SIGSTOP)
    time.sleep(0.1)
    s.proc.send_signal(signal.SIGCONT)
    time.sleep(0.5)
    assert s.proc.poll() is None, s.log()[-2000:]
    assert s.proc.wait(timeout=10) == 0
    assert time.monotonic() - t0 >= 1.4
    assert "ending the delay early" not in s.log()


def test_exit_deadline_ends_a_termination_that_runs_too_long(hola):
    """The exit watchdog: a termination still running --exit-deadline-ms after the signal (here
    a 30 s shutdown delay against a 1 s deadline) ends with status 3 and a line saying so,
    before the kubelet's SIGKILL would (terminationGracePeriodSeconds)."""
    import signal

    s = hola(args=["--shutdown-delay-ms", "30000", "--exit-deadline-ms", "1000"])
    s.expected_rc = 3
    t0 = time.monotonic()
    s.proc.send_signal(signal.SIGTERM)
    assert s.proc.wait(timeout=10) == 3
    # the report starts half way (a deadline under twice its 2.5 s budget), so the process has
    # exited by the deadline itself
    # (a sanitizer build takes longer over the report's stack walks)
    assert 0.45 <= time.monotonic() - t0 < (1.5 if not os.environ.get("HOLA_SANITIZER") else 4.0)
    assert "termination did not complete within 500 ms; exiting (exit deadline 1000 ms" in s.log()


def test_exit_watchdog_is_done_by_the_deadline_it_is_given(hola):
    """with --exit-deadline-ms set to the pod's terminationGracePeriodSeconds, the
    kubelet's SIGKILL comes at the deadline. The report (main's stack, every worker's) and
    the exit status 3 must come before it: the watchdog starts 2.5 s early."""
    import signal

    s = hola(args=["--shutdown-delay-ms", "30000", "--exit-deadline-ms", "6000"], threads=2)
    s.expected_rc = 3
    t0 = time.monotonic()
    s.proc.send_signal(signal.SIGTERM)
    assert s.proc.wait(timeout=15) == 3
    took = time.monotonic() - t0
    assert 3.4 <= took < (6.0 if not os.environ.get("HOLA_SANITIZER") else 8.0), took
    log = s.log()
    assert "termination did not complete within 3500 ms; exiting (exit deadline 6000 ms" in log
    assert re.search(r"hola: worker \d: pass \d+", log), log[-2000:]


def test_a_stuck_worker_cannot_hold_the_termination_forever(hola):
    """One worker thread held stopped (ptrace) stands for a worker stuck in its loop: the drain
    stops waiting for its answer (a warning names it), and the exit watchdog ends the process
    with status 3 at --exit-deadline-ms instead of hanging until a SIGKILL."""
    import ctypes
    import signal

    s = hola(args=["--drain-ms", "300", "--exit-deadline-ms", "3000"], threads=2)
    s.expected_rc = 3
    libc = ctypes.CDLL(None, use_errno=True)
    libc.ptrace.argtypes = [ctypes.c_long, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p]
    PTRACE_SEIZE, PTRACE_INTERRUPT, WALL = 0x4206, 0x4207, 0x40000000
    # the worker must be named and in its loop (blocked in epoll_wait) before it is stopped:
    # under load, or in a sanitizer build, it can still be starting when the listener is up
    deadline = time.monotonic() + 10
    tid = None
    while tid is None and time.monotonic() < deadline:
        tid = next((int(t.name) for t in Path(f"/proc/{s.proc.pid}/task").iterdir()
                    if (t / "comm").read_text().strip() == "hola-w1"), None)
        time.sleep(0.0 if tid else 0.02)
    assert tid is not None, "no hola-w1 thread"
    while "ep_poll" not in (Path(f"/proc/{s.proc.pid}/task/{tid}/wchan").read_text() or "") \
            and time.monotonic() < deadline:
        time.sleep(0.02)
    if libc.ptrace(PTRACE_SEIZE, tid, None, None) != 0:
        pytest.skip(f"ptrace not permitted here (errno {ctypes.get_errno()})")
    libc.ptrace(PTRACE_INTERRUPT, tid, None, None)
    os.waitpid(tid, WALL)  # hola-w1 is stopped now
    t0 = time.monotonic()
    s.proc.send_signal(signal.SIGTERM)
    # this process traces hola-w1, so it must reap that thread's exit itself, or the replica's
    # own exit status never reaches its parent (this process too)
    rc = None
    try:
        while rc is None and time.monotonic() - t0 < 20:
            try:
                os.waitpid(tid, os.WNOHANG | WALL)
            except ChildProcessError:
                pass
            rc = s.proc.poll()
            time.sleep(0.02)
    finally:
        if rc is None:  # let the thread go, so the fixture's teardown can stop the replica
            libc.ptrace(17, tid, None, None)  # PTRACE_DETACH
    took = time.monotonic() - t0
    log = s.log()
    assert rc == 3, (rc, log[-2000:])
    assert 1.4 <= took < 10
    assert "drain: worker 1 did not answer by the drain deadline" in log
    assert "termination did not complete within 1500 ms; exiting (exit deadline 3000 ms" in log
    # the stall report: where the stopped worker's loop was, and that it is not advancing
    # (held stopped in epoll_wait: a posted task would have woken a running loop)
    assert re.search(r"drain: worker did not answer: worker 1: pass \d+, phase wait, .*in epoll_wait, no pass over 100 ms", log), log
    print(log)


def test_default_exit_deadline_leaves_a_normal_termination_alone(hola):
    s = hola(args=["--shutdown-delay-ms", "200", "--drain-ms", "300"])
    import signal

    s.proc.send_signal(signal.SIGTERM)
    assert s.proc.wait(timeout=10) == 0
    assert "did not complete" not in s.log()


def test_every_thread_blocks_the_termination_signals(hola):
    """A process-directed SIGTERM goes to any thread that does not block it. Only main takes
    it (sigwait); a thread with it unblocked would die of its default action and take the
    replica with it, skipping the shutdown delay and the drain. The log writer, started while
    `--log-level` is parsed (before main blocks the signals), once was such a thread: the
    second SIGTERM of test_second_signal_ends_the_shutdown_delay killed the process."""
    import signal

    s = hola(args=["--shutdown-delay-ms", "1000"], threads=2)
    want = (1 << (signal.SIGTERM - 1)) | (1 << (signal.SIGINT - 1))
    names = []
    for task in Path(f"/proc/{s.proc.pid}/task").iterdir():
        if task.name == str(s.proc.pid):
            continue  # main: inside sigwait the waited signals show as unblocked
        status = (task / "status").read_text()
        fields = dict(line.split(":\t", 1) for line in status.splitlines() if ":\t" in line)
        if int(fields["SigBlk"], 16) & (1 << (signal.SIGSEGV - 1)):
            continue  # a sanitizer runtime's own thread (TSan's blocks everything); ours never block SIGSEGV
        names.append(fields["Name"].strip())
        assert int(fields["SigBlk"], 16) & want == want, (fields["Name"], fields["SigBlk"])
        # ... and only those: SIGPROF (--cpu-profile's sampling timer, the log writer
        # included) and the stall reports' capture signal (40) stay deliverable
        assert not int(fields["SigBlk"], 16) & (1 << (signal.SIGPROF - 1) | 1 << 39), (fields["Name"], fields["SigBlk"])
    assert "hola-log" in names, names


def test_drain_closes_busy_keepalive_connections_between_responses(hola):
    """Without a delay: SIGTERM while clients loop on kept-alive connections. Each client gets
    a complete response carrying `Connection: close` and then EOF; no request is left without
    a response (no close racing a request that was already on its way)."""
    import signal
    import threading

    s = hola(threads=2)
    results = []

    def client():
        c = socket.create_connection(("127.0.0.1", s.port), timeout=5)
        n, last = 0, None
        try:
            while True:
                st, h, _ = _raw_exchange(c)
                assert st == 200
                n += 1
                last = h.get("connection")
                if last == "close":
                    break
            results.append(("ok", n, c.recv(10)))
        except Exception as e:  # noqa: BLE001
            results.append(("error", n, repr(e)))

    ts = [threading.Thread(target=client) for _ in range(4)]
    for t in ts:
        t.start()
    time.sleep(0.3)
    s.proc.send_signal(signal.SIGTERM)
    for t in ts:
        t.join(timeout=10)
    assert s.proc.wait(timeout=10) == 0
    assert len(results) == 4 and all(r[0] == "ok" and r[1] > 0 and r[2] == b"" for r in results), results


def test_no_keepalive_response_is_followed_by_a_close_when_termination_begins(hola):
    """SIGTERM under closed-loop keep-alive load, many times: a response that announced
    keep-alive is never followed by the server closing that connection. The Connection header
    and the close decision come from one read of the closing flag; before that fix the server
    read it again after the handler, so a SIGTERM landing between the two reads closed a
    connection right after a keep-alive response, and the client's next request failed
    (7 loadgen errors in 80 terminations on the old binary, 0 after)."""
    import json as _json
    import signal
    import subprocess

    from hola_amd import native

    loadgen = str(native.binary("hola_loadgen"))
    errors = requests = 0
    for _ in range(40):
        s = hola(args=["--shutdown-delay-ms", "150", "--log-level", "warn"], threads=2)
        lg = subprocess.Popen([loadgen, "-t", "2", "-c", "32", "-d", "5s", "--json", f"{s.url}/api/hola"],
                              stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
        time.sleep(0.25)
        s.proc.send_signal(signal.SIGTERM)
        time.sleep(0.1)  # inside the delay: the clients are being moved off with Connection: close
        lg.send_signal(signal.SIGINT)
        out, _ = lg.communicate(timeout=30)
        assert s.proc.wait(timeout=10) == 0
        lat = _json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])["latency"]
        errors += lat["errors"]
        requests += lat["count"]
    assert requests > 10000
    assert errors == 0, errors


def _metric_value(s, name: str) -> float:
    for line in s.get("/metrics")[2].decode().splitlines():
        if line.startswith(name + " "):
            return float(line.split()[1])
    raise AssertionError(f"{name} missing")


def test_adaptive_busy_poll_resumes_when_load_returns(hola, hola_bin):
    """A worker that backed off its spin under light load spins again as soon as its blocking
    waits show events arriving within the spin budget, not at the end of its (up to 1.6 s)
    back-off: a saturated loop pushed off by a momentary stall must not stay in the slow,
    sleep-and-wake-up state (profiles/round5/02_chain_modes)."""
    import json as _json
    import subprocess

    s = hola(args=["--busy-poll-us", "auto"], threads=1)
    for _ in range(300):  # light load: back-offs escalate towards 1.6 s
        assert s.get("/api/hola")[0] == 200
        time.sleep(0.005)
    assert _metric_value(s, "hola_busy_poll_backoffs_total") >= 1
    loadgen = hola_bin.parent / "hola_loadgen"
    r = subprocess.run([str(loadgen), "-t", "1", "-c", "16", "-d", "1s", "--json", f"{s.url}/api/hola"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert _json.loads(r.stdout.strip().splitlines()[-1])["latency"]["errors"] == 0
    assert _metric_value(s, "hola_busy_poll_resumes_total") >= 1


def test_adaptive_busy_poll_backs_off_under_light_load(hola):
    """`--busy-poll-us auto`: spinning that mostly waits in vain (requests 10 ms apart) is
    switched off, so a lightly loaded replica does not burn its CPU; an idle one sleeps."""
    s = hola(args=["--busy-poll-us", "auto"], threads=1)
    for _ in range(150):
        assert s.get("/api/hola")[0] == 200
        time.sleep(0.01)
    assert _metric_value(s, "hola_busy_poll_backoffs_total") >= 1
    body = s.get("/metrics")[2].decode()
    hits = float(next(l for l in body.splitlines() if 'result="hit"' in l).split()[1])
    misses = float(next(l for l in body.splitlines() if 'result="miss"' in l).split()[1])
    assert misses > hits
    # idle: well under a tenth of a CPU
    cpu = lambda: sum(int(x) for x in open(f"/proc/{s.proc.pid}/stat").read().rsplit(")", 1)[1].split()[11:13])  # noqa: E731
    c0 = cpu()
    time.sleep(1.0)
    assert (cpu() - c0) / os.sysconf("SC_CLK_TCK") < 0.1


def test_exit_watchdog_reports_where_every_worker_is(hola):
    """The exit watchdog's stall report: for each worker its loop's pass counter, phase and last
    handler, and its stack, taken in the worker by a signal whose handler walks the frame
    pointers. Here the termination outlasts --exit-deadline-ms (a 5 s delay against a 1 s
    limit), so the workers are alive and waiting in epoll: their stacks name the event loop."""
    import signal
    import subprocess

    s = hola(args=["--shutdown-delay-ms", "5000", "--exit-deadline-ms", "1000"], threads=2)
    s.expected_rc = 3
    s.get("/api/hola")  # one request: worker 0 or 1 has run a connection handler
    s.proc.send_signal(signal.SIGTERM)
    assert s.proc.wait(timeout=10) == 3
    log = s.log()
    reports = re.findall(r"hola: worker (\d): pass (\d+), phase (\w+), .*?; stack((?: #\d+ \S+)+)", log)
    assert {r[0] for r in reports} == {"0", "1"}, log[-3000:]
    exe = str(s.exe)
    # Under TSan, epoll_wait and sigtimedwait are intercepted by libtsan, whose frames keep no
    # frame pointer: the walk ends there (test_sanitizers.py checks that report on its own).
    walks_through = os.environ.get("HOLA_SANITIZER") != "tsan"
    for worker, passes, phase, stack in reports:
        assert phase == "wait" and int(passes) >= 1, (worker, phase)
        if not walks_through:
            continue
        frames = re.findall(r"#\d+ (\S+)\+0x([0-9a-f]+)", stack)
        own = [off for obj, off in frames if obj == Path(exe).name]
        assert own, stack
        names = subprocess.run(["addr2line", "-f", "-C", "-e", exe, *[f"0x{o}" for o in own]],
                               capture_output=True, text=True).stdout
        assert "hola::EventLoop::run()" in names, names
    # the connection handler's record is decoded with its state bits
    assert re.search(r"last handler (connection [0-9a-f]+ \{[a-z_,]*\} in=\d+ unsent=\d+|loop-internal)", log), log
    # and main says which termination step it is in, with its own stack
    m = re.search(r"hola: main: shutdown delay; stack((?: #\d+ \S+)+)", log)
    assert m, log[-3000:]
    if not walks_through:
        return
    own = [off for obj, off in re.findall(r"#\d+ (\S+)\+0x([0-9a-f]+)", m.group(1)) if obj == Path(exe).name]
    names = subprocess.run(["addr2line", "-f", "-C", "-e", exe, *[f"0x{o}" for o in own]],
                           capture_output=True, text=True).stdout
    assert re.search(r"^main$", names, re.M), names


def test_date_header_is_current_after_an_idle_spell(hola):
    """The worker refreshes its Date header after its wait, as of the pass's own time (every
    4 ms of loop time at most): the first response after an idle spell carries the current
    second, not the one from before the loop went to sleep."""
    import email.utils

    s = hola(threads=1, args=["--busy-poll-us", "0"])
    st, h, _ = s.get("/api/health")
    assert st == 200
    time.sleep(2.5)
    st, h, _ = s.get("/api/health")
    sent = email.utils.parsedate_to_datetime(h["date"]).timestamp()
    assert abs(sent - time.time()) < 1.5, h["date"]


def test_sched_slice_option_reaches_the_workers(hola):
    """--sched-slice-us N: every worker asks the scheduler for an N us time slice (EEVDF custom
    slice), and /metrics reports the slice the kernel gave it. Kernels without custom slices
    report none, and the gauge is then absent."""
    s = hola(args=["--sched-slice-us", "500"])
    body = s.get("/metrics")[2].decode()
    vals = [float(l.split()[1]) for l in body.splitlines() if l.startswith("hola_worker_sched_slice_seconds ")]
    if vals:
        assert abs(vals[0] - 0.0005) < 1e-6, vals
