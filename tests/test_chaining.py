"""GET /api/hola-chaining against a fake aloha: success path, every failure mode falling
back to ["Aloha response (fallback)"] (HolaResource.java:111-112), the 600 ms timeout
(config.properties:17), the circuit breaker (config.properties:19) and the bulkhead."""
import json
import re
import socket
import threading
import time

import pytest

from hola_amd.testing.fakes import FakeAloha, closed_port

FALLBACK = "Aloha response (fallback)"


@pytest.fixture
def aloha():
    a = FakeAloha().start()
    yield a
    a.stop()


def chain(s):
    st, h, body = s.get("/api/hola-chaining", timeout=10)
    assert st == 200, body
    return json.loads(body)


def test_success_appends_aloha_list(hola, aloha):
    s = hola(args=["--aloha-url", aloha.url, "--no-tracing"], env={"HOSTNAME": "h"})
    assert chain(s) == ["Hola de h", "Aloha mai aloha-1", "Bonjour de bonjour-1"]
    assert aloha.requests[-1]["path"] == "/api/aloha-chaining"


@pytest.mark.parametrize("payload", [
    ["Aloha mai aloha-1", "Bonjour de bonjour-1"],
    [],
    ["één", "a/b", "x"],
    ['say "hi"', "back\\slash", "tab\tnl\n"],
    ["a", None, "b"],
    ["Aloha", 7, True],
])
def test_list_passed_on_as_written_or_reencoded_gives_the_same_body(hola, aloha, payload):
    """A list of plain strings written compactly (as Jackson writes one) is passed on as text
    (json::plain_string_list); any other list is decoded and re-encoded. Both give the body
    Jackson would: the same bytes for the same elements, whatever aloha's whitespace."""
    aloha.payload = payload
    s = hola(args=["--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none"], env={"HOSTNAME": "h"})
    bodies = []
    for mode in ("compact", "ok"):
        aloha.set_mode(mode)
        st, h, body = s.get("/api/hola-chaining", timeout=10)
        assert st == 200, body
        assert int(h["content-length"]) == len(body)
        bodies.append(body)
    assert bodies[0] == bodies[1]
    want = ["Hola de h"] + [None if v is None else (str(v).lower() if isinstance(v, bool) else str(v)) for v in payload]
    assert json.loads(bodies[0]) == want
    assert bodies[0] == json.dumps(want, separators=(",", ":"), ensure_ascii=False).encode()


def test_keepalive_reuse(hola, aloha):
    s = hola(args=["--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none"], threads=1)
    for _ in range(5):
        assert chain(s)[1] == "Aloha mai aloha-1"
    st, _, body = s.get("/metrics")
    assert st == 200


@pytest.mark.parametrize("mode", ["chunked", "chunked_lf"])
def test_chunked_response(hola, aloha, mode):
    aloha.set_mode(mode)
    s = hola(args=["--aloha-url", aloha.url])
    for _ in range(3):  # also over the kept-alive connection
        assert chain(s)[1:] == ["Aloha mai aloha-1", "Bonjour de bonjour-1"]


def test_header_name_with_a_cr_is_not_a_known_field(hola, aloha):
    """the client's case fold must not map CR onto '-': "Transfer\rEncoding:
    chunked" is some other header, so the Content-Length body is read as is (a chunked
    decode of it would fail and fall back)."""
    aloha.set_mode("cr_in_name")
    s = hola(args=["--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none"], env={"HOSTNAME": "h"})
    for _ in range(2):
        assert chain(s) == ["Hola de h", "Aloha mai aloha-1", "Bonjour de bonjour-1"]


@pytest.mark.parametrize("mode", ["cl_unparseable", "te_not_chunked"])
def test_response_framing_as_httpclient_reads_it(hola, aloha, mode):
    """Framing read like HttpClient 4.5's LaxContentLengthStrategy: a Content-Length that
    does not parse as a number is skipped for the one before it, and a Transfer-Encoding whose
    last coding is not chunked makes the body run to the connection's close, whatever
    Content-Length says (RFC 9112 §6.3)."""
    aloha.set_mode(mode)
    s = hola(args=["--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none"], env={"HOSTNAME": "h"})
    for _ in range(2):
        assert chain(s) == ["Hola de h", "Aloha mai aloha-1", "Bonjour de bonjour-1"]
    assert _events(s).get("SUCCESS") == 2


@pytest.mark.parametrize("pipeline", [1, 8])
def test_interim_1xx_responses_are_read_past(hola, aloha, pipeline):
    """aloha (or a front) sends 100 Continue and 103 Early Hints before each final response,
    unasked: HttpClient reads past interim responses, so the call succeeds (not A's fallback)
    and the connection stays in step for the next call, pipelined or not."""
    aloha.set_mode("interim")
    s = hola(args=["--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none",
                   "--aloha-pipeline", str(pipeline)], env={"HOSTNAME": "h"}, threads=1)
    for _ in range(4):
        assert chain(s) == ["Hola de h", "Aloha mai aloha-1", "Bonjour de bonjour-1"]
    assert len({r["peer_port"] for r in aloha.requests}) == 1  # one kept-alive connection
    assert _events(s).get("SUCCESS") == 4


def test_interim_then_close_is_a_transport_retry(hola, aloha):
    """a 100 Continue is not an answer. HttpClient 4.5 reads past it inside
    execute(); a connection that then closes before the final head throws
    NoHttpResponseException there, which DefaultHttpRequestRetryHandler re-sends for an
    idempotent GET. So the call is re-sent on a fresh connection and succeeds."""
    aloha.set_mode("interim_close_once")
    s = hola(args=["--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none", "--feign-retry", "off"],
             env={"HOSTNAME": "h"}, threads=1)
    assert chain(s) == ["Hola de h", "Aloha mai aloha-1", "Bonjour de bonjour-1"]
    assert len(aloha.requests) == 2
    assert _events(s).get("SUCCESS") == 1


@pytest.mark.parametrize("pipeline", [1, 8])
def test_interim_flood_is_bounded(hola, aloha, pipeline):
    """interim responses before a final one are capped at 64 KiB per call (they are
    dropped as they are read, never re-parsed). 96 KiB of 100 Continue is a malformed answer:
    the fallback, at once rather than at the 600 ms timeout."""
    aloha.set_mode("interim_flood")
    s = hola(args=["--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none", "--feign-retry", "off",
                   "--aloha-pipeline", str(pipeline)], env={"HOSTNAME": "h"}, threads=1)
    t0 = time.monotonic()
    assert chain(s) == ["Hola de h", FALLBACK]
    assert time.monotonic() - t0 < 0.5
    assert _events(s).get("TIMEOUT", 0) == 0


def _events(s) -> dict:
    """Rolling Hystrix event counts of the aloha command from /metrics."""
    _, _, body = s.get("/metrics")
    out = {}
    for line in body.decode().splitlines():
        if line.startswith("hola_hystrix_events_total{"):
            out[line.split('event="')[1].split('"')[0]] = int(float(line.rsplit(" ", 1)[1]))
    return out


def _wait_log(s, needle: str, count: int, timeout: float = 3.0) -> str:
    deadline = time.monotonic() + timeout
    while True:
        log = s.log()
        if log.count(needle) >= count or time.monotonic() > deadline:
            return log
        time.sleep(0.05)


@pytest.mark.parametrize("mode", ["error", "garbage"])
def test_response_failures_fall_back_fast_without_retry(hola, aloha, mode):
    """A 500 (FeignException) or an undecodable body (DecodeException) is not retryable:
    one HTTP execution, FAILURE at once."""
    aloha.set_mode(mode)
    s = hola(args=["--aloha-url", aloha.url])
    t0 = time.monotonic()
    assert chain(s) == ["Hola de testhost", FALLBACK]
    assert time.monotonic() - t0 < 0.3
    assert len(aloha.requests) == 1
    ev = _events(s)
    assert ev.get("FAILURE") == 1 and ev.get("TIMEOUT", 0) == 0


def test_dropped_connection_is_retried_until_the_hystrix_timeout(hola, aloha):
    """aloha closes without answering: NoHttpResponseException, an IOException. Apache
    HttpClient re-executes the GET 3 times on fresh connections, then Feign's Retryer sleeps
    150/225/... ms between attempts until the 600 ms Hystrix timeout wins (TIMEOUT)."""
    aloha.set_mode("close")
    s = hola(args=["--aloha-url", aloha.url])
    t0 = time.monotonic()
    assert chain(s) == ["Hola de testhost", FALLBACK]
    assert 0.55 <= time.monotonic() - t0 < 1.0
    # Feign attempts at ~0, 150, 375 ms, each 1 + 3 transport tries
    assert len(aloha.requests) == 12
    assert _events(s).get("TIMEOUT") == 1
    _, _, body = s.get("/metrics")
    assert b'hola_aloha_retries_total{kind="feign"} 2' in body
    assert b'hola_aloha_retries_total{kind="transport"} 9' in body


def test_connection_refused_retries_until_timeout_then_opens(hola):
    """Feign's default Retryer (HolaResource.java:104-112 sets none) retries the refused
    connect at +150 ms and +375 ms; the next sleep (337 ms) would end past the 600 ms Hystrix
    timeout (config.properties:17), so the call is a TIMEOUT at ~600 ms. After
    requestVolumeThreshold=5 (config.properties:19) such calls the breaker opens and
    short-circuits at once."""
    s = hola(args=["--aloha-url", f"http://127.0.0.1:{closed_port()}/",
                   "-Dhystrix.command.default.metrics.healthSnapshot.intervalInMilliseconds=0"])
    for _ in range(5):
        t0 = time.monotonic()
        assert chain(s)[1:] == [FALLBACK]
        assert 0.55 <= time.monotonic() - t0 < 1.0
    t0 = time.monotonic()
    assert chain(s)[1:] == [FALLBACK]
    assert time.monotonic() - t0 < 0.3  # short-circuited
    ev = _events(s)
    assert ev.get("TIMEOUT") == 5 and ev.get("SHORT_CIRCUITED") == 1 and ev.get("FAILURE", 0) == 0
    log = _wait_log(s, "---> GET", 15)
    assert log.count("[AlohaService#aloha] ---> GET ") == 15  # 3 attempts x 5 calls
    assert log.count("[AlohaService#aloha] ---> RETRYING") == 10
    assert "[AlohaService#aloha] <--- ERROR HttpHostConnectException: Connect to 127.0.0.1:" in log
    # The SSE stream shows the same rolling counts.
    with socket.create_connection(("127.0.0.1", s.port), timeout=5) as c:
        c.sendall(b"GET /hystrix.stream HTTP/1.1\r\nHost: x\r\n\r\n")
        data = b""
        while b'"type":"HystrixCommand"' not in data or not data.rstrip().endswith(b"}"):
            data += c.recv(65536)
    cmd = json.loads(next(l for l in data.decode().splitlines()
                          if l.startswith("data:") and '"HystrixCommand"' in l)[5:])
    assert cmd["rollingCountTimeout"] == 5 and cmd["isCircuitBreakerOpen"] is True


def test_feign_retry_off_fails_fast(hola):
    s = hola(args=["--aloha-url", f"http://127.0.0.1:{closed_port()}/", "--feign-retry", "off"])
    t0 = time.monotonic()
    assert chain(s)[1:] == [FALLBACK]
    assert time.monotonic() - t0 < 0.3
    assert _events(s).get("FAILURE") == 1


def test_retries_exhaust_before_a_long_timeout(hola):
    """With a generous Hystrix timeout the Retryer gives up after max_attempts executions and
    the command is a FAILURE (RetryableException propagated)."""
    s = hola(args=["--aloha-url", f"http://127.0.0.1:{closed_port()}/", "--hystrix-timeout-ms", "5000",
                   "--feign-retry", "10,1000,5"])
    t0 = time.monotonic()
    assert chain(s)[1:] == [FALLBACK]
    dt = time.monotonic() - t0
    assert 0.1 <= dt < 0.5, dt  # sleeps 15 + 22 + 33 + 50 ms
    assert _events(s).get("FAILURE") == 1
    log = _wait_log(s, "---> GET", 5)
    assert log.count("---> GET ") == 5 and log.count("---> RETRYING") == 4


def test_retry_after_makes_an_error_status_retryable(hola, aloha):
    """ErrorDecoder.Default: a non-2xx response with Retry-After is a RetryableException.
    Retry-After: 0 retries at once (5 executions, then FAILURE); a 1 s Retry-After is capped
    at the 1 s max period, so the 600 ms Hystrix timeout fires first."""
    aloha.set_mode("unavailable")
    s = hola(args=["--aloha-url", aloha.url, "--hystrix-request-volume", "100"])
    t0 = time.monotonic()
    assert chain(s)[1:] == [FALLBACK]
    assert time.monotonic() - t0 < 0.3
    assert len(aloha.requests) == 5
    assert _events(s).get("FAILURE") == 1
    aloha.retry_after = "1"
    t0 = time.monotonic()
    assert chain(s)[1:] == [FALLBACK]
    assert 0.55 <= time.monotonic() - t0 < 1.0
    assert len(aloha.requests) == 6
    assert _events(s).get("TIMEOUT") == 1
    log = _wait_log(s, "<--- HTTP/1.1 503", 6)
    assert "[AlohaService#aloha] <--- HTTP/1.1 503 Service Unavailable (" in log


def test_unknown_host_retries_until_timeout(hola):
    s = hola(args=["--aloha-url", "http://aloha.invalid:8080/"])
    t0 = time.monotonic()
    assert chain(s)[1:] == [FALLBACK]
    assert 0.55 <= time.monotonic() - t0 < 1.0
    assert _events(s).get("TIMEOUT") == 1
    log = _wait_log(s, "UnknownHostException", 1)
    assert "[AlohaService#aloha] <--- ERROR UnknownHostException: " in log


def test_timeout_600ms(hola, aloha):
    aloha.set_mode("slow", delay_s=2.0)
    s = hola(args=["--aloha-url", aloha.url])
    t0 = time.monotonic()
    assert chain(s)[1:] == [FALLBACK]
    dt = time.monotonic() - t0
    assert 0.55 <= dt < 1.5, dt


def test_timeout_is_configurable(hola, aloha):
    aloha.set_mode("slow", delay_s=1.0)
    s = hola(args=["--aloha-url", aloha.url,
                   "-Dhystrix.command.default.execution.isolation.thread.timeoutInMilliseconds=150"])
    t0 = time.monotonic()
    assert chain(s)[1:] == [FALLBACK]
    assert time.monotonic() - t0 < 0.6


def test_circuit_opens_after_volume_threshold(hola, aloha):
    aloha.set_mode("error")
    s = hola(args=["--aloha-url", aloha.url, "--feign-log", "none",
                   "-Dhystrix.command.default.metrics.healthSnapshot.intervalInMilliseconds=0"])
    for _ in range(5):  # requestVolumeThreshold=5, 100 % errors
        assert chain(s)[1:] == [FALLBACK]
    n_before = len(aloha.requests)
    aloha.set_mode("ok")
    for _ in range(5):  # open: short-circuited, aloha is not called
        assert chain(s)[1:] == [FALLBACK]
    assert len(aloha.requests) == n_before
    st, _, body = s.get("/metrics")
    assert b'hola_hystrix_circuit_open{command="aloha"} 1' in body
    assert b'event="SHORT_CIRCUITED"' in body


def test_circuit_half_open_recovers_after_sleep_window(hola, aloha):
    aloha.set_mode("error")
    s = hola(args=["--aloha-url", aloha.url, "--feign-log", "none",
                   "-Dhystrix.command.default.metrics.healthSnapshot.intervalInMilliseconds=0",
                   "-Dhystrix.command.default.circuitBreaker.sleepWindowInMilliseconds=300"])
    for _ in range(6):
        chain(s)
    aloha.set_mode("ok")
    assert chain(s)[1:] == [FALLBACK]  # still open
    time.sleep(0.4)
    assert chain(s)[1] == "Aloha mai aloha-1"  # single trial succeeds -> closed
    assert chain(s)[1] == "Aloha mai aloha-1"


def test_bulkhead_rejects_beyond_pool(hola, aloha):
    aloha.set_mode("slow", delay_s=0.4)
    s = hola(args=["--aloha-url", aloha.url, "--feign-log", "none",
                   "-Dhystrix.threadpool.default.coreSize=2",
                   "-Dhystrix.command.default.circuitBreaker.enabled=false"], threads=1)
    results = []

    def one():
        results.append(chain(s))

    ts = [threading.Thread(target=one) for _ in range(5)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    ok = [r for r in results if r[1] != FALLBACK]
    assert len(ok) == 2 and len(results) == 5
    st, _, body = s.get("/metrics")
    assert b'event="THREAD_POOL_REJECTED"' in body


def test_semaphore_isolation_rejects_beyond_max_concurrent(hola, aloha):
    aloha.set_mode("slow", delay_s=1.0)
    s = hola(args=["--aloha-url", aloha.url, "--feign-log", "none", "--no-tracing",
                   "-Dhystrix.command.default.execution.isolation.strategy=SEMAPHORE",
                   "-Dhystrix.command.default.execution.isolation.semaphore.maxConcurrentRequests=1",
                   "-Dhystrix.command.default.execution.isolation.thread.timeoutInMilliseconds=3000",
                   "-Dhystrix.command.default.circuitBreaker.enabled=false"], threads=2)
    results = []
    ts = [threading.Thread(target=lambda: results.append(chain(s))) for _ in range(3)]
    for t in ts:
        t.start()
        time.sleep(0.05)
    for t in ts:
        t.join()
    assert sorted(r[1] == FALLBACK for r in results) == [False, True, True]
    body = s.get("/metrics")[2]
    assert b'event="SEMAPHORE_REJECTED"} 2' in body and b"THREAD_POOL_REJECTED" not in body


def test_feign_read_timeout_when_hystrix_timeout_is_disabled(hola, aloha):
    """With execution.timeout.enabled=false nothing but Feign's Request.Options ends a call to
    an aloha that never answers: each attempt fails as SocketTimeoutException after the read
    timeout (an IOException, so Feign retries), then the command fails to the fallback. The
    bulkhead slot is released instead of being held for good."""
    aloha.set_mode("slow", delay_s=3.0)
    s = hola(args=["--aloha-url", aloha.url, "--feign-timeouts", "10000,300", "--feign-retry", "100,1000,2",
                   "-Dhystrix.command.default.execution.timeout.enabled=false",
                   "-Dhystrix.threadpool.default.coreSize=1"], threads=1)
    t0 = time.monotonic()
    assert chain(s)[1] == FALLBACK
    took = time.monotonic() - t0
    assert 0.65 <= took < 1.5, took  # 300 ms, 150 ms sleep, 300 ms
    m = s.get("/metrics")[2]
    assert b'event="FAILURE"} 1' in m and b"TIMEOUT" not in m
    assert b'hola_aloha_retries_total{kind="feign"} 1' in m
    assert b'hola_hystrix_pool_active{command="aloha"} 0' in m
    assert "<--- ERROR SocketTimeoutException: Read timed out" in _wait_log(s, "<--- ERROR SocketTimeoutException", 1)


def _metric(s, name) -> int:
    for line in s.get("/metrics")[2].decode().splitlines():
        if line.startswith(name + " "):
            return int(float(line.split()[1]))
    raise AssertionError(f"{name} missing from /metrics")


def test_read_timeouts_do_not_pile_up_timers(hola, aloha):
    """With the Hystrix timeout disabled, every aloha request is guarded by Feign's 60 s read
    timeout. Finished requests must not leave their timeout behind: the loop's pending timers
    follow the calls in flight, not calls x 60 s (a timer per request would reach millions at
    the chaining rate)."""
    s = hola(args=["--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none",
                   "-Dhystrix.command.default.execution.timeout.enabled=false"], threads=1)
    idle = _metric(s, "hola_event_loop_timers")
    for _ in range(200):
        assert chain(s)[1] == "Aloha mai aloha-1"
    assert _metric(s, "hola_event_loop_timers") <= idle + 4  # a timer each: read FIFO, sweep, ticks
    # the read timeout still fires for a request that gets no answer
    aloha.set_mode("slow", delay_s=3.0)
    s2 = hola(args=["--aloha-url", aloha.url, "--no-tracing", "--feign-timeouts", "10000,200", "--feign-retry", "off",
                    "-Dhystrix.command.default.execution.timeout.enabled=false"], threads=1)
    t0 = time.monotonic()
    assert chain(s2)[1] == FALLBACK
    assert 0.15 <= time.monotonic() - t0 < 1.0
    assert "<--- ERROR SocketTimeoutException: Read timed out" in _wait_log(s2, "<--- ERROR SocketTimeoutException", 1)


def test_feign_connect_timeout(hola):
    """A connect that never completes (aloha's accept queue is full, so its SYNs are dropped)
    fails as ConnectTimeoutException after Feign's connect timeout, and is retried by Feign."""
    srv = socket.socket()
    srv.bind(("127.0.0.1", 0))
    srv.listen(0)
    filler = socket.create_connection(srv.getsockname())  # the one queued connection
    try:
        s = hola(args=["--aloha-url", "http://127.0.0.1:%d/" % srv.getsockname()[1], "--feign-timeouts", "300,60000",
                       "--feign-retry", "100,1000,2", "-Dhystrix.command.default.execution.timeout.enabled=false"],
                 threads=1)
        t0 = time.monotonic()
        assert chain(s)[1] == FALLBACK
        took = time.monotonic() - t0
        assert 0.65 <= took < 1.5, took  # 300 ms, 150 ms sleep, 300 ms
        line = "<--- ERROR ConnectTimeoutException: Connect to 127.0.0.1:%d failed: connect timed out" % srv.getsockname()[1]
        log = _wait_log(s, line, 1)
        assert line in log, log
        assert b'hola_aloha_retries_total{kind="feign"} 1' in s.get("/metrics")[2]
    finally:
        filler.close()
        srv.close()


def test_fallback_disabled_turns_failures_into_500(hola):
    """hystrix.command.default.fallback.enabled=false: a failed aloha call raises
    HystrixRuntimeException out of aloha(), so holaChaining() fails with a 500 and no
    fallback is counted."""
    s = hola(args=["--aloha-url", f"http://127.0.0.1:{closed_port()}/", "--feign-retry", "off", "--feign-log", "none",
                   "-Dhystrix.command.default.fallback.enabled=false"])
    st, h, body = s.get("/api/hola-chaining")
    assert st == 500 and "access-control-allow-origin" not in h
    m = s.get("/metrics")[2]
    assert b'event="FAILURE"} 1' in m and b"FALLBACK_SUCCESS" not in m
    # /api/hola is unaffected
    assert s.get("/api/hola")[0] == 200


def _gauge(s, name: str) -> int:
    body = s.get("/metrics")[2].decode()
    return int(next(l.rsplit(" ", 1)[1] for l in body.splitlines() if l.startswith(name + "{")))


def test_pool_queue_serves_waiting_calls_in_order(hola, aloha):
    """-Dhystrix.threadpool.default.maxQueueSize=2: with one pool slot and a slow aloha, two
    more calls wait in the queue and are served one after another within the timeout; a
    fourth is rejected to the fallback at once."""
    aloha.set_mode("slow", delay_s=0.5)
    s = hola(args=["--aloha-url", aloha.url, "--feign-log", "none", "--no-tracing",
                   "-Dhystrix.threadpool.default.coreSize=1", "-Dhystrix.threadpool.default.maxQueueSize=2",
                   "-Dhystrix.threadpool.default.queueSizeRejectionThreshold=2",
                   "-Dhystrix.command.default.execution.isolation.thread.timeoutInMilliseconds=4000",
                   "-Dhystrix.command.default.circuitBreaker.enabled=false"], threads=2)
    results = []

    def one():
        t0 = time.monotonic()
        body = chain(s)
        results.append((body[1] == FALLBACK, time.monotonic() - t0))

    ts = []
    for _ in range(4):
        ts.append(threading.Thread(target=one))
        ts[-1].start()
        time.sleep(0.05)
    time.sleep(0.1)
    assert _gauge(s, "hola_hystrix_pool_queued") == 2 and _gauge(s, "hola_hystrix_pool_active") == 1
    for t in ts:
        t.join()
    rejected = [took for fb, took in results if fb]
    served = sorted(took for fb, took in results if not fb)
    assert len(rejected) == 1 and rejected[0] < 0.4, results  # the queue was full: at once
    # one at a time through the single slot: ~0.5, ~1.0, ~1.5 s after arrival
    assert len(served) == 3 and served[0] < 0.9 and served[1] >= 0.8 and served[2] >= 1.3, results
    assert _gauge(s, "hola_hystrix_pool_queued") == 0 and _gauge(s, "hola_hystrix_pool_active") == 0
    assert b'event="THREAD_POOL_REJECTED"} 1' in s.get("/metrics")[2]


def test_pool_queue_under_timeouts_leaks_no_slot(hola, aloha):
    """Queue, timeouts and rejections racing across two workers: afterwards no slot is held
    and nothing waits, and the next call goes straight through."""
    aloha.set_mode("slow", delay_s=0.08)
    s = hola(args=["--aloha-url", aloha.url, "--feign-log", "none", "--no-tracing",
                   "-Dhystrix.threadpool.default.coreSize=2", "-Dhystrix.threadpool.default.maxQueueSize=4",
                   "-Dhystrix.threadpool.default.queueSizeRejectionThreshold=4",
                   "-Dhystrix.command.default.execution.isolation.thread.timeoutInMilliseconds=150",
                   "-Dhystrix.command.default.circuitBreaker.enabled=false"], threads=2)
    outcomes = []

    def burst():
        for _ in range(6):
            outcomes.append(chain(s)[1])

    ts = [threading.Thread(target=burst) for _ in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert len(outcomes) == 48
    assert FALLBACK in outcomes and any(o != FALLBACK for o in outcomes)
    time.sleep(0.3)
    assert _gauge(s, "hola_hystrix_pool_active") == 0 and _gauge(s, "hola_hystrix_pool_queued") == 0
    aloha.set_mode("ok")
    assert chain(s)[1] != FALLBACK
    body = s.get("/metrics")[2].decode()
    assert 'event="TIMEOUT"' in body and 'event="SUCCESS"' in body


def _histogram(body: bytes, name: str) -> tuple[dict, float, int]:
    buckets, total, count = {}, None, None
    for line in body.decode().splitlines():
        if line.startswith(name + "_bucket{le=\""):
            le = line.split('"')[1]
            buckets[le] = int(line.rsplit(" ", 1)[1])
        elif line.startswith(name + "_sum "):
            total = float(line.split()[1])
        elif line.startswith(name + "_count "):
            count = int(line.split()[1])
    return buckets, total, count


def test_chaining_latency_histogram(hola, aloha):
    s = hola(args=["--aloha-url", aloha.url, "--feign-log", "none", "--no-tracing",
                   "-Dhystrix.command.default.circuitBreaker.enabled=false"], threads=2)
    for _ in range(4):
        chain(s)
    aloha.set_mode("slow", delay_s=1.0)
    for _ in range(2):  # both end at the 600 ms Hystrix timeout
        assert chain(s)[1:] == [FALLBACK]
    # a call is recorded on its worker as it finishes, which can be just after its answer
    # left: the scrape (on any worker) sees it within moments
    deadline = time.monotonic() + 3
    while True:
        _, _, body = s.get("/metrics")
        b, total, count = _histogram(body, "hola_chaining_duration_seconds")
        if count == 6 or time.monotonic() > deadline:
            break
        time.sleep(0.02)
    les = list(b)
    assert les[-1] == "+Inf" and count == 6 and b["+Inf"] == 6
    assert all(b[x] <= b[y] for x, y in zip(les, les[1:]))  # cumulative
    assert b["0.5"] == 4 and b["1"] == 6  # the timed-out calls sit between 0.5 s and 1 s
    assert 1.2 <= total < 2.5


def test_format_error_skips_downstream_call(hola, aloha, tmp_path):
    conf = tmp_path / "t.properties"
    conf.write_text("hello=%d\n")
    s = hola(args=["--aloha-url", aloha.url, f"-Dconf={conf}"])
    st, _, _ = s.get("/api/hola-chaining")
    assert st == 500
    assert aloha.requests == []


def test_feign_basic_logging(hola, aloha):
    """Feign Logger.ErrorLogger at BASIC (HolaResource.java:109): raw stderr lines tagged with
    the config key cut at '(' (Logger.methodTag), the reason phrase and the elapsed ms."""
    s = hola(args=["--aloha-url", aloha.url])
    chain(s)
    log = _wait_log(s, "<--- HTTP/1.1", 1)
    lines = [l for l in log.splitlines() if l.startswith("[AlohaService#aloha] ")]
    assert lines[0] == f"[AlohaService#aloha] ---> GET {aloha.url.rstrip('/')}/api/aloha-chaining HTTP/1.1"
    assert re.fullmatch(r"\[AlohaService#aloha\] <--- HTTP/1\.1 200 OK \(\d+ms\)", lines[1]), lines[1]


def test_hystrix_command_key_default_and_flag(hola, aloha):
    """feign-hystrix 8.15.1 keys the command by the method name ("aloha"); the group and pool
    are the target URL. --hystrix-command-key configkey gives the 9.x SetterFactory.Default
    key; per-command properties follow the key."""
    aloha.set_mode("slow", delay_s=1.0)
    s = hola(args=["--aloha-url", aloha.url, "--feign-log", "none",
                   "-Dhystrix.command.aloha.execution.isolation.thread.timeoutInMilliseconds=150"])
    t0 = time.monotonic()
    assert chain(s)[1:] == [FALLBACK]
    assert time.monotonic() - t0 < 0.5
    _, _, body = s.get("/metrics")
    assert b'hola_hystrix_events_total{command="aloha",event="TIMEOUT"} 1' in body
    s2 = hola(args=["--aloha-url", aloha.url, "--feign-log", "none", "--hystrix-command-key", "configkey",
                    "-Dhystrix.command.AlohaService#aloha().execution.isolation.thread.timeoutInMilliseconds=150"])
    t0 = time.monotonic()
    assert chain(s2)[1:] == [FALLBACK]
    assert time.monotonic() - t0 < 0.5
    _, _, body = s2.get("/metrics")
    assert b'command="AlohaService#aloha()",event="TIMEOUT"} 1' in body


def test_hystrix_command_key_beats_default_for_timeout(hola, aloha):
    """Archaius precedence: hystrix.command.<key>.* wins over hystrix.command.default.* for the
    same property, and the timeout is read from execution.isolation.thread.timeoutInMilliseconds
    only (Hystrix 1.5.1 has no execution.timeout.timeoutInMilliseconds; config.properties:17)."""
    aloha.set_mode("slow", delay_s=3.0)
    s = hola(args=["--aloha-url", aloha.url, "--feign-log", "none",
                   "-Dhystrix.command.default.execution.isolation.thread.timeoutInMilliseconds=100",
                   "-Dhystrix.command.default.execution.timeout.timeoutInMilliseconds=100",
                   "-Dhystrix.command.aloha.execution.isolation.thread.timeoutInMilliseconds=900"])
    t0 = time.monotonic()
    assert chain(s)[1:] == [FALLBACK]
    dt = time.monotonic() - t0
    assert 0.85 <= dt < 1.6, dt
    _, _, body = s.get("/metrics")
    assert b'hola_hystrix_events_total{command="aloha",event="TIMEOUT"} 1' in body


def test_hystrix_invented_timeout_key_is_ignored(hola, aloha):
    """execution.timeout.timeoutInMilliseconds is not a Hystrix key: setting it alone leaves the
    600 ms default (config.properties:17) in force."""
    aloha.set_mode("slow", delay_s=3.0)
    s = hola(args=["--aloha-url", aloha.url, "--feign-log", "none",
                   "-Dhystrix.command.default.execution.timeout.timeoutInMilliseconds=100"])
    t0 = time.monotonic()
    assert chain(s)[1:] == [FALLBACK]
    assert 0.55 <= time.monotonic() - t0 < 1.4


def test_hystrix_flag_shorthands(hola, aloha):
    aloha.set_mode("slow", delay_s=1.0)
    s = hola(args=["--aloha-url", aloha.url, "--hystrix-timeout-ms", "120", "--feign-log", "none"])
    t0 = time.monotonic()
    assert chain(s)[1:] == [FALLBACK]
    assert time.monotonic() - t0 < 0.6


def test_success_response_framing_get_and_head(hola, aloha):
    """The success response is assembled in one buffer: headers in the same order as every
    prepared response, Content-Length matching the body, and HEAD keeping the length."""
    aloha.payload = ["Aloha \"quoted\"", None, "tab\there"]
    s = hola(args=["--aloha-url", aloha.url, "--feign-log", "none"], env={"HOSTNAME": "h"})

    def raw(method):
        with socket.create_connection(("127.0.0.1", s.port), timeout=5) as c:
            c.sendall(f"{method} /api/hola-chaining HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n".encode())
            data = b""
            while chunk := c.recv(65536):
                data += chunk
        head, _, body = data.partition(b"\r\n\r\n")
        return head.decode().split("\r\n"), body

    lines, body = raw("GET")
    assert lines[0] == "HTTP/1.1 200 OK"
    names = [l.split(":")[0] for l in lines[1:]]
    assert names == ["Connection", "Access-Control-Allow-Origin", "Content-Type", "Content-Length", "Date"]
    assert json.loads(body) == ["Hola de h", "Aloha \"quoted\"", None, "tab\there"]
    length = int(dict(l.split(": ", 1) for l in lines[1:])["Content-Length"])
    assert length == len(body)
    hlines, hbody = raw("HEAD")
    assert hbody == b"" and dict(l.split(": ", 1) for l in hlines[1:])["Content-Length"] == str(length)


def test_shortened_timeout_does_not_wait_behind_older_calls(hola, aloha, tmp_path):
    """Timeouts are kept per worker in deadline order. A call started after the timeout was
    shortened (config reload) must time out on its own deadline, even while an older call with
    the longer deadline is still in flight on the same worker."""
    hc = tmp_path / "config.properties"
    key = "hystrix.command.default.execution.isolation.thread.timeoutInMilliseconds"
    hc.write_text(f"{key}=3000\n")
    aloha.set_mode("slow", delay_s=1.5)
    s = hola(args=["--aloha-url", aloha.url, "--hystrix-config", str(hc), "--feign-log", "none"], threads=1)

    def reloads():
        m = s.get("/metrics")[2].decode()
        return int(next(l for l in m.splitlines() if l.startswith("hola_config_reloads_total ")).split()[1])

    first = []
    t = threading.Thread(target=lambda: first.append(chain(s)))
    t.start()
    time.sleep(0.2)  # the first call is in flight with a 3000 ms deadline
    before = reloads()
    hc.write_text(f"{key}=150\n")
    deadline = time.monotonic() + 3
    while reloads() == before and time.monotonic() < deadline:
        time.sleep(0.02)
    t0 = time.monotonic()
    assert chain(s)[1:] == [FALLBACK]
    assert time.monotonic() - t0 < 0.8  # its own 150 ms deadline, not the older 3000 ms one
    t.join()
    assert first and first[0][1:] != [FALLBACK]  # the older call still completed normally


def test_retry_sleeps_hold_the_bulkhead_slot(hola):
    """Feign's retry sleeps run on the Hystrix thread, so a retrying call keeps its bulkhead
    slot until the timeout: with coreSize=1, a second concurrent call is rejected."""
    s = hola(args=["--aloha-url", f"http://127.0.0.1:{closed_port()}/", "--feign-log", "none",
                   "-Dhystrix.threadpool.default.coreSize=1",
                   "-Dhystrix.command.default.circuitBreaker.enabled=false"], threads=1)
    first = []
    t = threading.Thread(target=lambda: first.append(chain(s)))
    t.start()
    time.sleep(0.2)  # the first call is sleeping between Feign attempts
    t0 = time.monotonic()
    assert chain(s)[1:] == [FALLBACK]
    assert time.monotonic() - t0 < 0.3  # rejected at once, not retried
    t.join()
    assert first and first[0][1:] == [FALLBACK]
    ev = _events(s)
    assert ev.get("THREAD_POOL_REJECTED") == 1 and ev.get("TIMEOUT") == 1


@pytest.mark.parametrize("mode", ["empty", "json_null", "no_content"])
def test_list_decoding_to_null_is_a_500(hola, aloha, mode):
    """feign-jackson's JacksonDecoder returns null for an empty body, and Jackson maps JSON
    null to null: the Hystrix command succeeds, then greetings.addAll(null) throws in
    holaChaining() (HolaResource.java:76), which the container answers with a 500."""
    aloha.set_mode(mode)
    s = hola(args=["--aloha-url", aloha.url, "--feign-log", "none"])
    st, h, _ = s.get("/api/hola-chaining", timeout=10)
    assert st == 500 and "access-control-allow-origin" not in h
    assert _events(s).get("SUCCESS") == 1 and len(aloha.requests) == 1


def test_close_delimited_aloha_body(hola, aloha):
    aloha.set_mode("close_delimited")
    s = hola(args=["--aloha-url", aloha.url, "--feign-log", "none"], env={"HOSTNAME": "h"})
    for _ in range(3):  # a fresh connection each time
        assert chain(s) == ["Hola de h", "Aloha mai aloha-1", "Bonjour de bonjour-1"]


def test_idle_connection_closed_by_aloha_is_dropped(hola, aloha):
    """aloha closes a kept-alive connection while it sits idle in the pool: the pool drops it
    when the close arrives (or, if the next call races it, re-sends on a fresh connection)."""
    aloha.set_mode("drop_idle")
    s = hola(args=["--aloha-url", aloha.url, "--feign-log", "none"], env={"HOSTNAME": "h"}, threads=1)
    for _ in range(5):
        assert chain(s)[1:] == ["Aloha mai aloha-1", "Bonjour de bonjour-1"]
        time.sleep(0.05)
    assert _events(s).get("SUCCESS") == 5


@pytest.mark.parametrize("epoll", ["et", "lt"])
def test_input_arriving_while_a_request_is_parked(hola, aloha, epoll):
    """A parked /api/hola-chaining keeps its connection's input registered (edge-triggered)
    or not (level-triggered). Either way, requests pipelined behind it, requests sent while
    it waits, and a FIN sent while it waits are all handled, in order, once it completes."""
    aloha.set_mode("slow", delay_s=0.2)
    args = ["--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none"] + (["--epoll-lt"] if epoll == "lt" else [])
    s = hola(args=args, env={"HOSTNAME": "h"}, threads=1)
    chain_req = b"GET /api/hola-chaining HTTP/1.1\r\nHost: x\r\n\r\n"
    hola_req = b"GET /api/hola HTTP/1.1\r\nHost: x\r\n\r\n"

    def read_until_closed(c):
        out = b""
        c.settimeout(5)
        while True:
            b = c.recv(65536)
            if not b:
                return out
            out += b

    # 1) pipelined behind the parked request, in one write
    with socket.create_connection(("127.0.0.1", s.port)) as c:
        c.sendall(chain_req + hola_req + chain_req.replace(b"\r\n\r\n", b"\r\nConnection: close\r\n\r\n"))
        out = read_until_closed(c)
    assert out.count(b"HTTP/1.1 200 OK") == 3
    first, mid, last = out.find(b"Aloha mai"), out.find(b"\r\n\r\nHola de h"), out.rfind(b"Aloha mai")
    assert 0 < first < mid < last, out
    # 2) a second request and then a FIN, both sent while the first is parked
    with socket.create_connection(("127.0.0.1", s.port)) as c:
        c.sendall(chain_req)
        time.sleep(0.05)
        c.sendall(hola_req)
        time.sleep(0.05)
        c.shutdown(socket.SHUT_WR)
        out = read_until_closed(c)
    assert out.count(b"HTTP/1.1 200 OK") == 2
    assert 0 < out.find(b"Aloha mai") < out.rfind(b"Hola de h"), out


def _concurrent_chains(s, n):
    out = [None] * n

    def one(i):
        st, _, body = s.get("/api/hola-chaining", timeout=10)
        out[i] = (st, json.loads(body))

    ts = [threading.Thread(target=one, args=(i,)) for i in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return out


def test_pipelined_aloha_calls_share_connections(hola, aloha):
    """--aloha-pipeline N: concurrent aloha calls of a worker go out over shared kept-alive
    connections, several requests per connection in flight, and every call still gets its
    own answer in order."""
    s = hola(args=["--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none", "--aloha-pipeline", "8",
                   "-Dhystrix.threadpool.default.coreSize=64"], env={"HOSTNAME": "h"}, threads=1)
    for _ in range(3):
        res = _concurrent_chains(s, 24)
        assert all(st == 200 and body == ["Hola de h", "Aloha mai aloha-1", "Bonjour de bonjour-1"]
                   for st, body in res), res
    peers = {r["peer_port"] for r in aloha.requests}
    assert len(aloha.requests) == 72
    assert len(peers) < 24, peers  # fewer connections than concurrent calls
    m = s.get("/metrics")[2]
    assert b'event="SUCCESS"} 72' in m


@pytest.mark.parametrize("mode,expect_fallback", [("close", True), ("slow", True), ("error", True)])
def test_pipelined_failures(hola, aloha, mode, expect_fallback):
    """A dropped connection, a timeout and an error status on a pipelined connection: each
    call falls back on its own, and the next calls succeed on fresh connections."""
    aloha.set_mode(mode, delay_s=1.0)
    s = hola(args=["--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none", "--aloha-pipeline", "4",
                   "--feign-retry", "off", "-Dhystrix.threadpool.default.coreSize=64",
                   "-Dhystrix.command.default.circuitBreaker.enabled=false"], env={"HOSTNAME": "h"}, threads=1)
    t0 = time.monotonic()
    res = _concurrent_chains(s, 8)
    assert all(st == 200 and body == ["Hola de h", FALLBACK] for st, body in res), res
    assert time.monotonic() - t0 < 3.0
    aloha.set_mode("ok")
    res = _concurrent_chains(s, 8)
    assert all(st == 200 and body[1] == "Aloha mai aloha-1" for st, body in res), res


def test_pipelined_read_timeouts_do_not_pile_up(hola, aloha):
    """Pipelined calls with the Hystrix timeout disabled are guarded by Feign's read timeout
    (one FIFO of deadlines, one loop timer): answered calls leave the FIFO, and the pending
    loop timers do not grow with the call count."""
    s = hola(args=["--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none", "--aloha-pipeline", "4",
                   "-Dhystrix.command.default.execution.timeout.enabled=false",
                   "-Dhystrix.threadpool.default.coreSize=64"], threads=1)
    idle = _metric(s, "hola_event_loop_timers")
    for _ in range(10):
        assert all(st == 200 for st, _ in _concurrent_chains(s, 8))
    assert _metric(s, "hola_event_loop_timers") <= idle + 4


def test_pipelined_connection_is_not_reused_after_a_timeout(hola, aloha):
    """A call that times out on a pipelined connection gives the connection up: calls made
    afterwards do not queue behind the answer that never came."""
    s = hola(args=["--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none", "--aloha-pipeline", "8",
                   "--feign-retry", "off", "-Dhystrix.command.default.circuitBreaker.enabled=false"],
             env={"HOSTNAME": "h"}, threads=1)
    assert chain(s)[1] == "Aloha mai aloha-1"
    aloha.set_mode("slow", delay_s=5.0)
    assert chain(s)[1] == FALLBACK  # 600 ms
    aloha.set_mode("ok")
    t0 = time.monotonic()
    assert chain(s)[1] == "Aloha mai aloha-1"
    assert time.monotonic() - t0 < 0.5


def test_pipelined_mode_keeps_no_idle_plain_connections(hola, aloha):
    """Calls re-sent after a pipelined connection is given up run on plain connections; with
    pipelining on nothing would reuse those afterwards, so they are closed, not pooled."""
    import os
    s = hola(args=["--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none", "--aloha-pipeline", "4",
                   "--feign-retry", "off", "-Dhystrix.threadpool.default.coreSize=64",
                   "-Dhystrix.command.default.circuitBreaker.enabled=false"], threads=1)
    fds = lambda: len(os.listdir(f"/proc/{s.proc.pid}/fd"))  # noqa: E731
    _concurrent_chains(s, 8)
    base = fds()
    for _ in range(4):
        # one slow answer at the head of a pipelined connection: its call times out, the calls
        # queued behind it wait for their answers or their own timeouts (not re-sent), and the
        # connection closes once none of them is waited for
        aloha.set_mode("slow", delay_s=0.8)
        threading.Thread(target=lambda: s.get("/api/hola-chaining", timeout=10), daemon=True).start()
        time.sleep(0.05)
        aloha.set_mode("ok")
        _concurrent_chains(s, 8)
        time.sleep(0.8)
    assert fds() <= base + 4, (base, fds())


def test_uniformly_slow_aloha_gets_bounded_head_of_line_resends(hola, aloha):
    """aloha uniformly slower than the Hystrix timeout with --aloha-pipeline 8. A call
    is abandoned at its timeout; calls queued behind it on its pipelined connection with later
    deadlines would all be re-sent 50 ms later, second GETs to a downstream still working on
    the first, growing the load as it slows. The re-sends draw on a budget of 0.1 per call
    (burst 10): the requests reaching aloha stay near one per call."""
    aloha.set_mode("slow", delay_s=0.3)
    s = hola(args=["--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none", "--aloha-pipeline", "8",
                   "--feign-retry", "off", "--hystrix-timeout-ms", "200", "-Dhystrix.threadpool.default.coreSize=64",
                   "-Dhystrix.command.default.circuitBreaker.enabled=false"], env={"HOSTNAME": "h"}, threads=1)
    calls = 0
    for _ in range(12):
        # one call, then 7 more 70 ms later on the same pipelined connection: their deadlines
        # fall after the head's timeout plus the 50 ms grace, while its answer is still due
        head = threading.Thread(target=lambda: s.get("/api/hola-chaining", timeout=10))
        head.start()
        time.sleep(0.07)
        res = _concurrent_chains(s, 7)
        head.join()
        assert all(st == 200 and body == ["Hola de h", FALLBACK] for st, body in res), res
        calls += 8
    time.sleep(0.5)  # re-sends still in flight land in aloha's count
    resent = _retries(s).get("transport", 0)
    assert resent <= 10 + 0.1 * calls + 7, (resent, calls)
    assert len(aloha.requests) <= calls + 10 + 0.1 * calls + 7, (len(aloha.requests), calls)


def _retries(s) -> dict:
    out = {}
    for line in s.get("/metrics")[2].decode().splitlines():
        if line.startswith("hola_aloha_retries_total{"):
            out[line.split('kind="')[1].split('"')[0]] = int(float(line.rsplit(" ", 1)[1]))
    return out


_PIPE = ["--aloha-pipeline", "4", "-Dhystrix.threadpool.default.coreSize=64"]


@pytest.mark.parametrize("pipelined", [False, True], ids=["plain", "pipelined"])
def test_malformed_framing_after_a_valid_head_fails_once(hola, aloha, pipelined):
    """A valid 200 head followed by a malformed chunk: HttpClient never re-sends it (a protocol
    error after the response) and Feign does not retry it (the failure is in the body, after
    execute() returned). Both client modes: one aloha request, one FAILURE, no transport
    retry."""
    aloha.set_mode("bad_chunk")
    s = hola(args=["--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none"] + (_PIPE if pipelined else []),
             threads=1)
    t0 = time.monotonic()
    assert chain(s)[1:] == [FALLBACK]
    assert time.monotonic() - t0 < 0.3
    assert len(aloha.requests) == 1
    assert _events(s).get("FAILURE") == 1
    assert _retries(s).get("transport", 0) == 0


@pytest.mark.parametrize("pipelined", [False, True], ids=["plain", "pipelined"])
def test_malformed_status_line_is_not_resent_by_the_transport(hola, aloha, pipelined):
    """No parseable status line: ClientProtocolException from execute() is an IOException, so
    Feign's Retryer may retry the call, but the transport never re-sends it. With Feign retries
    off: one request, one FAILURE. With the default Retryer: every aloha request is a Feign
    attempt (transport retries stay 0) until the 600 ms Hystrix timeout."""
    aloha.set_mode("bad_status")
    base = ["--aloha-url", aloha.url, "--no-tracing"] + (_PIPE if pipelined else [])
    s = hola(args=base + ["--feign-log", "none", "--feign-retry", "off"], threads=1)
    assert chain(s)[1:] == [FALLBACK]
    assert len(aloha.requests) == 1
    assert _events(s).get("FAILURE") == 1
    assert _retries(s).get("transport", 0) == 0
    s2 = hola(args=base, threads=1)
    n0 = len(aloha.requests)
    assert chain(s2)[1:] == [FALLBACK]
    assert _events(s2).get("TIMEOUT") == 1
    r = _retries(s2)
    assert r.get("transport", 0) == 0
    assert r.get("feign", 0) >= 2
    assert len(aloha.requests) - n0 == r["feign"] + 1
    assert "<--- ERROR ClientProtocolException: malformed response" in _wait_log(s2, "ClientProtocolException", 1)


def test_pipelined_timeout_does_not_resend_the_calls_behind_it(hola, aloha):
    """A call abandoned on its Hystrix timeout no longer makes the client re-send the calls
    pipelined behind it, which aloha already has (that doubled aloha's load exactly when it was
    slow). Aloha sees each call once, no transport retry is spent, the connection is closed once
    every call on it is given up, and the next calls run on a fresh one."""
    import os
    aloha.set_mode("slow", delay_s=1.0)
    s = hola(args=["--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none", "--feign-retry", "off",
                   "-Dhystrix.command.default.circuitBreaker.enabled=false"] + _PIPE, threads=1)
    fds = lambda: len(os.listdir(f"/proc/{s.proc.pid}/fd"))  # noqa: E731
    base = fds()
    res = _concurrent_chains(s, 4)
    assert all(st == 200 and body[1:] == [FALLBACK] for st, body in res), res
    assert _events(s).get("TIMEOUT") == 4
    time.sleep(0.3)
    # the fake answers a connection's requests one at a time, so it has read only the first
    # by now; what matters is that nothing arrived on any other connection (a re-send)
    assert 1 <= len(aloha.requests) <= 4
    assert len({r["peer_port"] for r in aloha.requests}) == 1, aloha.requests
    assert _retries(s).get("transport", 0) == 0
    deadline = time.monotonic() + 2.0  # (the test client's own connections close asynchronously)
    while fds() > base and time.monotonic() < deadline:
        time.sleep(0.02)
    assert fds() <= base, (base, fds())  # given up once all four were abandoned
    aloha.set_mode("ok")
    assert chain(s)[1] == "Aloha mai aloha-1"
    assert len({r["peer_port"] for r in aloha.requests}) == 2


@pytest.mark.parametrize("pipelined", [False, True], ids=["plain", "pipelined"])
def test_refused_aloha_costs_no_transport_retry(hola, pipelined):
    """A refused connect is HttpHostConnectException: HttpClient's retry handler never re-sends
    it, in either client mode (before this fix a pipelined connection re-sent every call queued
    on it, one more connect each)."""
    s = hola(args=["--aloha-url", f"http://127.0.0.1:{closed_port()}/", "--no-tracing", "--feign-log", "none",
                   "--feign-retry", "off", "-Dhystrix.command.default.circuitBreaker.enabled=false"]
             + (_PIPE if pipelined else []), threads=1)
    res = _concurrent_chains(s, 6)
    assert all(st == 200 and body[1:] == [FALLBACK] for st, body in res), res
    assert _retries(s).get("transport", 0) == 0
    assert _events(s).get("FAILURE") == 6


def test_read_timeout_runs_after_a_slow_connect(hola):
    """Feign's read timeout is armed once the connect completes: a connect that takes longer
    than the read timeout (its SYN dropped by a full accept queue and retransmitted ~1 s later)
    followed by a server that never answers still ends with SocketTimeoutException, instead of
    the deadline expiring unused while the connect was pending and the call hanging."""
    lsock = socket.socket()
    lsock.bind(("127.0.0.1", 0))
    lsock.listen(0)  # one pending connection fills the accept queue
    port = lsock.getsockname()[1]
    filler = socket.create_connection(("127.0.0.1", port))
    filler2 = socket.socket()
    filler2.setblocking(False)
    filler2.connect_ex(("127.0.0.1", port))
    accepted = []

    def drain_later():
        time.sleep(0.5)  # after hola's SYN was dropped: make room for its retransmission
        deadline = time.monotonic() + 5
        lsock.settimeout(0.2)
        while time.monotonic() < deadline:
            try:
                accepted.append(lsock.accept()[0])  # accepted, never answered
            except OSError:
                pass

    s = hola(args=["--aloha-url", f"http://127.0.0.1:{port}/", "--no-tracing", "--feign-log", "basic",
                   "--feign-retry", "off", "--feign-timeouts", "5000,300",
                   "-Dhystrix.command.default.execution.timeout.enabled=false"], threads=1)
    t = threading.Thread(target=drain_later, daemon=True)
    t.start()
    t0 = time.monotonic()
    assert chain(s)[1:] == [FALLBACK]
    dt = time.monotonic() - t0
    assert dt < 4.5, dt
    assert "<--- ERROR SocketTimeoutException: Read timed out" in _wait_log(s, "SocketTimeoutException", 1)
    t.join()
    for c in accepted + [filler, filler2, lsock]:
        c.close()


def test_pipelined_calls_behind_a_slow_answer_are_not_held_to_their_timeouts(hola, aloha):
    """One slow aloha answer, then fast ones, on a shared pipelined connection: the
    slow call times out on its own 600 ms Hystrix deadline, and the calls queued behind it are
    re-sent on fresh connections shortly after (kDrainGraceMs) instead of waiting for the slow
    answer until their own deadlines: they succeed, no extra TIMEOUT reaches the breaker."""
    aloha.set_mode("slow_once", delay_s=3.0)
    s = hola(args=["--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none", "--feign-retry", "off",
                   "-Dhystrix.command.default.circuitBreaker.enabled=false"] + _PIPE, env={"HOSTNAME": "h"},
             threads=1)
    slow = {}
    t = threading.Thread(target=lambda: slow.update(r=chain(s)), daemon=True)
    t.start()
    time.sleep(0.3)  # the slow call is on the connection; the next calls queue behind it
    t0 = time.monotonic()
    res = _concurrent_chains(s, 3)
    took = time.monotonic() - t0
    t.join(timeout=5)
    assert slow["r"][1:] == [FALLBACK]
    assert all(st == 200 and body[1] == "Aloha mai aloha-1" for st, body in res), res
    assert took < 1.5, took  # re-sent ~50 ms after the slow call was abandoned (at ~0.3 s from t0)
    ev = _events(s)
    assert ev.get("TIMEOUT") == 1 and ev.get("SUCCESS") == 3, ev
    assert _retries(s).get("transport", 0) == 3  # each queued call went out once more


@pytest.mark.parametrize("compact", [False, True])
def test_a_call_parked_across_a_reload_answers_with_its_own_greeting(hola, aloha, tmp_path, compact):
    """The greeting is computed when the request arrives (HolaResource.java:75): a chaining
    call still waiting on aloha while the greeting file changes answers with the greeting of
    its own request, and the next request gets the new one. (The worker keeps the contents of
    the last configuration generations for such calls; the call holds its generation.)"""
    conf = tmp_path / "t.properties"
    conf.write_text("hello=old %s\n")
    aloha.compact = compact  # a list passed on as text, or decoded (json::plain_string_list)
    aloha.set_mode("slow_once", delay_s=2.0)
    s = hola(args=[f"-Dconf={conf}", "--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none",
                   "--config-poll-ms", "100", "-Dhystrix.command.default.execution.isolation.thread.timeoutInMilliseconds=5000"],
             env={"HOSTNAME": "h"}, threads=1)
    parked = {}
    t = threading.Thread(target=lambda: parked.update(r=chain(s)), daemon=True)
    t.start()
    time.sleep(0.3)  # the call is parked on aloha now
    conf.write_text("hello=new %s\n")
    deadline = time.monotonic() + 5
    while s.get("/api/hola")[2] != b"new h" and time.monotonic() < deadline:
        time.sleep(0.05)
    assert s.get("/api/hola")[2] == b"new h"
    t.join(timeout=10)
    assert parked["r"] == ["old h", "Aloha mai aloha-1", "Bonjour de bonjour-1"], parked
    assert chain(s) == ["new h", "Aloha mai aloha-1", "Bonjour de bonjour-1"]


def test_a_call_parked_across_many_reloads_answers_with_the_current_greeting(hola, aloha, tmp_path):
    """past the 8 kept generations a parked call's own content is gone; it answers
    with the current greeting (it names its content by generation, so a new content that
    reuses a freed one's address cannot pass for it)."""
    conf = tmp_path / "t.properties"
    conf.write_text("hello=g0 %s\n")
    aloha.set_mode("slow_once", delay_s=4.0)
    s = hola(args=[f"-Dconf={conf}", "--aloha-url", aloha.url, "--no-tracing", "--feign-log", "none",
                   "--config-poll-ms", "50", "-Dhystrix.command.default.execution.isolation.thread.timeoutInMilliseconds=9000"],
             env={"HOSTNAME": "h"}, threads=1)
    parked = {}
    t = threading.Thread(target=lambda: parked.update(r=chain(s)), daemon=True)
    t.start()
    time.sleep(0.3)
    for k in range(1, 11):  # ten reloads, each seen by the worker before the next
        conf.write_text(f"hello=g{k} %s\n")
        deadline = time.monotonic() + 3
        while s.get("/api/hola")[2] != f"g{k} h".encode() and time.monotonic() < deadline:
            time.sleep(0.02)
        assert s.get("/api/hola")[2] == f"g{k} h".encode()
    t.join(timeout=15)
    assert parked["r"] == ["g10 h", "Aloha mai aloha-1", "Bonjour de bonjour-1"], parked
