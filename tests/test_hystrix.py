"""Hystrix 1.5.1 circuit-breaker state machine on a fake clock (native Command), the
properties that tune it (config.properties:16-19) and /hystrix.stream (HystrixServlet.java)."""
import json
import os
import socket
import time

import pytest

from hola_amd.testing.fakes import FakeAloha

TUNED = {
    "hystrix.command.default.execution.isolation.thread.timeoutInMilliseconds": "600",
    "hystrix.command.default.circuitBreaker.requestVolumeThreshold": "5",
}


def fail_n(cmd, n, outcome="failure"):
    for _ in range(n):
        assert cmd.try_start() == "run"
        cmd.finish(outcome, 3)


def test_settings_resolution(native):
    c = native.HystrixCommand(TUNED)
    s = c.settings()
    assert s["timeout_ms"] == 600 and s["request_volume_threshold"] == 5
    assert s["error_threshold_pct"] == 50 and s["sleep_window_ms"] == 5000  # [lib-default]
    assert s["pool_core_size"] == 10 and s["rolling_window_ms"] == 10000
    # command-specific keys beat the defaults
    c = native.HystrixCommand({**TUNED, "hystrix.command.AlohaService#aloha().circuitBreaker.requestVolumeThreshold": "7",
                               "hystrix.threadpool.aloha.coreSize": "3"})
    assert c.settings()["request_volume_threshold"] == 7 and c.settings()["pool_core_size"] == 3


def test_below_volume_threshold_stays_closed(native):
    c = native.HystrixCommand(TUNED)
    fail_n(c, 4)
    c.advance(600)
    assert not c.is_open()
    assert c.try_start() == "run"


def test_trips_at_threshold_and_error_percentage(native):
    c = native.HystrixCommand(TUNED)
    fail_n(c, 5)
    c.advance(600)  # health snapshot interval (500 ms)
    assert c.is_open()
    assert c.try_start() == "short_circuited"
    h = c.health()
    assert h["total"] == 5 and h["errors"] == 5 and h["error_pct"] == 100


def test_error_percentage_below_50_stays_closed(native):
    c = native.HystrixCommand(TUNED)
    fail_n(c, 4)
    fail_n(c, 6, "success")
    c.advance(600)
    assert not c.is_open()
    assert c.health()["error_pct"] == 40


def test_timeouts_count_as_errors(native):
    c = native.HystrixCommand(TUNED)
    fail_n(c, 5, "timeout")
    c.advance(600)
    assert c.is_open()


def test_single_trial_after_sleep_window(native):
    c = native.HystrixCommand(TUNED)
    fail_n(c, 5)
    c.advance(600)
    assert c.try_start() == "short_circuited"
    c.advance(5000)
    assert c.try_start() == "short_circuited"   # sleepWindow must be strictly exceeded
    c.advance(1)
    assert c.try_start() == "run"               # the single test request
    assert c.try_start() == "short_circuited"   # only one per window
    c.finish("failure", 1)                      # trial fails: stays open
    c.advance(100)
    assert c.try_start() == "short_circuited"
    c.advance(5001)
    assert c.try_start() == "run"
    c.finish("success", 1)                      # trial succeeds: closes and resets
    assert not c.is_open()
    assert c.health()["total"] == 0  # markSuccess() resets the health stream
    assert c.try_start() == "run"


def test_a_call_running_when_the_circuit_opens_closes_it(native):
    """Hystrix 1.5.1's markSuccess closes an open circuit on any success, so a call admitted
    before the trip that then succeeds closes it before the sleep window; /metrics counts the
    two kinds of close apart (hola_hystrix_circuit_transitions_total)."""
    c = native.HystrixCommand(TUNED)
    assert c.try_start() == "run"  # admitted while closed, still running
    fail_n(c, 5)
    c.advance(600)
    assert c.is_open() and c.try_start() == "short_circuited"
    c.finish("success", 1)  # the running call completes
    assert not c.is_open() and c.health()["total"] == 0
    assert c.transitions() == {"opened": 1, "closed_trial": 0, "closed_inflight": 1}
    fail_n(c, 5)
    c.advance(600)
    assert c.is_open()
    c.advance(5001)
    assert c.try_start() == "run"  # the sleep window's trial
    c.finish("success", 1)
    assert c.transitions() == {"opened": 2, "closed_trial": 1, "closed_inflight": 1}


def test_rolling_window_expires_old_failures(native):
    c = native.HystrixCommand(TUNED)
    fail_n(c, 4)
    c.advance(10_500)  # older than the 10 s window
    fail_n(c, 1)
    c.advance(600)
    assert not c.is_open()


def test_bulkhead(native):
    c = native.HystrixCommand({**TUNED, "hystrix.threadpool.default.coreSize": "2"})
    assert c.try_start() == "run" and c.try_start() == "run"
    assert c.try_start() == "rejected"
    c.finish("success", 1)
    assert c.try_start() == "run"


QUEUE = {**TUNED, "hystrix.threadpool.default.coreSize": "1", "hystrix.threadpool.default.maxQueueSize": "3",
         "hystrix.threadpool.default.queueSizeRejectionThreshold": "2"}


def test_pool_queue_admission_and_fifo(native):
    """maxQueueSize > 0: beyond coreSize, calls wait in a FIFO holding fewer than
    min(maxQueueSize, queueSizeRejectionThreshold); a released slot goes to the oldest."""
    c = native.HystrixCommand(QUEUE)
    assert [c.try_start(t) for t in range(5)] == ["run", "queued", "queued", "rejected", "rejected"]
    assert c.queue_size() == 2
    assert c.next_queued() is None          # no slot free yet
    c.finish("success", 1)
    assert c.next_queued() == 1             # oldest first, and it holds the slot now
    assert c.next_queued() is None
    assert c.try_start(7) == "queued"       # room again behind ticket 2
    c.finish("success", 1)
    assert c.next_queued() == 2
    c.finish("success", 1)
    assert c.next_queued() == 7
    pool = json.loads(c.pool_json())
    assert pool["currentQueueSize"] == 0 and pool["currentActiveCount"] == 1
    assert pool["rollingCountThreadsExecuted"] == 4 and pool["rollingCountCommandRejections"] == 2


def test_pool_queue_threshold_and_default(native):
    # the smaller of maxQueueSize and the rejection threshold bounds the queue
    c = native.HystrixCommand({**QUEUE, "hystrix.threadpool.default.maxQueueSize": "1",
                               "hystrix.threadpool.default.queueSizeRejectionThreshold": "5"})
    assert [c.try_start(t) for t in range(3)] == ["run", "queued", "rejected"]
    # default maxQueueSize -1 (SynchronousQueue): never queued, even when offered
    c = native.HystrixCommand({**TUNED, "hystrix.threadpool.default.coreSize": "1"})
    assert [c.try_start(t) for t in range(2)] == ["run", "rejected"] and c.queue_size() == 0


def test_pool_queue_timeout_and_cancel(native):
    """A queued call that times out leaves the queue and counts as a TIMEOUT (an error for
    the breaker); a call popped after its timeout hands its slot back."""
    c = native.HystrixCommand(QUEUE)
    assert [c.try_start(t) for t in range(3)] == ["run", "queued", "queued"]
    assert c.cancel_queued(1) and not c.cancel_queued(1)
    c.queued_timeout(600)
    assert c.queue_size() == 1
    c.finish("success", 1)
    assert c.next_queued() == 2
    c.release_slot()                         # ticket 2 timed out meanwhile: slot handed back
    assert c.try_start(9) == "run"
    cmd = json.loads(c.stream_json())
    assert cmd["rollingCountTimeout"] == 1 and cmd["rollingCountFallbackSuccess"] == 1
    c.advance(600)
    assert c.health()["errors"] == 1


def test_force_open_and_closed(native):
    c = native.HystrixCommand({"hystrix.command.default.circuitBreaker.forceOpen": "true"})
    assert c.try_start() == "short_circuited"
    c = native.HystrixCommand({**TUNED, "hystrix.command.default.circuitBreaker.forceClosed": "true"})
    fail_n(c, 10)
    c.advance(600)
    assert c.try_start() == "run"


def test_stream_json_schema(native):
    c = native.HystrixCommand(TUNED)
    fail_n(c, 2)
    fail_n(c, 3, "success")
    d = json.loads(c.stream_json())
    assert d["type"] == "HystrixCommand" and d["name"] == "AlohaService#aloha()"
    for k in ("errorPercentage", "errorCount", "requestCount", "rollingCountSuccess", "rollingCountFailure",
              "rollingCountTimeout", "rollingCountShortCircuited", "rollingCountThreadPoolRejected",
              "rollingCountFallbackSuccess", "isCircuitBreakerOpen", "latencyExecute", "latencyTotal",
              "latencyExecute_mean", "propertyValue_circuitBreakerRequestVolumeThreshold",
              "propertyValue_executionIsolationThreadTimeoutInMilliseconds", "reportingHosts", "currentTime"):
        assert k in d, k
    assert d["rollingCountSuccess"] == 3 and d["rollingCountFailure"] == 2
    assert d["rollingCountFallbackSuccess"] == 2
    assert set(d["latencyExecute"]) == {"0", "25", "50", "75", "90", "95", "99", "99.5", "100"}
    assert d["propertyValue_circuitBreakerRequestVolumeThreshold"] == 5
    assert d["propertyValue_executionIsolationThreadTimeoutInMilliseconds"] == 600
    p = json.loads(c.pool_json())
    assert p["type"] == "HystrixThreadPool" and p["currentCorePoolSize"] == 10


def _read_sse(port, path="/hystrix.stream?delay=100", seconds=0.6) -> bytes:
    with socket.create_connection(("127.0.0.1", port), timeout=3) as s:
        s.sendall(f"GET {path} HTTP/1.1\r\nHost: x\r\n\r\n".encode())
        s.settimeout(0.2)
        out = b""
        end = time.monotonic() + seconds
        while time.monotonic() < end:
            try:
                b = s.recv(65536)
                if not b:
                    break
                out += b
            except socket.timeout:
                pass
    return out


def test_stream_pings_before_first_command(hola):
    s = hola()
    out = _read_sse(s.port)
    head, _, body = out.partition(b"\r\n\r\n")
    assert b"200 OK" in head and b"text/event-stream" in head
    assert b"access-control-allow-origin" not in head.lower()  # servlet, not JAX-RS
    assert b"ping: " in body


def test_stream_reports_command_after_chaining(hola):
    with FakeAloha() as aloha:
        s = hola(args=["--aloha-url", aloha.url, "--feign-log", "none"])
        s.get("/api/hola-chaining")
        out = _read_sse(s.port)
    events = [json.loads(l[6:]) for l in out.decode(errors="replace").splitlines() if l.startswith("data: {")]
    types = {e["type"] for e in events}
    assert types == {"HystrixCommand", "HystrixThreadPool"}
    cmd = next(e for e in events if e["type"] == "HystrixCommand")
    assert cmd["name"] == "aloha" and cmd["group"] == aloha.url and cmd["rollingCountSuccess"] >= 1


def test_semaphore_isolation(native):
    """execution.isolation.strategy=SEMAPHORE: semaphore.maxConcurrentRequests bounds the
    calls, rejections are SEMAPHORE_REJECTED, nothing queues and no pool task is counted."""
    c = native.HystrixCommand({**QUEUE, "hystrix.command.default.execution.isolation.strategy": "SEMAPHORE",
                               "hystrix.command.default.execution.isolation.semaphore.maxConcurrentRequests": "2"})
    assert [c.try_start(t) for t in range(3)] == ["run", "run", "rejected"]
    assert c.queue_size() == 0
    c.finish("success", 1)
    assert c.try_start() == "run"
    cmd = json.loads(c.stream_json())
    assert cmd["rollingCountSemaphoreRejected"] == 1 and cmd["rollingCountThreadPoolRejected"] == 0
    assert cmd["propertyValue_executionIsolationStrategy"] == "SEMAPHORE"
    pool = json.loads(c.pool_json())
    assert pool["currentCompletedTaskCount"] == 0 and pool["rollingCountThreadsExecuted"] == 0


def test_stream_has_no_pool_frame_for_semaphore_commands(hola):
    """HystrixMetricsPoller publishes a thread pool only after a task completed on it."""
    with FakeAloha() as aloha:
        s = hola(args=["--aloha-url", aloha.url, "--feign-log", "none",
                       "-Dhystrix.command.default.execution.isolation.strategy=SEMAPHORE"])
        s.get("/api/hola-chaining")
        out = _read_sse(s.port)
    events = [json.loads(l[6:]) for l in out.decode(errors="replace").splitlines() if l.startswith("data: {")]
    assert {e["type"] for e in events} == {"HystrixCommand"}
    assert events[0]["rollingCountSuccess"] >= 1


def test_rolling_percentile_disabled_reports_minus_one(native):
    c = native.HystrixCommand({**TUNED, "hystrix.command.default.metrics.rollingPercentile.enabled": "false"})
    assert c.try_start() == "run"
    c.finish("success", 12)
    cmd = json.loads(c.stream_json())
    assert set(cmd["latencyExecute"].values()) == {-1} and cmd["latencyExecute_mean"] == -1
    assert set(cmd["latencyTotal"].values()) == {-1} and cmd["latencyTotal_mean"] == -1


def test_stream_connection_limit(hola):
    s = hola(args=["--hystrix-stream-max", "1"])
    with socket.create_connection(("127.0.0.1", s.port), timeout=3) as first:
        first.sendall(b"GET /hystrix.stream HTTP/1.1\r\nHost: x\r\n\r\n")
        first.recv(100)
        st, _, body = s.get("/hystrix.stream")
        assert st == 503
    time.sleep(0.2)
    out = _read_sse(s.port, seconds=0.3)
    assert b"200 OK" in out


@pytest.mark.parametrize("args", [["--hystrix-stream-max", "2"], ["-Dhystrix.stream.maxConcurrentConnections=2"]])
def test_stream_limit_message_uses_configured_max(hola, args):
    """The 503 text names the configured limit, as HystrixMetricsStreamServlet does; the limit
    comes from --hystrix-stream-max or the servlet's Archaius property."""
    s = hola(args=args)
    subs = []
    try:
        for _ in range(2):
            c = socket.create_connection(("127.0.0.1", s.port), timeout=3)
            c.sendall(b"GET /hystrix.stream HTTP/1.1\r\nHost: x\r\n\r\n")
            assert b"200 OK" in c.recv(100)
            subs.append(c)
        st, _, body = s.get("/hystrix.stream")
        assert st == 503 and body == b"MaxConcurrentConnections reached: 2"
    finally:
        for c in subs:
            c.close()


def _metric(s, name: str) -> int:
    _, _, body = s.get("/metrics")
    line = next(l for l in body.decode().splitlines() if l.startswith(name + " "))
    return int(float(line.split()[1]))


def test_stalled_subscriber_is_bounded_then_closed(hola):
    """A subscriber that never reads: frames stop being queued once 64 KB are unsent (memory
    stays bounded), and after --hystrix-stream-stall-ms it is closed, freeing its slot."""
    with FakeAloha() as aloha:
        s = hola(args=["--aloha-url", aloha.url, "--feign-log", "none", "--hystrix-stream-max", "1",
                       "--hystrix-stream-stall-ms", "1500"], threads=1)
        s.get("/api/hola-chaining")  # the command has run: every frame carries its JSON
    rss0 = s.memory_kb().get("VmRSS", 0)
    c = socket.socket()
    c.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 2048)
    c.connect(("127.0.0.1", s.port))
    try:
        c.sendall(b"GET /hystrix.stream?delay=10 HTTP/1.1\r\nHost: x\r\n\r\n")
        deadline = time.monotonic() + 10
        while _metric(s, "hola_hystrix_stream_frames_skipped_total") == 0 and time.monotonic() < deadline:
            time.sleep(0.1)
        assert _metric(s, "hola_hystrix_stream_frames_skipped_total") > 0
        assert s.get("/hystrix.stream")[0] == 503  # the stalled subscriber still holds the slot
        while _metric(s, "hola_hystrix_stream_stalled_closed_total") == 0 and time.monotonic() < deadline:
            time.sleep(0.1)
        assert _metric(s, "hola_hystrix_stream_stalled_closed_total") == 1
        assert _metric(s, "hola_hystrix_stream_subscribers") == 0
        if not os.environ.get("HOLA_SANITIZER"):  # sanitizer allocators grow RSS on their own
            assert s.memory_kb().get("VmRSS", 0) - rss0 < 4096
        out = _read_sse(s.port, seconds=0.3)  # the slot is free again
        assert b"200 OK" in out
    finally:
        c.close()


@pytest.mark.parametrize("fail_every", [0, 1, 3])
def test_concurrent_accounting_adds_up(native, fail_every):
    """8 C++ threads share one command (as the server's workers do). The per-thread metric
    shards, the atomic bulkhead and the CAS-driven breaker must account for every call."""
    r = native.hystrix_stress(threads=8, iters=20000, pool=4, fail_every=fail_every, volume=5)
    ev = r["events"]
    total = 8 * 20000
    assert r["runs"] + r["short_circuited"] + r["rejected"] == total
    assert ev.get("SUCCESS", 0) + ev.get("FAILURE", 0) == r["runs"] == r["completed"]
    assert ev.get("FAILURE", 0) == r["failures"]
    assert ev.get("SHORT_CIRCUITED", 0) == r["short_circuited"]
    assert ev.get("THREAD_POOL_REJECTED", 0) == r["rejected"]
    assert ev.get("FALLBACK_SUCCESS", 0) == r["failures"] + r["short_circuited"] + r["rejected"]
    assert r["concurrent"] == 0 and 1 <= r["largest"] <= 4
    if fail_every == 1:  # every call fails: the breaker must open and short-circuit most calls
        assert r["short_circuited"] > total // 2
    if fail_every == 0:
        # no call fails, but bulkhead rejections count as errors in Hystrix's health counts:
        # the breaker may open only if some were rejected (8 threads share 4 slots)
        assert r["short_circuited"] == 0 or r["rejected"] > 0, r


def test_per_thread_bulkhead_is_exact_for_one_thread(native):
    """The per-thread bulkhead (Command::set_per_thread_bulkhead, pools of 64 or more): one
    thread's share is pool / 16, and past it the thread borrows from the other shares, so it
    can still hold the whole pool; the next call is rejected, as with one shared count."""
    c = native.HystrixCommand({"hystrix.threadpool.default.coreSize": "100",
                               "hystrix.command.default.circuitBreaker.requestVolumeThreshold": "1000000"})
    c.set_per_thread_bulkhead(True)
    assert [c.try_start() for _ in range(100)] == ["run"] * 100
    assert c.try_start() == "rejected"
    pool = json.loads(c.pool_json())
    assert pool["currentActiveCount"] == 100 and pool["currentLargestPoolSize"] == 100
    for _ in range(100):
        c.finish("success", 1)
    assert json.loads(c.pool_json())["currentActiveCount"] == 0
    assert [c.try_start() for _ in range(100)] == ["run"] * 100  # every borrowed slot went back


def test_per_thread_bulkhead_leaves_small_pools_shared(native):
    """Below 64 slots (the reference's 10) the one shared, exact count stays in use."""
    c = native.HystrixCommand({"hystrix.threadpool.default.coreSize": "10"})
    c.set_per_thread_bulkhead(True)
    assert [c.try_start() for _ in range(11)] == ["run"] * 10 + ["rejected"]


@pytest.mark.parametrize("fail_every", [0, 3])
def test_per_thread_bulkhead_accounting_adds_up(native, fail_every):
    """Eight C++ threads on one command with the per-thread bulkhead: every call accounted
    for, no slot left taken, and the pool never exceeded (borrowing included)."""
    r = native.hystrix_stress(threads=8, iters=20000, pool=64, fail_every=fail_every, volume=1000000,
                              per_thread=True)
    ev = r["events"]
    assert r["runs"] + r["short_circuited"] + r["rejected"] == 8 * 20000
    assert ev.get("SUCCESS", 0) + ev.get("FAILURE", 0) == r["runs"] == r["completed"]
    assert r["concurrent"] == 0 and 1 <= r["largest"] <= 64


def test_bulkhead_stays_exact_across_a_reload_that_switches_modes(native):
    """A reload of coreSize across kPerThreadMinPool switches between the per-thread shares and
    the one shared count with calls in flight. Hystrix's pool never runs more than coreSize
    (ThreadPoolExecutor.setCorePoolSize lets the excess finish, and rejects meanwhile), and
    neither may this: each mode counts the calls the other one admitted."""
    props = {"hystrix.command.default.circuitBreaker.requestVolumeThreshold": "1000000"}
    c = native.HystrixCommand({**props, "hystrix.threadpool.default.coreSize": "128"})
    c.set_per_thread_bulkhead(True)
    assert [c.try_start() for _ in range(100)] == ["run"] * 100  # per-thread shares
    c.update({**props, "hystrix.threadpool.default.coreSize": "10"})  # shared count now
    assert c.try_start() == "rejected"  # 100 still running against a pool of 10
    for _ in range(95):
        c.finish("success", 1)
    assert [c.try_start() for _ in range(6)] == ["run"] * 5 + ["rejected"]
    c.update({**props, "hystrix.threadpool.default.coreSize": "128"})  # per-thread again
    assert [c.try_start() for _ in range(119)] == ["run"] * 118 + ["rejected"]
    assert json.loads(c.pool_json())["currentActiveCount"] == 128
    for _ in range(128):
        c.finish("success", 1)
    assert json.loads(c.pool_json())["currentActiveCount"] == 0
    assert [c.try_start() for _ in range(129)] == ["run"] * 128 + ["rejected"]
