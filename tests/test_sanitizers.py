"""Race / memory-error detection: the server built with ThreadSanitizer and
with AddressSanitizer+UBSan is driven through every subsystem concurrently — pipelined and
parallel requests, chaining against a fake aloha in several failure modes (timeouts fire on
the event loop while responses race them), /hystrix.stream subscribers, config hot reloads
from the watcher thread, span reporting to a fake Zipkin — then shut down with SIGTERM.
Any sanitizer report fails the test. Host code only (no GPU code exists)."""
import os
import signal
import socket
import threading
import time

import pytest

from hola_amd.native import build, build_dir
from hola_amd.server import HolaProcess
from hola_amd.testing.fakes import FakeAloha, FakeZipkin

pytestmark = pytest.mark.sanitizer

SAN_ENV = {
    "tsan": {"TSAN_OPTIONS": "halt_on_error=1 exitcode=66 second_deadlock_stack=1"},
    "asan": {"ASAN_OPTIONS": "detect_leaks=1 halt_on_error=1 exitcode=66",
             "UBSAN_OPTIONS": "halt_on_error=1 print_stacktrace=1 exitcode=66"},
}


def _workload(s: HolaProcess, aloha: FakeAloha, conf):
    errors = []

    def hammer(path, n):
        try:
            for _ in range(n):
                st, _, _ = s.get(path, timeout=10)
                if st not in (200, 406):
                    errors.append((path, st))
        except Exception as e:  # noqa: BLE001
            errors.append((path, repr(e)))

    def pipelined():
        try:
            with socket.create_connection(("127.0.0.1", s.port), timeout=10) as c:
                c.sendall(b"GET /api/hola HTTP/1.1\r\nHost: x\r\n\r\n" * 50 +
                          b"GET /api/health HTTP/1.1\r\nConnection: close\r\n\r\n")
                data = b""
                while True:
                    b = c.recv(65536)
                    if not b:
                        break
                    data += b
                if data.count(b"200 OK") != 51:
                    errors.append(("pipelined", data.count(b"200 OK")))
        except Exception as e:  # noqa: BLE001
            errors.append(("pipelined", repr(e)))

    def stream():
        with socket.create_connection(("127.0.0.1", s.port), timeout=5) as c:
            c.sendall(b"GET /hystrix.stream?delay=20 HTTP/1.1\r\nHost: x\r\n\r\n")
            end = time.monotonic() + 1.0
            c.settimeout(0.2)
            while time.monotonic() < end:
                try:
                    c.recv(65536)
                except socket.timeout:
                    pass

    def modes():
        for m in ("ok", "error", "slow", "garbage", "ok", "close", "unavailable", "ok"):
            aloha.set_mode(m, delay_s=0.3)
            time.sleep(0.25)

    def reload():
        for i in range(10):
            conf.write_text(f"hello=v{i} %s\n")
            time.sleep(0.08)

    ts = [threading.Thread(target=hammer, args=("/api/hola", 150)) for _ in range(3)]
    ts += [threading.Thread(target=hammer, args=("/api/hola-chaining", 40)) for _ in range(4)]
    ts += [threading.Thread(target=hammer, args=("/metrics", 20)), threading.Thread(target=pipelined),
           threading.Thread(target=stream), threading.Thread(target=stream), threading.Thread(target=modes),
           threading.Thread(target=reload)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return errors


def tsan_wrapper():
    """gcc 11's TSan aborts with "unexpected memory mapping" on kernels with high mmap ASLR
    entropy (seen on the MI355X host's 6.18 kernel); run it with address randomisation off."""
    import platform
    import shutil

    return ["setarch", platform.machine(), "-R"] if shutil.which("setarch") else []


# "default": the server's defaults. "round3": the round-3 paths together — pipelined aloha
# calls (shared connections drained on Hystrix timeouts), Feign BASIC logging through the log
# rings, adaptive busy-polling, and a SIGTERM that first runs the shutdown delay (readiness
# failing, `Connection: close` on every response) before the drain.
VARIANTS = {
    "default": ["--feign-log", "none"],
    "round3": ["--feign-log", "basic", "--aloha-pipeline", "4", "--busy-poll-us", "auto",
               "--shutdown-delay-ms", "300"],
}


@pytest.mark.parametrize("variant", sorted(VARIANTS))
@pytest.mark.parametrize("preset", ["tsan", "asan"])
def test_sanitized_server(preset, variant, tmp_path):
    build(preset)
    exe = build_dir(preset) / "hola"
    conf = tmp_path / "t.properties"
    conf.write_text("hello=v %s\n")
    with FakeAloha() as aloha, FakeZipkin() as zipkin:
        s = HolaProcess(args=["--aloha-url", aloha.url, "--zipkin-url", zipkin.url, *VARIANTS[variant],
                              f"-Dconf={conf}", "-Dhystrix.command.default.metrics.healthSnapshot.intervalInMilliseconds=0"],
                        env={"HOSTNAME": "san", **SAN_ENV[preset]}, threads=4, exe=exe, log_level="warn",
                        wrapper=tsan_wrapper() if preset == "tsan" else None)
        s.start(timeout=60)
        try:
            errors = _workload(s, aloha, conf)
        finally:
            rc = s.stop(signal.SIGTERM, timeout=60)
        log = s.log()
    assert "ThreadSanitizer" not in log, log[-6000:]
    assert "AddressSanitizer" not in log and "runtime error" not in log, log[-6000:]
    assert "LeakSanitizer" not in log, log[-6000:]
    assert rc == 0, (rc, log[-3000:])
    assert not errors, errors[:10]


@pytest.mark.parametrize("preset", ["tsan", "asan"])
def test_sanitized_proxy(preset, tmp_path):
    """hola_rrproxy built with a sanitizer: parallel short and keep-alive sessions, pipelined
    bursts, half-closes and a backend killed mid-run (connect failover + health thread racing
    the loops), then SIGTERM with sessions still open (closed and freed at exit)."""
    import subprocess

    from hola_amd.parallel.replicas import ReplicaSet

    build(preset)
    exe = build_dir(preset) / "hola_rrproxy"
    port_file = tmp_path / "port"
    log_path = tmp_path / "proxy.log"
    with ReplicaSet(2, threads_per_replica=2, supervise=False) as rs, open(log_path, "wb") as log:
        cmd = (tsan_wrapper() if preset == "tsan" else []) + [
            str(exe), "--host", "127.0.0.1", "--port", "0", "--threads", "3", "--health-ms", "30",
            "--backends", ",".join(f"{h}:{p}" for h, p in rs.targets), "--port-file", str(port_file)]
        proc = subprocess.Popen(cmd, stderr=log, env={**os.environ, **SAN_ENV[preset]})
        deadline = time.monotonic() + 60
        while not port_file.exists() and time.monotonic() < deadline and proc.poll() is None:
            time.sleep(0.02)
        assert port_file.exists(), log_path.read_text(errors="replace")[-3000:]
        port = int(port_file.read_text())
        errors = []

        def one(path, keep):
            try:
                with socket.create_connection(("127.0.0.1", port), timeout=10) as sk:
                    for k in range(keep):
                        last = k == keep - 1
                        sk.sendall(f"GET {path} HTTP/1.1\r\nHost: x\r\n{'Connection: close' if last else ''}\r\n\r\n"
                                   .encode())
                    if keep == 1:
                        sk.shutdown(socket.SHUT_WR)
                    data = b""
                    while chunk := sk.recv(1 << 16):
                        data += chunk
                if data.count(b"HTTP/1.1 200") != keep:
                    errors.append((path, keep, data[:200]))
            except OSError as e:
                errors.append((path, keep, repr(e)))

        def worker(i):
            for j in range(40):
                one("/api/swagger.json" if j % 5 == 0 else "/api/hola", 1 + (i + j) % 6)

        ts = [threading.Thread(target=worker, args=(i,)) for i in range(6)]
        for t in ts:
            t.start()
        time.sleep(0.3)
        rs.kill(1)  # sessions on it end; new ones fail over, then the health thread marks it down
        for t in ts:
            t.join()
        idle = socket.create_connection(("127.0.0.1", port), timeout=10)  # left open at SIGTERM
        time.sleep(0.1)
        proc.send_signal(signal.SIGTERM)
        rc = proc.wait(timeout=60)
        idle.close()
    text = log_path.read_text(errors="replace")
    assert "Sanitizer" not in text and "runtime error" not in text, text[-6000:]
    assert rc == 0, (rc, text[-3000:])
    # only requests in flight on the killed replica may fail
    assert len(errors) <= 12, errors[:5]


@pytest.mark.parametrize("preset", ["tsan", "asan"])
def test_sanitized_proxy_endpoints_mode(preset, tmp_path):
    """hola_rrproxy in the executor's Service mode (--endpoints-file, no failover) built with a
    sanitizer: keep-alive sessions through it while the endpoints file is replaced again and
    again (the follower thread publishing new backend sets under the session loops), then
    SIGTERM with sessions open. From generation 10 on the lines carry topology hints
    (`h:p@0`), so a reload adds a hint to backends of the set the loops are dealing from: the
    hints live in the published set, never in a Backend a loop is reading."""
    import subprocess

    from hola_amd.parallel.replicas import ReplicaSet

    build(preset)
    exe = build_dir(preset) / "hola_rrproxy"
    port_file = tmp_path / "port"
    eps = tmp_path / "eps"
    log_path = tmp_path / "proxy.log"
    with ReplicaSet(3, threads_per_replica=1, supervise=False) as rs, open(log_path, "wb") as log:
        targets = [f"{h}:{p}" for h, p in rs.targets]

        def publish(gen, chosen):
            tmp = tmp_path / "eps.tmp"
            hint = "@0" if gen >= 10 else ""  # CPU 0's L3, where the proxy threads run here
            tmp.write_text(f"# gen {gen}\n" + "".join(t + hint + "\n" for t in chosen))
            os.replace(tmp, eps)

        publish(1, targets)
        cmd = (tsan_wrapper() if preset == "tsan" else []) + [
            str(exe), "--host", "127.0.0.1", "--port", "0", "--threads", "3", "--endpoints-file", str(eps),
            "--health-ms", "0", "--no-failover", "--idle-timeout-ms", "0", "--port-file", str(port_file)]
        proc = subprocess.Popen(cmd, stderr=log, env={**os.environ, **SAN_ENV[preset]})
        deadline = time.monotonic() + 60
        while not port_file.exists() and time.monotonic() < deadline and proc.poll() is None:
            time.sleep(0.02)
        assert port_file.exists(), log_path.read_text(errors="replace")[-3000:]
        port = int(port_file.read_text())
        errors = []
        stop = threading.Event()

        def client():
            while not stop.is_set():
                try:
                    with socket.create_connection(("127.0.0.1", port), timeout=10) as sk:
                        for _ in range(20):
                            sk.sendall(b"GET /api/hola HTTP/1.1\r\nHost: x\r\n\r\n")
                            data = sk.recv(1 << 16)
                            if b"200 OK" not in data:
                                errors.append(data[:100])
                                break
                except OSError as e:
                    errors.append(repr(e))

        ts = [threading.Thread(target=client) for _ in range(4)]
        for t in ts:
            t.start()
        for gen in range(2, 40):  # every backend stays up: sets change, no connection may fail
            publish(gen, targets[gen % 3:] + targets[:gen % 3][:1])
            time.sleep(0.03)
        stop.set()
        for t in ts:
            t.join()
        applied = (tmp_path / "eps.applied").read_text().strip()
        idle = socket.create_connection(("127.0.0.1", port), timeout=10)
        time.sleep(0.1)
        proc.send_signal(signal.SIGTERM)
        rc = proc.wait(timeout=60)
        idle.close()
    text = log_path.read_text(errors="replace")
    assert "Sanitizer" not in text and "runtime error" not in text, text[-6000:]
    assert rc == 0, (rc, text[-3000:])
    stats = [ln for ln in text.splitlines() if "sessions closed" in ln]
    assert stats, text[-3000:]  # the proxy's own account of why sessions ended
    assert not errors, (errors[:5], stats, text[-3000:])
    assert int(applied) >= 30  # the follower acknowledged the sets as they came


@pytest.mark.parametrize("preset", ["asan", "tsan"])
def test_shutdown_with_parked_calls_and_streams_frees_everything(preset, tmp_path):
    """SIGTERM while a chaining call is parked on a slow aloha (past a short drain), an SSE
    subscriber is open and another never reads: every connection, ticker and pending callback
    must be freed (LeakSanitizer at exit) without touching freed objects."""
    build(preset)
    exe = build_dir(preset) / "hola"
    with FakeAloha() as aloha:
        aloha.set_mode("slow", delay_s=3.0)
        s = HolaProcess(args=["--aloha-url", aloha.url, "--feign-log", "none", "--drain-ms", "100",
                              "--hystrix-timeout-ms", "5000"],
                        env={"HOSTNAME": "san", **SAN_ENV[preset]}, threads=2, exe=exe, log_level="warn",
                        wrapper=tsan_wrapper() if preset == "tsan" else None)
        s.start(timeout=60)
        socks = []
        try:
            def parked():
                try:
                    s.get("/api/hola-chaining", timeout=10)
                except Exception:  # noqa: BLE001 - the server goes away under this request
                    pass

            t = threading.Thread(target=parked, daemon=True)
            t.start()
            for rcvbuf in (None, 2048):
                c = socket.socket()
                if rcvbuf:
                    c.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, rcvbuf)
                c.connect(("127.0.0.1", s.port))
                c.sendall(b"GET /hystrix.stream?delay=10 HTTP/1.1\r\nHost: x\r\n\r\n")
                socks.append(c)
            time.sleep(0.5)  # the call is parked, the streams are ticking
        finally:
            rc = s.stop(signal.SIGTERM, timeout=60)
            for c in socks:
                c.close()
        log = s.log()
    assert "Sanitizer" not in log and "runtime error" not in log, log[-6000:]
    assert rc == 0, (rc, log[-3000:])


@pytest.mark.parametrize("preset", ["asan", "tsan"])
def test_sanitized_exit_watchdog_stall_report(preset, tmp_path):
    """The exit watchdog's stall report under the sanitizers: the loops' activity records are
    read from another thread, and each worker's stack is captured by a signal whose handler
    walks the frame pointers. A termination that outlasts --exit-deadline-ms (a 3 s delay
    against a 0.5 s limit) takes that path with the workers alive."""
    build(preset)
    exe = build_dir(preset) / "hola"
    s = HolaProcess(args=["--shutdown-delay-ms", "3000", "--exit-deadline-ms", "500"],
                    env={"HOSTNAME": "san", **SAN_ENV[preset]}, threads=4, exe=exe, log_level="warn",
                    wrapper=tsan_wrapper() if preset == "tsan" else None)
    s.start(timeout=60)
    try:
        for _ in range(50):
            assert s.get("/api/hola")[0] == 200
        s.proc.send_signal(signal.SIGTERM)
        rc = s.proc.wait(timeout=60)
    finally:
        if s.proc.poll() is None:
            s.proc.kill()
            s.proc.wait()
    log = s.log()
    assert "ThreadSanitizer" not in log, log[-6000:]
    assert "AddressSanitizer" not in log and "runtime error" not in log, log[-6000:]
    assert rc == 3, (rc, log[-3000:])
    assert log.count("hola: worker ") == 4 and "hola: main: shutdown delay" in log, log[-3000:]


@pytest.mark.parametrize("preset", ["release", "tsan", "asan"])
@pytest.mark.parametrize("per_thread", [False, True])
def test_hystrix_shard_lock_held_while_refreshes_and_finishes_run(preset, per_thread):
    """one Hystrix shard's test-and-set lock (released with a plain release
    store) held over and over while eight workers run try_start / complete / circuit_open with
    a health snapshot refreshed on every call (each refresh walks every shard and meets the
    held one) and a reader takes snapshots: no sanitizer report, no deadlock, and the event
    totals add up (bench/probes/hystrix_shard_race.cc)."""
    import subprocess

    build(preset)
    exe = build_dir(preset) / "hola_hystrix_race"
    wrapper = tsan_wrapper() if preset == "tsan" else []
    env = {**os.environ, **SAN_ENV.get(preset, {})}
    # per_thread: the per-thread bulkhead, 64 slots in 4-slot shares, so the workers borrow
    r = subprocess.run([*wrapper, str(exe), "--iters", "20000" if preset == "release" else "4000"]
                       + (["--per-thread"] if per_thread else []),
                       capture_output=True, text=True, timeout=300, env=env)
    assert "ThreadSanitizer" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-6000:]
    assert "runtime error" not in r.stderr, r.stderr[-3000:]
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr[-3000:])
    import json
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["success"] + out["failure"] == out["started"] > 0 and out["holds"] > 0
