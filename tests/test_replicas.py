"""Replica scale-out without a cluster: N pinned replicas behind the
native round-robin proxy, greeting rotation, failure of a replica under load, supervisor
restarts, graceful shutdown."""
import json
import os
import signal
import socket
import subprocess
import threading
import time

import pytest

from hola_amd.parallel.replicas import ReplicaSet, RRProxy
from hola_amd.utils.net import http_get



def _log_has(proc, text: str, timeout: float = 3.0) -> bool:
    """The log writer thread may lag the event that logged: wait for the line."""
    deadline = time.monotonic() + timeout
    while text not in proc.log():
        if time.monotonic() > deadline:
            return False
        time.sleep(0.05)
    return True

def greeting_via(port):
    st, _, body = http_get("127.0.0.1", port, "/api/hola")
    assert st == 200
    return body.decode()


def test_proxy_round_robin_rotation():
    with ReplicaSet(3, threads_per_replica=1, supervise=False) as rs, RRProxy(rs.targets) as px:
        seen = [greeting_via(px.port) for _ in range(6)]  # one connection per request
    assert sorted(set(seen)) == ["Hola de replica-0", "Hola de replica-1", "Hola de replica-2"]
    assert seen[:3] != seen[3:6] or len(set(seen[:3])) == 3


def test_proxy_skips_dead_replica_and_recovers():
    rs = ReplicaSet(2, threads_per_replica=1, supervise=False).start()
    try:
        with RRProxy(rs.targets, health_ms=50) as px:
            rs.kill(1)
            time.sleep(0.3)  # health checker marks it DOWN
            seen = {greeting_via(px.port) for _ in range(8)}
            assert seen == {"Hola de replica-0"}
            assert _log_has(px, "is DOWN")
            rs.procs[1] = rs._spawn(1)  # platform restarts the pod
            time.sleep(0.3)
            seen = {greeting_via(px.port) for _ in range(8)}
            assert seen == {"Hola de replica-0", "Hola de replica-1"}
    finally:
        rs.stop()


def test_proxy_half_close_and_backpressure():
    """The proxy passes a client's FIN on after its request (the response still arrives), and
    relays a pipelined burst far larger than its 16 KiB buffers in order."""
    import socket

    with ReplicaSet(1, threads_per_replica=1, supervise=False) as rs, RRProxy(rs.targets) as px:
        with socket.create_connection(("127.0.0.1", px.port), timeout=5) as sk:
            sk.sendall(b"GET /api/health HTTP/1.1\r\nHost: x\r\n\r\n")
            sk.shutdown(socket.SHUT_WR)
            data = b""
            while chunk := sk.recv(65536):
                data += chunk
        assert data.startswith(b"HTTP/1.1 200") and data.endswith(b"I'm ok")
        n = 300  # ~300 x the swagger document through one session
        req = b"GET /api/swagger.json HTTP/1.1\r\nHost: x\r\n\r\n"
        with socket.create_connection(("127.0.0.1", px.port), timeout=10) as sk:
            sk.sendall(req * n + b"GET /api/hola HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
            data = b""
            while chunk := sk.recv(1 << 20):
                data += chunk
        assert data.count(b"HTTP/1.1 200 OK") == n + 1
        assert data.endswith(b"Hola de replica-0")


def test_proxy_idle_timeout_closes_silent_sessions():
    """A session with no traffic either way for --idle-timeout-ms is closed by the proxy; an
    active one is not."""
    import socket

    with ReplicaSet(1, threads_per_replica=1, supervise=False) as rs, \
            RRProxy(rs.targets, idle_timeout_ms=300) as px:
        idle = socket.create_connection(("127.0.0.1", px.port), timeout=5)
        busy = socket.create_connection(("127.0.0.1", px.port), timeout=5)
        t0 = time.monotonic()
        while time.monotonic() - t0 < 1.2:
            busy.sendall(b"GET /api/health HTTP/1.1\r\nHost: x\r\n\r\n")
            assert busy.recv(4096).startswith(b"HTTP/1.1 200")
            time.sleep(0.1)
        idle.settimeout(2)
        assert idle.recv(16) == b""  # closed by the proxy
        idle.close()
        busy.close()


def test_proxy_fails_over_on_refused_connect():
    """A backend that refuses is marked DOWN at once and the connection goes to the next one,
    before any health check has run."""
    rs = ReplicaSet(2, threads_per_replica=1, supervise=False).start()
    try:
        with RRProxy(rs.targets, health_ms=60000) as px:
            time.sleep(0.3)  # the one health round (at start) saw both UP
            assert "is DOWN" not in px.log()
            rs.kill(0)
            time.sleep(0.1)
            seen = {greeting_via(px.port) for _ in range(6)}
            assert seen == {"Hola de replica-1"}
            assert _log_has(px, "is DOWN")
    finally:
        rs.stop()


def test_proxy_reports_why_sessions_ended():
    """At exit the proxy accounts for sessions that ended on an error, by side, with the last
    errno: a client that resets its connection, and a connect refused by a dead backend."""
    import struct

    rs = ReplicaSet(2, threads_per_replica=1, supervise=False).start()
    try:
        with RRProxy(rs.targets, health_ms=60000) as px:
            sk = socket.create_connection(("127.0.0.1", px.port), timeout=5)
            sk.sendall(b"GET /api/health HTTP/1.1\r\nHost: x\r\n\r\n")
            assert sk.recv(4096).startswith(b"HTTP/1.1 200")
            sk.setsockopt(socket.SOL_SOCKET, socket.SO_LINGER, struct.pack("ii", 1, 0))
            sk.close()  # RST to the proxy
            time.sleep(0.2)
            rs.kill(0)
            time.sleep(0.1)
            for _ in range(4):  # one of these meets the dead backend and fails over
                assert greeting_via(px.port) == "Hola de replica-1"
            px.stop()
            stats = [ln for ln in px.log().splitlines() if "sessions closed" in ln]
    finally:
        rs.stop()
    assert len(stats) == 1, stats
    line = stats[0]
    assert "client side 1 (last Connection reset by peer)" in line, line
    assert "backend side 0 (last -)" in line, line
    assert "backend connects failed 1 (last Connection refused)" in line, line


def test_proxy_reads_its_endpoints_before_it_listens(tmp_path):
    """Service mode (--endpoints-file): the set is read before the port is bound and the port
    file written, so the first client is routed, not reset on an empty set (a race the
    sanitized endpoints test once met as `backend connects failed 2`)."""
    from hola_amd.native import binary

    eps, port_file, log_path = tmp_path / "eps", tmp_path / "port", tmp_path / "proxy.log"
    with ReplicaSet(2, threads_per_replica=1, supervise=False) as rs, open(log_path, "wb") as log:
        eps.write_text("# gen 7\n" + "".join(f"{h}:{p}\n" for h, p in rs.targets))
        proc = subprocess.Popen([str(binary("hola_rrproxy")), "--host", "127.0.0.1", "--port", "0",
                                 "--endpoints-file", str(eps), "--health-ms", "0", "--no-failover",
                                 "--port-file", str(port_file)], stderr=log)
        try:
            deadline = time.monotonic() + 10
            while not port_file.exists() and time.monotonic() < deadline:
                time.sleep(0.001)
            assert greeting_via(int(port_file.read_text())).startswith("Hola de replica-")
        finally:
            proc.send_signal(signal.SIGTERM)
            proc.wait(timeout=10)
    text = log_path.read_text()
    assert text.index("endpoints now 2 backends") < text.index("listening on"), text
    assert "-> 2 backends" in text and "backend connects failed 0" in text, text
    assert (tmp_path / "eps.applied").read_text().strip() == "7"


def test_supervisor_restarts_crashed_replica():
    with ReplicaSet(2, threads_per_replica=1, supervise=True) as rs:
        old = rs.procs[0].proc.pid
        rs.kill(0)
        deadline = time.time() + 10
        while time.time() < deadline and (rs.restarts[0] == 0):
            time.sleep(0.05)
        assert rs.restarts[0] == 1 and rs.procs[0].proc.pid != old
        assert greeting_via(rs.ports[0]) == "Hola de replica-0"


def test_supervisor_backs_off_a_crash_looping_replica():
    """A replica that cannot come back (its port is taken) is retried with growing delays,
    0.1 s doubling up to the cap, like kubelet's CrashLoopBackOff, not every poll; once the
    port is free again it is back within one capped delay."""
    import socket

    with ReplicaSet(1, threads_per_replica=1, supervise=True, max_backoff_s=1.0) as rs:
        port = rs.ports[0]
        rs.kill(0)
        blocker = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        blocker.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        blocker.bind(("0.0.0.0", port))
        blocker.listen(1)
        try:
            time.sleep(2.5)
            fails = rs.failed_restarts[0]
            # delays 0.1, 0.2, 0.4, 0.8, 1.0 s: about 4 tries in 2.5 s (polling every 50 ms
            # without back-off would make dozens)
            assert 2 <= fails <= 6, fails
            assert rs.restarts[0] == 0
        finally:
            blocker.close()
        deadline = time.time() + 5
        while time.time() < deadline and rs.restarts[0] == 0:
            time.sleep(0.05)
        assert rs.restarts[0] == 1
        assert greeting_via(port) == "Hola de replica-0"


def test_kill_replica_under_load_client_rr():
    """Chaos: SIGKILL one replica mid-run; the other keeps answering, the loadgen reconnects."""
    from hola_amd.parallel.loadgen import ControlledLoadgen

    with ReplicaSet(2, threads_per_replica=1, supervise=True) as rs:
        lg = ControlledLoadgen(rs.targets, connections=8, threads=1)
        try:
            lg.run(50)
            rs.kill(1)
            r = lg.run(50)  # reconnects to the restarted replica
            assert r["requests"] >= 8 * 50 - 8
        finally:
            lg.close()


def test_reuseport_group_spreads_and_survives_a_kill():
    """--lb reuseport: replicas share one port; the kernel spreads connections over the
    SO_REUSEPORT group, and a killed replica's listeners leave it, so every new connection
    lands on a live replica (no proxy, no health check needed)."""
    with ReplicaSet(3, threads_per_replica=1, supervise=False, shared_port=0) as rs:
        assert len(set(rs.ports)) == 1 and rs.targets == [("127.0.0.1", rs.shared_port)]
        seen = {greeting_via(rs.shared_port) for _ in range(60)}
        assert seen == {"Hola de replica-0", "Hola de replica-1", "Hola de replica-2"}
        rs.kill(1)
        after = [greeting_via(rs.shared_port) for _ in range(40)]
        assert "Hola de replica-1" not in after
        assert set(after) == {"Hola de replica-0", "Hola de replica-2"}


def test_graceful_shutdown_drains_inflight(hola):
    """SIGTERM while a chaining request waits on a slow aloha: the response still completes."""
    from hola_amd.testing.fakes import FakeAloha

    with FakeAloha(mode="slow", delay_s=0.3) as aloha:
        s = hola(args=["--aloha-url", aloha.url, "--feign-log", "none"])
        out = {}

        def req():
            out["r"] = s.get("/api/hola-chaining", timeout=5)

        t = threading.Thread(target=req)
        t.start()
        time.sleep(0.1)
        s.proc.send_signal(signal.SIGTERM)
        t.join()
        assert out["r"][0] == 200 and json.loads(out["r"][2])[1] == "Aloha mai aloha-1"
        assert s.proc.wait(timeout=10) == 0
        assert "shutdown complete" in s.log()


def test_scaling_harness_smoke():
    from hola_amd.parallel import scaling

    rows = []
    import io
    import contextlib

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        scaling.main(["--replicas", "1,2", "--duration", "0.5", "--warmup", "0.2", "--budget", "6",
                      "--connections-per-replica", "8"])
    lines = [json.loads(l) for l in buf.getvalue().splitlines() if l.startswith("{")]
    assert [r["replicas"] for r in lines] == [1, 2]
    assert all(r["rps"] > 0 and r["errors"] == 0 for r in lines)
    assert lines[1]["connections"] == 16


def test_scaling_harness_plain_dealing():
    """--lb plain: the client-side front blind to topology. Every load-generator
    thread deals its connections over every replica, every body is checked against the replica
    that answered it, and each replica serves its share."""
    from hola_amd.parallel import scaling
    import io
    import contextlib

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        scaling.main(["--replicas", "2", "--duration", "0.5", "--warmup", "0.2", "--budget", "6",
                      "--connections-per-replica", "8", "--lb", "plain"])
    (row,) = [json.loads(l) for l in buf.getvalue().splitlines() if l.startswith("{")]
    assert row["lb"] == "plain" and row["errors"] == 0 and row["body_mismatch"] == 0, row
    assert row["lb_detail"]["dealing"].startswith("thread t -> every replica")
    reqs = [r["requests"] for r in row["per_replica"]]
    assert min(reqs) > 0.25 * sum(reqs), reqs


def test_scaling_harness_proxy_mode():
    """--lb proxy: load generator -> hola_rrproxy -> replicas, with the mirrored core plan."""
    from hola_amd.parallel import scaling
    import io
    import contextlib

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        scaling.main(["--replicas", "1,2", "--duration", "0.5", "--warmup", "0.2", "--budget", "8",
                      "--connections-per-replica", "8", "--lb", "proxy"])
    lines = [json.loads(l) for l in buf.getvalue().splitlines() if l.startswith("{")]
    assert [r["replicas"] for r in lines] == [1, 2]
    assert all(r["rps"] > 0 and r["errors"] == 0 and r["lb"] == "proxy" for r in lines)
    assert all(r["cpu_map"]["proxy"] for r in lines)


def test_open_loop_rate_mode(hola):
    from hola_amd.parallel.loadgen import run_duration

    s = hola(threads=1)
    res = run_duration([("127.0.0.1", s.port)], 8, 1, 1.0, 0.3, rate=5000)
    assert res["mode"] == "open-loop"
    assert 4500 <= res["rps"] <= 5500
    assert res["latency"]["errors"] == 0 and res["latency"]["p50_ns"] > 0


def _cpu_s(pid: int) -> float:
    import os
    f = open(f"/proc/{pid}/stat").read().rsplit(")", 1)[1].split()
    return (int(f[11]) + int(f[12])) / os.sysconf("SC_CLK_TCK")


def _exhaust_fds_then_recover(pid: int, port: int, fd_limit: int):
    """Lowers the process's RLIMIT_NOFILE, holds enough client connections to hit it, checks
    that the process idles (a still-armed level-triggered listener would spin a core at
    100 %), then frees the connections and checks that accepting resumes."""
    import resource
    import socket

    soft, hard = resource.prlimit(pid, resource.RLIMIT_NOFILE)
    resource.prlimit(pid, resource.RLIMIT_NOFILE, (fd_limit, hard))  # soft limit only: no privilege needed
    held = []
    try:
        for _ in range(fd_limit + 8):
            c = socket.create_connection(("127.0.0.1", port), timeout=5)
            held.append(c)
        time.sleep(0.3)  # every fd is in use and the rest wait in the backlog
        c0 = _cpu_s(pid)
        time.sleep(1.0)
        assert _cpu_s(pid) - c0 < 0.3, "accept loop spins at the fd limit"
    finally:
        for c in held:
            c.close()
    resource.prlimit(pid, resource.RLIMIT_NOFILE, (soft, hard))
    deadline = time.monotonic() + 5
    while True:
        try:
            assert greeting_via(port).startswith("Hola de")
            return
        except (OSError, AssertionError):
            if time.monotonic() > deadline:
                raise
            time.sleep(0.1)


def test_proxy_backs_off_at_fd_limit():
    with ReplicaSet(1, threads_per_replica=1, supervise=False) as rs, RRProxy(rs.targets) as px:
        _exhaust_fds_then_recover(px.proc.pid, px.port, 48)
        assert _log_has(px, "fd limit")
        assert "is DOWN" not in px.log()  # running out of local fds says nothing about a backend


@pytest.mark.skipif(os.environ.get("HOLA_SANITIZER") in ("asan", "tsan"),
                    reason="UBSan's vptr check tests vtable readability through a pipe(2); at "
                           "RLIMIT_NOFILE that pipe cannot be created and every virtual call is "
                           "reported as 'invalid vptr' (a sanitizer false positive)")
def test_server_backs_off_at_fd_limit(hola):
    s = hola(env={"HOSTNAME": "h"}, threads=1)
    _exhaust_fds_then_recover(s.proc.pid, s.port, 48)


def test_loadgen_service_mode_dnats_each_new_connection(tmp_path, hola):
    """`hola_loadgen --endpoints-file F` (the Service's iptables/IPVS semantics in the client):
    each new connection goes to a current endpoint of F, established ones keep their pod when
    F changes, bodies are checked per pod, and a connect refused by a listed endpoint that is
    gone counts as an error (no failover)."""
    from hola_amd import native

    a = hola(env={"HOSTNAME": "a"}, threads=1)
    b = hola(env={"HOSTNAME": "b"}, threads=1)
    eps = tmp_path / "eps"

    def publish(*ports):
        tmp = tmp_path / "eps.tmp"
        tmp.write_text("# gen\n" + "".join(f"127.0.0.1:{p}\n" for p in ports))
        os.replace(tmp, eps)

    def run(seconds, conns, *extra):
        r = subprocess.run([str(native.binary("hola_loadgen")), "-t", "2", "-c", str(conns), "-d", f"{seconds}s",
                            "--json", "--verify-body", "--endpoints-file", str(eps), *extra,
                            "http://127.0.0.2:9/api/hola"],
                           capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr
        return json.loads(r.stdout.strip().splitlines()[-1])

    publish(a.port, b.port)
    r = run(1, 8)
    lat = r["latency"]
    assert r["targets"] == 2 and lat["errors"] == 0 and lat["body_mismatch"] == 0
    assert lat["body_checked"] == lat["count"] > 100
    # a listed endpoint that refuses: each refused (re)connect is an error, the other endpoint
    # still serves (every request on its own connection here, so connects keep happening)
    gone = socket.socket()
    gone.bind(("127.0.0.1", 0))
    dead_port = gone.getsockname()[1]
    gone.close()
    publish(a.port, dead_port)
    r = run(1, 4, "-H", "Connection: close")
    assert r["latency"]["errors"] > 0 and r["latency"]["count"] > 100, r
    assert r["latency"]["reconnects"] > 100 and r["latency"]["body_mismatch"] == 0
    # established connections keep their pod: the file changes under a running load
    publish(a.port)
    lg = subprocess.Popen([str(native.binary("hola_loadgen")), "-t", "1", "-c", "4", "-d", "3s", "--json",
                           "--verify-body", "--endpoints-file", str(eps), "http://127.0.0.2:9/api/hola"],
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    time.sleep(1.0)
    publish(b.port)
    out, err = lg.communicate(timeout=30)
    r = json.loads(out.strip().splitlines()[-1])
    assert r["targets"] == 1 and r["latency"]["errors"] == 0, r  # never reconnected, never saw b


def test_targets_follow_replica_order():
    """ReplicaSet.targets[i] is replica i (HOSTNAME replica-<i>, CPUs cpu_plan[i]), whatever
    order the free ports came in: the scaling harness places load-generator thread t next to
    replica t's cores and deals it target t. (Sorted ports put half of the N = 2 miniature's
    clients on the wrong replica's core, profiles/round5/04_scale_mini.)"""
    from hola_amd.parallel.replicas import ReplicaSet

    rs = ReplicaSet(3, supervise=False)
    rs.ports = [40003, 40001, 40002]
    assert [p for _, p in rs.targets] == [40003, 40001, 40002]
    rs.ports = [40005] * 3  # a shared (reuseport) port: one address
    assert [p for _, p in rs.targets] == [40005]


def test_reuseport_group_hands_connections_by_incoming_cpu(hola_bin):
    """--accept reuseport --reuseport-cpu self: two replicas share one port, each worker's
    listener names its own CPU as the incoming CPU, and the kernel (Linux 6.1+) hands each new
    connection to the replica whose worker sits on the CPU the connection's SYN came from: the
    replica-local placement client-side round-robin gets, without a client that knows the
    replicas (profiles/round5/04_scale_mini)."""
    import os
    import socket

    from hola_amd.server import HolaProcess
    from hola_amd.utils.net import free_port

    cpus = sorted(os.sched_getaffinity(0))
    if len(cpus) < 2:
        pytest.skip("needs two CPUs")
    a_cpu, b_cpu = cpus[0], cpus[-1]
    port = free_port()
    args = ["--accept", "reuseport", "--reuseport-cpu", "self", "--no-tracing", "--log-level", "warn"]
    with HolaProcess(args=args, env={"HOSTNAME": "a"}, port=port, threads=1, cpu_list=str(a_cpu)), \
            HolaProcess(args=args, env={"HOSTNAME": "b"}, port=port, threads=1, cpu_list=str(b_cpu)):
        old = os.sched_getaffinity(0)
        seen = {}
        try:
            for cpu, want in ((a_cpu, b"Hola de a"), (b_cpu, b"Hola de b")):
                os.sched_setaffinity(0, {cpu})
                for _ in range(16):
                    with socket.create_connection(("127.0.0.1", port), timeout=5) as c:
                        c.sendall(b"GET /api/hola HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
                        body = c.recv(4096).split(b"\r\n\r\n", 1)[1]
                    seen.setdefault(cpu, []).append(body == want)
        finally:
            os.sched_setaffinity(0, old)
    if os.uname().release.split(".")[:2] < ["6", "1"] and not all(all(v) for v in seen.values()):
        pytest.skip("kernel without SO_INCOMING_CPU selection in reuseport groups")
    assert all(all(v) for v in seen.values()), seen
