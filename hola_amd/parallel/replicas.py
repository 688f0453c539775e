"""Pinned replica sets with a supervisor, and the round-robin proxy in front of them.

This is the node-local version of the reference's deployment model: N
stateless `hola` pods behind a `LoadBalancer` Service (pom.xml:77-80), readiness-gated on
/api/health (pom.xml:90-94), restarted by the platform when they die.
"""
from __future__ import annotations

import os
import signal
import subprocess
import tempfile
import threading
import time
from pathlib import Path

from hola_amd.native import binary
from hola_amd.server import HolaProcess
from hola_amd.utils.cpu import format_cpu_list
from hola_amd.utils.net import free_port, wait_http


class ReplicaSet:
    """N `hola` replicas, each pinned to its own CPU list.

    By default every replica has its own port (a front — client-side round-robin or
    :class:`RRProxy` — spreads the load). With ``shared_port`` all replicas listen on that
    one port with ``--accept reuseport``: they join a single SO_REUSEPORT group and the
    kernel spreads incoming connections over every replica's listeners, with no proxy hop.
    A replica that dies leaves the group when its sockets close, so new connections go to
    the survivors (the role of kube-proxy's endpoint removal).

    HOSTNAME is set to ``replica-<i>`` so responses identify the replica (the k8s pod name
    plays that role in the reference). With ``supervise=True`` a background thread restarts
    any replica that exits (the platform's restart policy), with kubelet's CrashLoopBackOff
    shape: a replica that dies (or fails to come up) within ``stable_s`` of its start waits
    0.1 s, then twice as long after each further quick death, up to ``max_backoff_s``; one
    that ran for longer is restarted at once and its delay is reset.
    """

    def __init__(self, n: int, cpu_plan: list[list[int]] | None = None, threads_per_replica: int = 1,
                 args: list[str] | None = None, env: dict | None = None, supervise: bool = True,
                 base_port: int = 0, log_level: str = "warn", shared_port: int | None = None,
                 stable_s: float = 10.0, max_backoff_s: float = 10.0):
        self.n = n
        self.cpu_plan = cpu_plan
        self.threads = threads_per_replica
        self.args = list(args or [])
        self.env = dict(env or {})
        self.supervise = supervise
        self.log_level = log_level
        self.shared_port = shared_port
        self._base_port = base_port or (shared_port or 0)
        if shared_port is not None:
            self.shared_port = shared_port or free_port()
            self.ports = [self.shared_port] * n
            self.args = ["--accept", "reuseport", *self.args]
        else:
            self.ports = [base_port + i if base_port else free_port() for i in range(n)]
        self.procs: list[HolaProcess | None] = [None] * n
        self.restarts = [0] * n
        self.failed_restarts = [0] * n  # respawns that did not come up (counted towards back-off)
        self.stable_s = stable_s
        self.max_backoff_s = max_backoff_s
        self._started = [0.0] * n
        self._backoff = [0.0] * n
        self._next = [0.0] * n  # when a dead replica may be respawned (0 = death not seen yet)
        self._stop = threading.Event()
        self._lock = threading.Lock()
        self._sup: threading.Thread | None = None

    def _spawn(self, i: int, may_repick: bool = False) -> HolaProcess:
        cpus = self.cpu_plan[i] if self.cpu_plan else None
        for attempt in range(4):
            p = HolaProcess(args=self.args, env={**self.env, "HOSTNAME": f"replica-{i}"}, port=self.ports[i],
                            threads=len(cpus) if cpus else self.threads,
                            cpu_list=format_cpu_list(cpus) if cpus else None, log_level=self.log_level)
            try:
                return p.start()
            except RuntimeError as e:
                # A port picked by free_port() can be taken by another process before the
                # replica binds it: pick again (a shared port only before its first replica).
                # (Only at start-up: a restarted replica keeps its address.)
                own_pick = may_repick and not self._base_port and (self.shared_port is None or i == 0)
                if "Address already in use" not in str(e) or not own_pick or attempt == 3:
                    raise
                if self.shared_port is None:
                    self.ports[i] = free_port()
                else:
                    self.shared_port = free_port()
                    self.ports = [self.shared_port] * self.n
        raise AssertionError("unreachable")

    def start(self, timeout: float = 30.0) -> "ReplicaSet":
        for i in range(self.n):
            self.procs[i] = self._spawn(i, may_repick=True)
            self._started[i] = time.monotonic()
        for i in range(self.n):
            if not wait_http("127.0.0.1", self.ports[i], timeout=timeout):
                raise RuntimeError(f"replica {i} not ready")
        if self.supervise:
            self._sup = threading.Thread(target=self._supervise, daemon=True)
            self._sup.start()
        return self

    def _next_backoff(self, i: int, ran_s: float) -> float:
        if ran_s >= self.stable_s:
            return 0.0
        return min(self.max_backoff_s, max(0.1, self._backoff[i] * 2))

    def _supervise(self) -> None:
        while not self._stop.wait(0.05):
            for i, p in enumerate(self.procs):
                if p is None or p.proc is None or p.proc.poll() is None:
                    continue
                now = time.monotonic()
                if self._next[i] == 0.0:  # the death is new: schedule the restart
                    self._backoff[i] = self._next_backoff(i, now - self._started[i])
                    self._next[i] = now + self._backoff[i]
                if now < self._next[i]:
                    continue
                with self._lock:
                    if self._stop.is_set():
                        return
                    self._started[i] = time.monotonic()
                    try:
                        self.procs[i] = self._spawn(i)
                    except Exception:
                        # did not come up: a quick death, so the next try waits longer
                        self.failed_restarts[i] += 1
                        self._backoff[i] = self._next_backoff(i, 0.0)
                        self._next[i] = time.monotonic() + self._backoff[i]
                        continue
                    self.restarts[i] += 1
                    self._next[i] = 0.0

    def kill(self, i: int, sig: int = signal.SIGKILL) -> None:
        p = self.procs[i]
        if p and p.proc and p.proc.poll() is None:
            p.proc.send_signal(sig)
            p.proc.wait()

    @property
    def targets(self) -> list[tuple[str, int]]:
        """One address per replica, in replica order (target i is replica i, whose CPUs are
        cpu_plan[i]: a load generator that places thread t next to replica t relies on it);
        one address in all with a shared port."""
        return [("127.0.0.1", p) for p in dict.fromkeys(self.ports)]

    def stop(self) -> None:
        self._stop.set()
        if self._sup:
            self._sup.join(timeout=5)
        with self._lock:
            for p in self.procs:
                if p:
                    p.stop()

    def __enter__(self) -> "ReplicaSet":
        try:
            return self.start()
        except BaseException:  # a failed or interrupted start leaves no replica behind
            self.stop()
            raise

    def __exit__(self, *exc) -> None:
        self.stop()


class RRProxy:
    """`hola_rrproxy`: L4 round-robin over healthy backends (health = GET /api/health)."""

    def __init__(self, backends: list[tuple[str, int]], port: int = 0, threads: int = 1,
                 cpu_list: str | None = None, health_ms: int = 200, busy_poll_us: int = 0,
                 exe: str | None = None, host: str = "127.0.0.1", idle_timeout_ms: int | None = None,
                 backend_cpus: list[list[int]] | None = None):
        """`backend_cpus[i]`: the CPUs backend i's workers run on (topology hints: each proxy
        thread then prefers the backends in its own L3)."""
        self._tmp = tempfile.TemporaryDirectory(prefix="rrproxy-")
        self.port_file = os.path.join(self._tmp.name, "port")
        hints = [("@" + ";".join(map(str, c)) if c else "") for c in (backend_cpus or [[]] * len(backends))]
        cmd = [exe or str(binary("hola_rrproxy")), "--host", host, "--port", str(port),
               "--threads", str(threads),
               "--backends", ",".join(f"{h}:{p}{hint}" for (h, p), hint in zip(backends, hints)),
               "--health-ms", str(health_ms), "--port-file", self.port_file]
        if cpu_list:
            cmd += ["--cpu-list", cpu_list]
        if busy_poll_us:
            cmd += ["--busy-poll-us", str(busy_poll_us)]
        if idle_timeout_ms is not None:
            cmd += ["--idle-timeout-ms", str(idle_timeout_ms)]
        self.cmd = cmd
        self.proc: subprocess.Popen | None = None
        self.port = port
        self.log_path = os.path.join(self._tmp.name, "stderr.log")

    def start(self, timeout: float = 10.0) -> "RRProxy":
        self._log = open(self.log_path, "wb")
        self.proc = subprocess.Popen(self.cmd, stdout=subprocess.DEVNULL, stderr=self._log)
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            if self.proc.poll() is not None:
                raise RuntimeError(f"rrproxy exited: {self.log()}")
            if os.path.exists(self.port_file):
                self.port = int(Path(self.port_file).read_text())
                return self
            time.sleep(0.01)
        raise RuntimeError("rrproxy did not start")

    def log(self) -> str:
        try:
            return Path(self.log_path).read_text(errors="replace")
        except OSError:
            return ""

    def stop(self) -> None:
        if self.proc and self.proc.poll() is None:
            self.proc.send_signal(signal.SIGTERM)
            try:
                self.proc.wait(timeout=10)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()
        try:
            self._log.close()
        except Exception:
            pass

    def __enter__(self) -> "RRProxy":
        try:
            return self.start()
        except BaseException:
            self.stop()
            self._tmp.cleanup()
            raise

    def __exit__(self, *exc) -> None:
        self.stop()
        self._tmp.cleanup()
