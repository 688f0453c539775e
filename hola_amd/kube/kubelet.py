"""Pods on one node: what the kubelet does for the hola container, as host processes.

A pod is one `hola` process started from the image's ENTRYPOINT with the container's env
(`HOSTNAME` from `fieldRef: metadata.name`, as `deploy/openshift/hola-dc.yaml:78-81` asks),
its args, and its own pod IP on the loopback network (127.a.b.n: every pod binds :8080 on its
own address, the part of a network namespace the service contract needs). Around it:

* volumes: ConfigMaps are projected the way the kubelet's atomic writer does it: the files
  live in a `..<timestamp>` directory, `..data` links to it, and each key is a link through
  `..data`; an update writes a new directory and swaps `..data` with one rename (the case
  hola's parent-directory watcher exists for);
* the readiness probe with its real parameters (`initialDelaySeconds`, `periodSeconds`,
  `timeoutSeconds`, `successThreshold`, `failureThreshold`; k8s defaults where the manifest
  has none), run off the control loop in a small thread pool;
* restartPolicy Always with CrashLoopBackOff (immediate first restart, then 10 s doubling to
  300 s, reset after 10 min of running);
* termination: the pod leaves the Service endpoints at once, its preStop hook (if any) runs,
  then SIGTERM, and SIGKILL once `terminationGracePeriodSeconds` (30 s) have passed;
* resources: under the static CPU manager policy a Guaranteed pod with integer CPUs gets an
  exclusive cpuset (its process affinity); everything else runs on the shared pool. A memory
  limit is enforced the way the cgroup OOM killer would: resident memory above it gets the
  container SIGKILLed (OOMKilled) and restarted. A CPU limit is CFS bandwidth control from
  user space (`CpuBandwidth`): limits.cpu x 100 ms of CPU time per 100 ms period, the
  container stopped (SIGSTOP) for the rest of a period once it has used that, and continued
  at the next; the container sees its quota as `HOLA_CGROUP_CPU_MAX` (cpu.max's format), as
  it would see its cgroup's cpu.max, which the executor cannot write without root.

Delays (probe delay and period, restart back-off, ConfigMap sync) are multiplied by the
cluster's `time_scale` so tests can run the same state machine faster; deadlines
(probe timeout, grace period) are not.
"""
from __future__ import annotations

import ctypes
import http.client
import os
import re
import shutil
import signal
import subprocess
import threading
import time
from concurrent.futures import Future, ThreadPoolExecutor
from dataclasses import dataclass, field
from pathlib import Path

from hola_amd.kube import manifests as m

PROBE_DEFAULTS = {"initialDelaySeconds": 0, "periodSeconds": 10, "timeoutSeconds": 1, "successThreshold": 1,
                  "failureThreshold": 3}
BACKOFF_INITIAL_S, BACKOFF_MAX_S, BACKOFF_RESET_S = 10.0, 300.0, 600.0
DEFAULT_GRACE_S = 30.0
MEM_CHECK_S = 0.2
CFS_PERIOD_S = 0.1  # cpu.cfs_period_us's default
CFS_POLL_S = 0.005
_CLK_TCK = os.sysconf("SC_CLK_TCK")
KILL_CAPTURE_S = 6.0  # the grace-expiry capture's limit (hola_fpstack gets 5 s) before a plain SIGKILL
# resolved in the parent: a forked child of this multi-threaded process only calls it
_PRCTL = ctypes.CDLL(None, use_errno=True).prctl


def project_configmap(vol_dir: Path, data: dict[str, str], items: list[dict] | None = None) -> None:
    """Writes (or updates) a ConfigMap volume with the kubelet's layout and atomic swap."""
    vol_dir.mkdir(parents=True, exist_ok=True)
    files = {it["path"]: data[it["key"]] for it in items if it.get("key") in data} if items else dict(data)
    ts = time.strftime("..%Y_%m_%d_%H_%M_%S", time.gmtime()) + f".{time.time_ns() % 10**9:09d}"
    new = vol_dir / ts
    new.mkdir()
    for rel, content in files.items():
        p = new / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(content)
    old = os.readlink(vol_dir / "..data") if (vol_dir / "..data").is_symlink() else None
    tmp = vol_dir / "..data_tmp"
    if tmp.is_symlink():
        tmp.unlink()
    tmp.symlink_to(ts)
    os.rename(tmp, vol_dir / "..data")  # the one atomic step readers can observe
    for rel in {r.split("/")[0] for r in files}:
        link = vol_dir / rel
        if not link.is_symlink():
            link.symlink_to(Path("..data") / rel)
    for entry in vol_dir.iterdir():  # keys that disappeared
        if entry.is_symlink() and not entry.name.startswith("..") and entry.name not in {r.split("/")[0] for r in files}:
            entry.unlink()
    if old and old != ts:
        shutil.rmtree(vol_dir / old, ignore_errors=True)


def http_probe(host: str, port: int, path: str, timeout_s: float, headers: dict | None = None) -> tuple[bool, str]:
    """kubelet httpGet: success is a status in [200, 400)."""
    try:
        conn = http.client.HTTPConnection(host, port, timeout=timeout_s)
        try:
            conn.request("GET", path, headers={"User-Agent": "kube-probe/1.29", **(headers or {})})
            r = conn.getresponse()
            r.read()
            return 200 <= r.status < 400, f"HTTP {r.status}"
        finally:
            conn.close()
    except OSError as e:
        return False, f"{type(e).__name__}: {e}"


@dataclass
class Pod:
    name: str
    owner: str  # ReplicationController / ReplicaSet name
    revision: int
    template: dict
    ip: str
    dir: Path
    labels: dict = field(default_factory=dict)
    cpus: list[int] | None = None  # exclusive cpuset (static CPU manager) or None (shared pool)
    cpu_request: float = 0.0
    mem_limit: int = 0  # bytes; 0 = none
    cfs: dict = field(default_factory=dict)  # CPU bandwidth control counters (CpuBandwidth)
    rss_peak: int = 0
    next_mem_check: float = 0.0
    created: float = field(default_factory=time.monotonic)
    scheduled: bool = False
    pending_reason: str = ""
    # container state
    proc: subprocess.Popen | None = None
    started_at: float = 0.0
    restarts: int = 0
    next_start_at: float = 0.0
    backoff_s: float = 0.0
    last_exit: int | None = None
    # readiness
    ready: bool = False
    ready_since: float = 0.0
    probe_ok: int = 0
    probe_fail: int = 0
    next_probe_at: float = 0.0
    probe_future: Future | None = None
    last_probe: str = ""
    # termination
    terminating: bool = False
    deletion_at: float = 0.0
    grace_deadline: float = 0.0
    prestop: subprocess.Popen | None = None
    prestop_http: Future | None = None
    term_sent: bool = False
    kill_sent: bool = False
    kill_future: Future | None = None  # grace-expiry capture + SIGKILL, in the diagnostics thread
    prestop_cmd: list[str] | None = None  # an exec preStop hook the control loop starts next tick
    gone: bool = False

    @property
    def container(self) -> dict:
        return self.template["spec"]["containers"][0]

    @property
    def running(self) -> bool:
        return self.proc is not None and self.proc.poll() is None

    @property
    def log_path(self) -> Path:
        return self.dir / "container.log"

    def status(self) -> str:
        if self.terminating:
            return "Terminating"
        if not self.scheduled:
            return "Pending"
        if self.running:
            return "Running"
        if self.last_exit is not None and self.restarts and self.backoff_s >= BACKOFF_INITIAL_S:
            return "CrashLoopBackOff"
        return "ContainerCreating" if self.proc is None else "Error"

    def summary(self) -> dict:
        return {"name": self.name, "ip": self.ip, "status": self.status(), "ready": self.ready,
                "restarts": self.restarts, "revision": self.revision, "owner": self.owner,
                "cpus": self.cpus, "pid": self.proc.pid if self.running else None,
                "rss_peak_mb": round(self.rss_peak / 2**20, 1),
                "cpu_throttle": {k: (round(v, 3) if isinstance(v, float) else v) for k, v in self.cfs.items()},
                "last_probe": self.last_probe, "pending_reason": self.pending_reason}


def _proc_cpu_s(pid: int) -> float | None:
    """User + system CPU time of a process (all its threads), from /proc/PID/stat."""
    try:
        f = Path(f"/proc/{pid}/stat").read_text().rsplit(")", 1)[1].split()
        return (int(f[11]) + int(f[12])) / _CLK_TCK  # utime, stime (fields 14 and 15)
    except (OSError, IndexError, ValueError):
        return None


def _proc_rss(pid: int) -> int | None:
    """Resident memory of a process in bytes, from /proc/PID/status."""
    try:
        status = Path(f"/proc/{pid}/status").read_text()
        return int(next(ln for ln in status.splitlines() if ln.startswith("VmRSS:")).split()[1]) * 1024
    except (OSError, StopIteration, ValueError):
        return None


@dataclass
class _Bandwidth:
    pod: Pod
    proc: subprocess.Popen
    quota_s: float  # CPU seconds per period
    period: int = -1
    base_s: float = 0.0  # the container's CPU time when the period began
    stopped: bool = False
    stopped_at: float = 0.0


class CpuBandwidth:
    """CFS bandwidth control for containers with limits.cpu, from user space: every 100 ms
    period a container may use limits.cpu x 100 ms of CPU time; once it has, its process group
    is stopped (SIGSTOP) until the period ends and continued (SIGCONT) at the next, which is
    what the kernel's throttling does to a cgroup over its cpu.max. Usage is read from /proc
    every 5 ms at the kernel's accounting granularity (USER_HZ, 10 ms), so a period can run
    over by a poll and a tick. Each pod's `cfs` counts periods, throttled periods and the time
    spent stopped (cpu.stat's nr_periods, nr_throttled, throttled_usec)."""

    def __init__(self):
        self._lock = threading.Lock()
        self._groups: dict[str, _Bandwidth] = {}
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="kube-cfs", daemon=True)
        self._thread.start()

    def add(self, pod: Pod, proc: subprocess.Popen, cpus: float) -> None:
        with self._lock:
            old = self._groups.pop(pod.name, None)
            if old is not None:
                self._resume(old)
            if not pod.cfs:  # the counters span the pod's restarts, as a cgroup's cpu.stat does
                pod.cfs = {"quota_cpus": cpus, "nr_periods": 0, "nr_throttled": 0, "throttled_s": 0.0}
            self._groups[pod.name] = _Bandwidth(pod, proc, cpus * CFS_PERIOD_S)

    def remove(self, pod_name: str) -> None:
        with self._lock:
            g = self._groups.pop(pod_name, None)
            if g is not None:
                self._resume(g)

    def close(self) -> None:
        self._stop.set()
        self._thread.join(timeout=2)
        with self._lock:
            for g in self._groups.values():
                self._resume(g)
            self._groups.clear()

    @staticmethod
    def _signal(g: _Bandwidth, sig: int) -> None:
        if g.proc.poll() is None:  # never a reaped pid (it could be another process's by now)
            try:
                os.killpg(g.proc.pid, sig)  # the container's session: its pid is the group
            except (ProcessLookupError, PermissionError):
                pass

    def _resume(self, g: _Bandwidth) -> None:
        if g.stopped:
            self._signal(g, signal.SIGCONT)
            g.stopped = False
            g.pod.cfs["throttled_s"] += time.monotonic() - g.stopped_at

    def _run(self) -> None:
        t0 = time.monotonic()
        while not self._stop.wait(CFS_POLL_S):
            try:
                self._pass(int((time.monotonic() - t0) / CFS_PERIOD_S))
            except Exception:  # noqa: BLE001 - the controller must outlive one bad pass
                pass

    def _pass(self, k: int) -> None:
        """One poll: `k` is the current period's index."""
        now = time.monotonic()
        with self._lock:
            for name, g in list(self._groups.items()):
                if g.proc.poll() is not None:
                    del self._groups[name]
                    continue
                cpu = _proc_cpu_s(g.proc.pid)
                if cpu is None:
                    continue
                if k != g.period:  # a new period: the quota refills
                    self._resume(g)
                    g.period, g.base_s = k, cpu
                    g.pod.cfs["nr_periods"] += 1
                elif not g.stopped and cpu - g.base_s >= g.quota_s:
                    self._signal(g, signal.SIGSTOP)
                    g.stopped, g.stopped_at = True, now
                    g.pod.cfs["nr_throttled"] += 1


class Kubelet:
    """Runs the pods' containers, probes, volumes and terminations; driven by ticks from the
    cluster's control loop (every state change happens on that thread)."""

    def __init__(self, cluster, probe_workers: int = 16):
        self.cluster = cluster
        self.cfs = CpuBandwidth()
        self.pool = ThreadPoolExecutor(max_workers=probe_workers, thread_name_prefix="kube-probe")
        # grace-expiry captures + SIGKILLs, off the control loop and off the probes' pool
        self.diag = ThreadPoolExecutor(max_workers=4, thread_name_prefix="kube-diag")

    # ------------------------------------------------------------------ container start
    def _probe_spec(self, pod: Pod) -> dict | None:
        rp = pod.container.get("readinessProbe")
        if not rp:
            return None
        return {**PROBE_DEFAULTS, **rp}

    @staticmethod
    def cpu_limit(pod: Pod) -> float:
        """limits.cpu of the container in cores (0 = none)."""
        return m.parse_cpu(((pod.container.get("resources") or {}).get("limits") or {}).get("cpu"))

    def _env(self, pod: Pod) -> dict[str, str]:
        c = self.cluster
        env = {"PATH": os.environ.get("PATH", "/usr/bin:/bin"), "HOME": str(pod.dir)}
        limit = self.cpu_limit(pod)
        if limit > 0:  # the cgroup's cpu.max as the container would read it
            env["HOLA_CGROUP_CPU_MAX"] = f"{int(round(limit * CFS_PERIOD_S * 1e6))} {int(CFS_PERIOD_S * 1e6)}"
        for k in ("LANG", "LC_ALL", "TMPDIR", "LD_LIBRARY_PATH", "SSL_CERT_FILE", "SSL_CERT_DIR"):
            if k in os.environ:
                env[k] = os.environ[k]
        env.update(c.image.env)
        # Service links the kubelet injects (<NAME>_SERVICE_HOST/_PORT) for the cluster's Services
        for svc, (host, port) in c.service_addresses().items():
            key = re.sub(r"[^A-Z0-9]", "_", svc.upper())
            env[f"{key}_SERVICE_HOST"] = host
            env[f"{key}_SERVICE_PORT"] = str(port)
        for e in pod.container.get("env") or []:
            name = e["name"]
            if "value" in e:
                env[name] = _expand(str(e["value"]), env)
            elif "valueFrom" in e:
                vf = e["valueFrom"]
                if "fieldRef" in vf:
                    fp = vf["fieldRef"]["fieldPath"]
                    env[name] = {"metadata.name": pod.name, "metadata.namespace": c.namespace,
                                 "status.podIP": pod.ip, "spec.nodeName": c.node_name}.get(fp, "")
                elif "configMapKeyRef" in vf:
                    ref = vf["configMapKeyRef"]
                    env[name] = c.configmaps.get(ref["name"], {}).get(ref["key"], "")
        # cluster DNS: a URL naming a Service of this cluster reaches that Service's address
        return {k: c.rewrite_service_urls(self.map_paths(pod, v)) for k, v in env.items()}

    def map_paths(self, pod: Pod, value: str) -> str:
        """Container paths inside a value (whitespace-separated tokens: `/x`, `-Dk=/x`,
        `--f=/x`) resolved to the host files that back them: a volume mount first, then the
        image's root filesystem."""
        def one(tok: str) -> str:
            m = re.match(r"^((?:-D[^=]+=)|(?:--[^=]+=))?(/.*)$", tok)
            if not m:
                return tok
            host = self.host_path(pod, m.group(2))
            return (m.group(1) or "") + host if host else tok
        return " ".join(one(t) for t in value.split(" "))

    def host_path(self, pod: Pod, cpath: str) -> str | None:
        best = None
        for vm in pod.container.get("volumeMounts") or []:
            mp = vm["mountPath"].rstrip("/")
            if cpath == mp or cpath.startswith(mp + "/"):
                if best is None or len(mp) > len(best[0]):
                    best = (mp, pod.dir / "volumes" / vm["name"])
        if best:
            return str(best[1]) + cpath[len(best[0]):]
        root = pod.dir.parent.parent / "rootfs"
        norm = os.path.normpath(cpath)
        if norm in self.cluster.image.files or any(f.startswith(norm + "/") for f in self.cluster.image.files):
            return str(root) + norm
        return None

    def _argv(self, pod: Pod) -> list[str]:
        c, img = pod.container, self.cluster.image
        if c.get("command"):
            argv = list(c["command"]) + list(c.get("args") or [])
        else:
            argv = list(img.entrypoint) + list(c.get("args") if c.get("args") is not None else img.cmd)
        argv = [self.map_paths(pod, a) for a in argv]
        # the pod's own network namespace, reduced to what the contract needs: its address
        return argv + ["--host", pod.ip]

    def setup_volumes(self, pod: Pod) -> None:
        for v in pod.template["spec"].get("volumes") or []:
            d = pod.dir / "volumes" / v["name"]
            if "configMap" in v:
                cm = v["configMap"]
                project_configmap(d, self.cluster.configmaps.get(cm["name"], {}), cm.get("items"))
            else:  # emptyDir and anything else: a plain directory
                d.mkdir(parents=True, exist_ok=True)

    def start_container(self, pod: Pod, now: float) -> None:
        pod.dir.mkdir(parents=True, exist_ok=True)
        if pod.proc is None and pod.restarts == 0:
            self.setup_volumes(pod)
        argv, env = self._argv(pod), self._env(pod)
        workdir = self.host_path(pod, self.cluster.image.workdir) or str(pod.dir)
        if not os.path.isdir(workdir):
            workdir = str(pod.dir)
        cpus = pod.cpus if pod.cpus is not None else self.cluster.shared_pool()
        log = open(pod.log_path, "ab")
        log.write(f"--- start {time.strftime('%H:%M:%S')} restart={pod.restarts} argv={argv}\n".encode())
        log.flush()
        try:
            pod.proc = subprocess.Popen(argv, env=env, cwd=workdir, stdout=log, stderr=log,
                                        preexec_fn=lambda: die_with_parent(cpus), start_new_session=True)
        except OSError as e:
            # CreateContainerError / RunContainerError: retried with the restart back-off
            log.write(f"--- cannot start the container: {e}\n".encode())
            log.close()
            pod.proc = subprocess.Popen(["/bin/false"])  # an exited container, for the back-off
            pod.proc.wait()
            pod.started_at = now
            self.cluster.event(pod.name, "Failed", f"cannot start the container: {e}")
            return
        log.close()
        limit = self.cpu_limit(pod)
        # an exclusive cpuset no larger than the quota cannot exceed it: nothing to enforce
        if limit > 0 and not (pod.cpus and len(pod.cpus) <= limit):
            self.cfs.add(pod, pod.proc, limit)
        pod.started_at = now
        pod.next_mem_check = now + 0.05  # a container over its limit from the start dies before probing
        pod.ready = False
        pod.probe_ok = pod.probe_fail = 0
        # a probe still in flight was sent to the container that died: its answer (possibly from
        # this new container, on the same address) must not count, or a restarted container
        # turns Ready before its initialDelaySeconds, as no kubelet lets it (the probe worker
        # belongs to the container)
        pod.probe_future = None
        ps = self._probe_spec(pod)
        pod.next_probe_at = now + (ps["initialDelaySeconds"] * self.cluster.time_scale if ps else 0.0)
        self.cluster.event(pod.name, "Started", f"pid {pod.proc.pid} on {pod.ip}, cpus {cpus}")

    # ------------------------------------------------------------------ the tick
    def tick(self, pod: Pod, now: float) -> None:
        if pod.gone or not pod.scheduled:
            return
        ts = self.cluster.time_scale
        if pod.terminating:
            self._tick_terminating(pod, now)
            return
        if pod.proc is not None and pod.proc.poll() is not None and pod.last_exit is None:
            # the container died: NotReady at once, restart with back-off
            pod.last_exit = pod.proc.returncode
            pod.ready = False
            ran = now - pod.started_at
            if ran >= BACKOFF_RESET_S * ts:
                pod.backoff_s = 0.0
            delay = pod.backoff_s
            pod.backoff_s = BACKOFF_INITIAL_S if pod.backoff_s == 0 else min(BACKOFF_MAX_S, pod.backoff_s * 2)
            pod.next_start_at = now + delay * ts
            self.cluster.event(pod.name, "BackOff" if delay else "Died",
                               f"container exited {pod.last_exit}; restart in {delay * ts:.1f}s")
        if pod.proc is None or (pod.last_exit is not None and now >= pod.next_start_at):
            if pod.proc is not None:
                pod.restarts += 1
            pod.last_exit = None
            self.start_container(pod, now)
            return
        if pod.last_exit is not None or not pod.running:
            return
        if now >= pod.next_mem_check:
            self._check_memory(pod, now)
            if not pod.running:
                return
        self._tick_probe(pod, now)

    def _check_memory(self, pod: Pod, now: float) -> None:
        """limits.memory, as the cgroup's OOM killer applies it: a container whose resident
        memory exceeds the limit is SIGKILLed (reason OOMKilled) and restarted with back-off.
        Sampled every 0.2 s from /proc (the executor cannot write cgroup limits)."""
        pod.next_mem_check = now + MEM_CHECK_S
        limit = pod.mem_limit
        if limit <= 0:
            return
        rss = _proc_rss(pod.proc.pid)
        if rss is None:
            return
        pod.rss_peak = max(pod.rss_peak, rss)
        if rss > limit:
            pod.proc.kill()
            pod.proc.wait()
            self.cluster.event(pod.name, "OOMKilled", f"resident {rss >> 20} MiB > limit {limit >> 20} MiB")

    def _tick_probe(self, pod: Pod, now: float) -> None:
        ps = self._probe_spec(pod)
        if ps is None:
            if not pod.ready:
                pod.ready, pod.ready_since = True, now
            return
        f = pod.probe_future
        if f is not None:
            if not f.done():
                return
            pod.probe_future = None
            ok, detail = f.result()
            pod.last_probe = detail
            if ok:
                pod.probe_ok += 1
                pod.probe_fail = 0
                if not pod.ready and pod.probe_ok >= int(ps["successThreshold"]):
                    pod.ready, pod.ready_since = True, now
                    self.cluster.event(pod.name, "Ready", detail)
            else:
                pod.probe_fail += 1
                pod.probe_ok = 0
                if pod.ready and pod.probe_fail >= int(ps["failureThreshold"]):
                    pod.ready = False
                    self.cluster.event(pod.name, "Unhealthy", f"Readiness probe failed: {detail}")
        if now >= pod.next_probe_at:
            hg = ps.get("httpGet") or {}
            port = _port_number(pod.container, hg.get("port", 8080))
            headers = {h["name"]: h["value"] for h in hg.get("httpHeaders") or []}
            pod.probe_future = self.pool.submit(http_probe, pod.ip, port, hg.get("path", "/"),
                                                float(ps["timeoutSeconds"]), headers)
            pod.next_probe_at = now + float(ps["periodSeconds"]) * self.cluster.time_scale

    # ------------------------------------------------------------------ termination
    def begin_delete(self, pod: Pod, now: float, grace_s: float | None = None) -> None:
        if pod.terminating:
            return
        pod.terminating = True
        pod.ready = False
        pod.deletion_at = now
        spec_grace = pod.template["spec"].get("terminationGracePeriodSeconds", DEFAULT_GRACE_S)
        pod.grace_deadline = now + float(spec_grace if grace_s is None else grace_s)
        pre = ((pod.container.get("lifecycle") or {}).get("preStop") or {})
        if pod.running and "exec" in pre:
            # Started by the control loop's next tick (_tick_terminating), not here: begin_delete
            # also runs on `oc` request threads, and a process started there would get its
            # parent-death signal when that thread ends (die_with_parent).
            pod.prestop_cmd = [self.map_paths(pod, a) for a in pre["exec"]["command"]]
        elif pod.running and "httpGet" in pre:  # off the control loop, like the probes
            hg = pre["httpGet"]
            pod.prestop_http = self.pool.submit(http_probe, pod.ip, _port_number(pod.container, hg.get("port", 8080)),
                                                hg.get("path", "/"), float(pod.grace_deadline - now))
        self.cluster.event(pod.name, "Killing", f"grace {pod.grace_deadline - now:.0f}s")

    def _tick_terminating(self, pod: Pod, now: float) -> None:
        kf = pod.kill_future
        if kf is not None:
            if not kf.done():
                if now >= pod.grace_deadline + KILL_CAPTURE_S:  # the capture is stuck: kill anyway
                    pod.proc.kill()
                if pod.running or now < pod.grace_deadline + KILL_CAPTURE_S:
                    return  # "Killed" comes before "Deleted"
                note = "capture did not finish"
            else:
                try:
                    note = kf.result()
                except Exception as e:  # noqa: BLE001 - a diagnostic; the SIGKILL was sent (finally)
                    note = f"capture failed: {e!r}"
            pod.kill_future = None
            self.cluster.event(pod.name, "Killed", f"grace period expired: SIGKILL ({note})")
        if not pod.running:
            pod.gone = True
            if pod.prestop and pod.prestop.poll() is None:
                pod.prestop.kill()
            self.cluster.event(pod.name, "Deleted",
                               f"exit {pod.proc.returncode if pod.proc else None} after {now - pod.deletion_at:.2f}s")
            return
        if pod.prestop_cmd is not None:
            cmd, pod.prestop_cmd = pod.prestop_cmd, None
            pod.prestop = subprocess.Popen(cmd, env=self._env(pod), stdout=subprocess.DEVNULL,
                                           stderr=subprocess.DEVNULL, start_new_session=True,
                                           preexec_fn=die_with_parent)
        hook_done = (pod.prestop is None or pod.prestop.poll() is not None) and \
            (pod.prestop_http is None or pod.prestop_http.done())
        if not pod.term_sent and (hook_done or now >= pod.grace_deadline):
            pod.proc.send_signal(signal.SIGTERM)
            pod.term_sent = True
        if now >= pod.grace_deadline and not pod.kill_sent:
            # What it was doing when the grace ran out (thread states, user-space stacks), then
            # the SIGKILL: in the diagnostics thread, so a slow capture (ptrace of every thread)
            # never holds the control loop, whose other pods' probes, endpoint syncs and rollout
            # steps go on meanwhile. The next ticks see the exit.
            pod.kill_sent = True
            pod.kill_future = self.diag.submit(self.capture_and_kill, pod.proc, pod.dir / "fpstack.txt")

    def capture_and_kill(self, proc: subprocess.Popen, stacks_out: Path) -> str:
        """Diagnostics thread: thread states and stacks of a container whose grace period ran
        out, then its SIGKILL; returns the note for the `Killed` event."""
        try:
            threads = _thread_states(proc.pid)
            stacks = _fpstack(proc.pid, stacks_out)
        finally:
            proc.kill()
        return f"threads: {threads}{stacks}"

    def kill_container(self, pod: Pod, sig: int = signal.SIGKILL) -> None:
        if pod.running:
            pod.proc.send_signal(sig)

    def shutdown(self) -> None:
        self.cfs.close()
        self.pool.shutdown(wait=False, cancel_futures=True)
        self.diag.shutdown(wait=False, cancel_futures=True)


def die_with_parent(cpus: list[int] | None = None) -> None:
    """preexec_fn of every process the executor starts: the kernel SIGKILLs it when the thread
    that started it ends (the control loop, which starts every pod, hook and Service process), so an executor that dies, or a test process cut
    off before its teardown, leaves no pods behind (a pod keeps its own session, so a signal to
    the executor's process group would not reach it). Optionally applies the cpuset."""
    _PRCTL(1, int(signal.SIGKILL), 0, 0, 0)  # PR_SET_PDEATHSIG
    if cpus:
        os.sched_setaffinity(0, cpus)


def _thread_states(pid: int) -> str:
    """`name:state:wchan` of each thread of a process, from /proc (the kernel's view of where a
    container that outlived its grace period was waiting)."""
    out = []
    try:
        tasks = sorted(os.listdir(f"/proc/{pid}/task"), key=int)
    except OSError:
        return "?"
    for t in tasks:
        base = f"/proc/{pid}/task/{t}"
        try:
            with open(f"{base}/stat") as f:
                stat = f.read()
            with open(f"{base}/wchan") as f:
                wchan = f.read().strip() or "-"
        except OSError:
            continue
        name = stat[stat.index("(") + 1:stat.rindex(")")]
        state = stat[stat.rindex(")") + 2:].split(" ", 1)[0]
        out.append(f"{name}:{state}:{wchan}")
    return " ".join(out) or "?"


def _fpstack(pid: int, out: Path) -> str:
    """User-space stacks of every thread (`hola_fpstack`, a frame-pointer walk under ptrace)
    written to `out`; returns a note for the event, or "" when the tool is not built."""
    from hola_amd import native

    try:
        exe = native.binary("hola_fpstack", build_if_missing=False)
    except Exception:  # noqa: BLE001 - a diagnostic only
        return ""
    if not exe.exists():
        return ""
    try:
        r = subprocess.run([str(exe), str(pid)], capture_output=True, text=True, timeout=5)
        out.write_text(r.stdout + r.stderr)
    except (OSError, subprocess.SubprocessError):
        return ""
    return f"; stacks in {out}"


def _port_number(container: dict, port) -> int:
    if isinstance(port, int) or str(port).isdigit():
        return int(port)
    for p in container.get("ports") or []:
        if p.get("name") == port:
            return int(p["containerPort"])
    raise ValueError(f"unknown named port {port!r}")


def _expand(value: str, env: dict[str, str]) -> str:
    """$(VAR) references to earlier variables, as the kubelet expands them ($$ escapes)."""
    return re.sub(r"\$\$|\$\(([A-Za-z_][A-Za-z0-9_]*)\)",
                  lambda m: "$" if m.group(0) == "$$" else env.get(m.group(1), m.group(0)), value)
