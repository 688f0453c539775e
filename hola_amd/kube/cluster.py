"""A one-node cluster that executes `deploy/openshift/*.yaml` (BASELINE config 5).

`Cluster` plays the control plane, the kubelet and kube-proxy for the objects the
reference's `mvn fabric8:json fabric8:apply` created (`/root/reference/pom.xml:65-94`,
`/root/reference/Readme.md:18-24`), without a container runtime or root:

* **workload**: a DeploymentConfig (`oc` era, hola-dc.yaml) or an apps/v1 Deployment
  (hola.yaml). Each template revision is a ReplicationController `hola-<n>` (pods
  `hola-<n>-<5 chars>`) or a ReplicaSet `hola-<template hash>`; `scale`, `set_env` and
  `patch` behave like `oc scale`, `oc set env` / `oc env` and `oc patch`: a template change
  is a ConfigChange trigger, i.e. a new revision rolled out with the Rolling strategy's
  maxSurge / maxUnavailable (25 % / 25 % by default);
* **pods** (`kubelet.Kubelet`): one `hola` process each, from the image's ENTRYPOINT with
  the container's env (HOSTNAME = pod name), on its own loopback pod IP, readiness-probed
  with the manifest's parameters, restarted with back-off, terminated with SIGTERM and a
  grace period;
* **scheduling**: CPU requests are checked against the node's allocatable CPUs (pods that do
  not fit stay Pending); under `cpu_manager_policy="static"` a Guaranteed pod with integer
  CPUs gets an exclusive cpuset;
* **Service**: `hola_rrproxy` on the Service's port in Endpoints mode: its backend set is
  exactly the Ready, non-terminating pods the selector matches, as the endpoints controller
  publishes them, applied `endpoint_sync_s` after each change (kube-proxy's sync delay). A
  connection to an endpoint that stopped listening fails as it does through kube-proxy's DNAT
  (no failover). That is kube-proxy's old userspace mode, one proxy hop per request. The
  iptables/IPVS modes DNAT each new connection in the client's kernel instead: a client that
  reads `endpoints_file()` at connect time (`hola_loadgen --endpoints-file`) gets exactly that,
  with no hop;
* **ConfigMaps**: projected into every pod that mounts one, updated `configmap_sync_s` after an
  edit through the kubelet's `..data` symlink swap;
* **cluster DNS**: a URL in a pod's env or args naming a Service of this cluster (`aloha`,
  `zipkin-query`) is pointed at that Service's address. With `zipkin=True` a native discard
  collector (`hola_zipkin_sink`) stands in for `zipkin-query:9411`, so the image's
  `ZIPKIN_SERVER_URL` (Dockerfile) has a collector as in the demo.

Everything runs on one control-loop thread (`_loop`); the public methods take the same lock.
"""
from __future__ import annotations

import collections
import copy
import os
import random
import signal
import string
import subprocess
import tempfile
import threading
import time
from pathlib import Path

from hola_amd import native
from hola_amd.utils.cpu import cpu_budget
from hola_amd.kube import manifests as m
from hola_amd.kube.image import Image
from hola_amd.kube.kubelet import Kubelet, Pod, die_with_parent, project_configmap

TICK_S = 0.02


def _listening_127_nets() -> set[int]:
    """The second octets of 127.<a>.x.x addresses with a listening TCP socket on this host
    (/proc/net/tcp, state 0A): /16s that a new cluster must not claim."""
    out: set[int] = set()
    try:
        lines = Path("/proc/net/tcp").read_text().splitlines()[1:]
    except OSError:
        return out
    for ln in lines:
        f = ln.split()
        if len(f) > 3 and f[3] == "0A":
            ip_hex = f[1].split(":")[0]
            b = bytes.fromhex(ip_hex)[::-1]  # little-endian on x86
            if b[0] == 127:
                out.add(b[1])
    return out


class ClusterError(RuntimeError):
    pass


class ReplicationController:
    """One template revision of the workload (RC for a DeploymentConfig, RS for a Deployment)."""

    def __init__(self, name: str, revision: int, template: dict, replicas: int = 0):
        self.name, self.revision, self.template, self.replicas = name, revision, template, replicas


class Cluster:
    def __init__(self, files: list[str | Path], patches: list[str | Path] = (), state_dir: str | Path | None = None,
                 replicas: int | None = None, node_cpus: float | None = None, reserved_cpus: int = 1,
                 cpu_manager_policy: str = "none", time_scale: float = 1.0, endpoint_sync_s: float = 1.0,
                 configmap_sync_s: float = 60.0, service_host: str = "127.0.0.1", service_port: int | None = None,
                 zipkin: bool = True, proxy_threads: int = 0, proxy_cpus: str | None = None,
                 namespace: str = "myproject", dockerfile: str | Path | None = None):
        if cpu_manager_policy not in ("none", "static"):
            raise ValueError("cpu_manager_policy is 'none' or 'static'")
        self.objects = m.load_objects(files)
        self.patches = [o for p in patches for o in m.load_objects([p])]
        # absolute: pods run with their own working directory
        self.state = Path(state_dir).resolve() if state_dir else Path(tempfile.mkdtemp(prefix="hola-cluster-"))
        self.state.mkdir(parents=True, exist_ok=True)
        self.namespace, self.node_name = namespace, "mi355x-node"
        self.time_scale = float(time_scale)
        self.endpoint_sync_s, self.configmap_sync_s = endpoint_sync_s, configmap_sync_s
        self.policy = cpu_manager_policy
        self.real_cpus = sorted(os.sched_getaffinity(0))
        self.node_cpus = float(node_cpus) if node_cpus else float(len(self.real_cpus))
        self.reserved = list(self.real_cpus[:reserved_cpus]) if reserved_cpus else []
        self.allocatable = self.node_cpus - len(self.reserved)
        # The userspace Service proxy carries every request twice (in and out), so a fixed 2
        # threads capped a rollout under load at ~160 k req/s (profiles/round3/13_kube): by
        # default it gets a quarter of the CPUs this executor may keep busy (its affinity mask
        # within any cgroup quota), 2 to 16 threads.
        self.proxy_threads = proxy_threads or max(2, min(16, cpu_budget() // 4))
        self.proxy_cpus = proxy_cpus
        self.service_host, self.service_port_override = service_host, service_port
        self.want_zipkin = zipkin
        self.image = Image.from_dockerfile(dockerfile) if dockerfile else Image.from_dockerfile()
        self.image.materialize(self.state / "rootfs")
        self.lock = threading.RLock()
        # the latest events (the full stream is in events.log)
        self.events: collections.deque[tuple[float, str, str, str]] = collections.deque(maxlen=20000)
        self._events_f = open(self.state / "events.log", "a")
        self.t0 = time.monotonic()
        # pod network: 127.<a>.0.0/16 per cluster (127.<a>.0.1 = stand-in Services, pods from
        # 127.<a>.0.2 on; .0 and .255 host parts are skipped): room for 65 k pods over the
        # executor's life, so rollouts never exhaust it
        self._net_lock = self._claim_network()
        self.subnet = f"{self.net}.0"
        self._ips = (f"{self.net}.{b}.{c}" for b in range(256) for c in range(1, 255) if (b, c) != (0, 1))
        self.services: dict[str, dict] = {}
        self.configmaps: dict[str, dict[str, str]] = {}
        self.workload: dict | None = None
        for o in self.objects:
            kind, name = o.get("kind"), o.get("metadata", {}).get("name")
            if kind == "Service":
                self.services[name] = o
            elif kind == "ConfigMap":
                self.configmaps[name] = dict(o.get("data") or {})
            elif kind in ("DeploymentConfig", "Deployment"):
                if self.workload is not None:
                    raise ClusterError("one DeploymentConfig or Deployment per cluster (apply hola-dc.yaml or "
                                       "hola.yaml, not both)")
                self.workload = copy.deepcopy(o)
            else:
                self.event(f"{kind}/{name}", "Ignored", "kind not modelled by this executor")
        if self.workload is None:
            raise ClusterError("no DeploymentConfig or Deployment in the manifests")
        for p in self.patches:  # `oc patch dc/hola -p "$(cat translation-patch.yaml)"`
            self.workload = m.strategic_merge(self.workload, p)
        if replicas is not None:
            self.workload["spec"]["replicas"] = int(replicas)
        self.kind = self.workload["kind"]
        self.name = self.workload["metadata"]["name"]
        self.rcs: list[ReplicationController] = []
        self.pods: dict[str, Pod] = {}
        self.kubelet = Kubelet(self)
        self._cm_due: list[tuple[float, str, str]] = []  # (due, pod, configmap)
        self._ep_desired: dict[str, list[str]] = {}
        self._ep_published: dict[str, list[str]] = {}
        self._ep_written: dict[str, tuple[int, list[str]]] = {}  # (generation, endpoints) in the file
        self._ep_pending_since: dict[str, float] = {}
        self.endpoint_history: dict[str, list[tuple[float, list[str]]]] = {}
        self._last_rollout_step = 0.0
        self._completed_rev = 0
        self.proxies: list[subprocess.Popen] = []  # one hola_rrproxy per Service
        self.sink: subprocess.Popen | None = None
        self._logs: list = []  # stderr files of the helper processes
        self.service_ports: dict[str, tuple[str, int]] = {}
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self.ticks = 0  # control-loop passes (a stalled loop shows as a count that stops)

    def _claim_network(self):
        """Takes a free 127.<a>.0.0/16 for this cluster's pods and stand-in Services: every pod
        binds :8080 on its own address, so two clusters on one host (parallel tests, a bench
        next to a test) must never share one. The claim is an flock held for the cluster's
        life, so it also holds across processes, and is released when the process exits."""
        import fcntl

        lock_dir = Path(tempfile.gettempdir()) / "hola-kube-nets"
        lock_dir.mkdir(exist_ok=True)
        busy = _listening_127_nets()
        for a in random.sample(range(100, 250), 150):
            if a in busy:
                # something still listens there without holding the claim: pods of an executor
                # that was SIGKILLed before it could stop them (their parent-death signal goes
                # with the thread that started them), whose addresses would refuse our pods
                continue
            f = open(lock_dir / f"127.{a}.lock", "w")
            try:
                fcntl.flock(f, fcntl.LOCK_EX | fcntl.LOCK_NB)
            except OSError:
                f.close()
                continue
            self.net = f"127.{a}"
            return f
        raise ClusterError("no free 127.x.0.0/16 pod network on this host")

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> "Cluster":
        # Every process the executor starts gets a parent-death signal (kubelet.die_with_parent),
        # which the kernel ties to the *thread* that started it. The Services' proxies and the
        # collector are therefore started by the control-loop thread itself, like the pods, so
        # they live exactly as long as the executor whichever thread calls start().
        started = threading.Event()
        failed: list[BaseException] = []

        def run() -> None:
            try:
                self._start_services()
            except BaseException as e:  # noqa: BLE001 - re-raised in the caller's thread
                failed.append(e)
                self._stop_services()
                started.set()
                return
            started.set()
            self._loop()

        self._thread = threading.Thread(target=run, name="kube-control", daemon=True)
        self._thread.start()
        started.wait()
        if failed:
            self._thread.join()
            self._thread = None
            raise failed[0]
        with self.lock:
            self._new_revision(self.workload["spec"]["template"], initial=True)
        return self

    def close(self, grace_s: float = 10.0) -> None:
        with self.lock:
            now = time.monotonic()
            self.workload["spec"]["replicas"] = 0
            for rc in self.rcs:
                rc.replicas = 0
            for p in self.pods.values():
                if p.scheduled and not p.gone and not p.terminating:
                    self.kubelet.begin_delete(p, now, grace_s=grace_s)
        deadline = time.monotonic() + grace_s + 2
        while time.monotonic() < deadline and any(p.running for p in list(self.pods.values())):
            time.sleep(0.05)
        self._stop.set()
        if self._thread:
            self._thread.join(timeout=5)
        for p in self.pods.values():
            if p.running:
                p.proc.kill()
                p.proc.wait()
        self._stop_services()
        self.kubelet.shutdown()
        self._events_f.close()
        self._net_lock.close()  # releases the pod network

    def _stop_services(self) -> None:
        for proc in [*self.proxies, self.sink]:
            if proc and proc.poll() is None:
                proc.send_signal(signal.SIGTERM)
                try:
                    proc.wait(timeout=5)
                except subprocess.TimeoutExpired:
                    proc.kill()
                    proc.wait()
        for f in self._logs:
            f.close()
        self._logs.clear()

    def __enter__(self) -> "Cluster":
        return self.start()

    def __exit__(self, *exc) -> None:
        self.close()

    # ------------------------------------------------------------------ services
    def _start_services(self) -> None:
        epdir = self.state / "endpoints"
        epdir.mkdir(exist_ok=True)
        if self.want_zipkin:
            ip = f"{self.subnet}.1"
            pf = self.state / "zipkin.port"
            self._logs.append(open(self.state / "zipkin.log", "ab"))
            self.sink = subprocess.Popen([str(native.binary("hola_zipkin_sink")), "--host", ip, "--port", "9411",
                                          "--port-file", str(pf)], stdout=subprocess.DEVNULL, stderr=self._logs[-1],
                                         preexec_fn=die_with_parent)
            self.service_ports["zipkin-query"] = (ip, self._wait_port(pf, self.sink))
        for name, svc in self.services.items():
            port = svc["spec"]["ports"][0]
            bind_port = self.service_port_override if self.service_port_override is not None else int(port["port"])
            ep = epdir / name
            ep.write_text("")
            pf = self.state / f"service-{name}.port"
            cmd = [str(native.binary("hola_rrproxy")), "--host", self.service_host, "--port", str(bind_port),
                   "--endpoints-file", str(ep), "--health-ms", "0", "--no-failover", "--idle-timeout-ms", "0",
                   "--threads", str(self.proxy_threads), "--port-file", str(pf)]
            if self.proxy_cpus:
                cmd += ["--cpu-list", self.proxy_cpus]
            self._logs.append(open(self.state / f"service-{name}.log", "ab"))
            proxy = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=self._logs[-1], preexec_fn=die_with_parent)
            self.proxies.append(proxy)
            self.service_ports[name] = (self.service_host, self._wait_port(pf, proxy))
            self.event(f"service/{name}", "Listening",
                       f"{svc['spec'].get('type', 'ClusterIP')} {self.service_host}:{self.service_ports[name][1]}")

    @staticmethod
    def _wait_port(pf: Path, proc: subprocess.Popen, timeout: float = 10.0) -> int:
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            if proc.poll() is not None:
                raise ClusterError(f"{proc.args[0]} exited {proc.returncode}")
            try:
                return int(pf.read_text().strip())
            except (OSError, ValueError):
                time.sleep(0.01)
        raise ClusterError(f"{proc.args[0]} did not start")

    def service_addresses(self) -> dict[str, tuple[str, int]]:
        return dict(self.service_ports)

    def service_url(self, name: str | None = None) -> str:
        host, port = self.service_ports[name or next(iter(self.services))]
        return f"http://{host}:{port}"

    def endpoints_file(self, name: str | None = None) -> Path:
        """The Service's endpoints as the executor publishes them (`ip:port` per line, replaced
        atomically on each sync): the DNAT table of kube-proxy's iptables/IPVS modes, for a
        client that resolves the Service at connect time (`hola_loadgen --endpoints-file`)
        instead of going through the userspace proxy."""
        return self.state / "endpoints" / (name or next(iter(self.services)))

    def rewrite_service_urls(self, value: str) -> str:
        import re

        def sub(mt):
            host = mt.group(2)
            short = host.split(".")[0]
            if host not in self.service_ports and not (
                    short in self.service_ports and host.endswith((f".{self.namespace}", ".svc", ".svc.cluster.local"))):
                return mt.group(0)
            h, p = self.service_ports[host if host in self.service_ports else short]
            return f"{mt.group(1)}{h}:{p}"
        return re.sub(r"(https?://)([A-Za-z0-9.-]+)(?::\d+)?", sub, value)

    # ------------------------------------------------------------------ events
    def event(self, obj: str, reason: str, msg: str) -> None:
        t = time.monotonic() - self.t0
        self.events.append((t, obj, reason, msg))
        try:
            self._events_f.write(f"{t:9.3f} {obj:<28} {reason:<14} {msg}\n")
            self._events_f.flush()
        except ValueError:
            pass

    # ------------------------------------------------------------------ workload
    @property
    def desired(self) -> int:
        return int(self.workload["spec"].get("replicas", 1))

    def _new_revision(self, template: dict, initial: bool = False) -> ReplicationController:
        rev = (self.rcs[-1].revision + 1) if self.rcs else 1
        if self.kind == "DeploymentConfig":
            name = f"{self.name}-{rev}"
            self.workload.setdefault("status", {})["latestVersion"] = rev
        else:
            name = f"{self.name}-{m.template_hash(template)}"
            existing = next((rc for rc in self.rcs if rc.name == name), None)
            if existing is not None:  # a Deployment rolled back to an earlier template
                self.rcs.remove(existing)
                self.rcs.append(existing)
                return existing
        rc = ReplicationController(name, rev, copy.deepcopy(template), self.desired if initial else 0)
        self.rcs.append(rc)
        self.event(f"rc/{name}", "Created", f"revision {rev}" + (" (initial)" if initial else ": rolling out"))
        return rc

    def _template_changed(self, template: dict) -> None:
        self.workload["spec"]["template"] = template
        if m.template_hash(template) != m.template_hash(self.rcs[-1].template):
            self._new_revision(template)

    def _strategy(self) -> tuple[str, object, object, float]:
        st = self.workload["spec"].get("strategy") or {}
        if self.kind == "DeploymentConfig":
            kind = st.get("type", "Rolling")
            rp = st.get("rollingParams") or {}
            return kind, rp.get("maxSurge", "25%"), rp.get("maxUnavailable", "25%"), float(rp.get("updatePeriodSeconds", 1))
        kind = st.get("type", "RollingUpdate")
        ru = st.get("rollingUpdate") or {}
        return ("Rolling" if kind == "RollingUpdate" else kind), ru.get("maxSurge", "25%"), ru.get("maxUnavailable", "25%"), 0.0

    def _live(self, rc: ReplicationController) -> list[Pod]:
        return [p for p in self.pods.values() if p.owner == rc.name and not p.terminating and not p.gone]

    def _reconcile_rollout(self, now: float) -> None:
        cur, olds = self.rcs[-1], [rc for rc in self.rcs[:-1] if rc.replicas > 0 or self._live(rc)]
        n = self.desired
        if not olds:
            cur.replicas = n
            return
        kind, surge_v, unavail_v, period = self._strategy()
        if kind == "Recreate":
            for rc in olds:
                rc.replicas = 0
            if not any(p.owner != cur.name and not p.gone for p in self.pods.values()):
                cur.replicas = n
            return
        if now - self._last_rollout_step < period * self.time_scale:
            return
        self._last_rollout_step = now
        surge = m.resolve_int_or_percent(surge_v, n, True)
        unavail = m.resolve_int_or_percent(unavail_v, n, False)
        if surge == 0 and unavail == 0:
            unavail = 1
        live_all = [p for rc in self.rcs for p in self._live(rc)]
        # scale the new revision up within the surge budget
        room = n + surge - len(live_all)
        if cur.replicas < n and room > 0:
            cur.replicas += min(n - cur.replicas, room)
        # scale old revisions down, unready pods first, keeping n - maxUnavailable ready
        ready = sum(1 for p in live_all if p.ready)
        removable = ready - (n - unavail)
        for rc in olds:
            unready_old = sum(1 for p in self._live(rc) if not p.ready)
            cut = min(rc.replicas, unready_old + max(0, removable))
            if cut > 0:
                ready_cut = max(0, cut - unready_old)
                removable -= ready_cut
                rc.replicas -= cut
        if all(rc.replicas == 0 and not self._live(rc) for rc in olds) and \
                sum(1 for p in self._live(cur) if p.ready) >= n and self._completed_rev != cur.revision:
            self._completed_rev = cur.revision
            self.event(f"rc/{cur.name}", "Complete", f"rollout to revision {cur.revision} finished")

    def _reconcile_replicas(self, now: float) -> None:
        for rc in self.rcs:
            live = self._live(rc)
            if len(live) < rc.replicas:
                for _ in range(rc.replicas - len(live)):
                    self._create_pod(rc, now)
            elif len(live) > rc.replicas:
                # deletion order of the replica controllers: unscheduled, not ready, then newest
                victims = sorted(live, key=lambda p: (p.scheduled, p.ready, -p.created))
                for p in victims[: len(live) - rc.replicas]:
                    if not p.scheduled:
                        p.gone = True
                        self.event(p.name, "Deleted", "never scheduled")
                    else:
                        self.kubelet.begin_delete(p, now)

    def _create_pod(self, rc: ReplicationController, now: float) -> Pod:
        suffix = "".join(random.choice(string.ascii_lowercase + string.digits) for _ in range(5))
        name = f"{rc.name}-{suffix}"
        labels = dict(rc.template.get("metadata", {}).get("labels") or {})
        if self.kind == "DeploymentConfig":
            labels.update({"deployment": rc.name, "deploymentconfig": self.name})
        else:
            labels["pod-template-hash"] = rc.name.rsplit("-", 1)[-1]
        ip = next(self._ips, None)
        if ip is None:
            raise ClusterError("pod network exhausted")
        c = rc.template["spec"]["containers"][0]
        res = c.get("resources") or {}
        req = m.parse_cpu((res.get("requests") or {}).get("cpu", (res.get("limits") or {}).get("cpu")))
        mem = m.parse_memory((res.get("limits") or {}).get("memory"))
        pod = Pod(name=name, owner=rc.name, revision=rc.revision, template=rc.template, ip=ip,
                  dir=self.state / "pods" / name, labels=labels, cpu_request=req, mem_limit=mem, created=now)
        self.pods[name] = pod
        self.event(name, "Created", f"{rc.name}, ip {ip}, cpu request {req:g}")
        return pod

    # ------------------------------------------------------------------ scheduling + CPU manager
    def _schedule(self, now: float) -> None:
        for p in sorted((p for p in self.pods.values() if not p.scheduled and not p.gone), key=lambda p: p.created):
            used = sum(q.cpu_request for q in self.pods.values() if q.scheduled and not q.gone)
            if used + p.cpu_request > self.allocatable + 1e-9:
                reason = f"0/1 nodes are available: 1 Insufficient cpu ({used:g} of {self.allocatable:g} requested)"
                if p.pending_reason != reason:
                    p.pending_reason = reason
                    self.event(p.name, "FailedScheduling", reason)
                continue
            p.scheduled = True
            p.pending_reason = ""
            c = p.template["spec"]["containers"][0]
            if self.policy == "static" and m.qos_class(c) == "Guaranteed" and float(p.cpu_request).is_integer():
                taken = {x for q in self.pods.values() if q.cpus and not q.gone for x in q.cpus}
                free = [x for x in self.real_cpus if x not in taken and x not in self.reserved]
                need = int(p.cpu_request)
                if len(free) >= need:
                    p.cpus = free[:need]
            self.event(p.name, "Scheduled", f"cpus {p.cpus if p.cpus else 'shared pool'}")

    def shared_pool(self) -> list[int]:
        taken = {x for q in self.pods.values() if q.cpus and not q.gone for x in q.cpus}
        pool = [x for x in self.real_cpus if x not in taken]
        return pool or list(self.real_cpus)

    # ------------------------------------------------------------------ endpoints
    def _reconcile_endpoints(self, now: float) -> None:
        for name, svc in self.services.items():
            sel = svc["spec"].get("selector") or {}
            port = svc["spec"]["ports"][0]
            target = port.get("targetPort", port["port"])
            eps = []
            for p in sorted(self.pods.values(), key=lambda p: p.name):
                if p.gone or p.terminating or not p.ready or not m.selector_matches(sel, p.labels):
                    continue
                tp = target if isinstance(target, int) or str(target).isdigit() else next(
                    (cp["containerPort"] for cp in p.container.get("ports") or [] if cp.get("name") == target), 8080)
                eps.append(f"{p.ip}:{int(tp)}")
            if eps != self._ep_desired.get(name):
                self._ep_desired[name] = eps
                self._ep_pending_since.setdefault(name, now)
            since = self._ep_pending_since.get(name)
            if since is not None and now - since >= self.endpoint_sync_s * self.time_scale:
                del self._ep_pending_since[name]
                cur = self._ep_desired[name]
                if cur != self._ep_written.get(name, (0, None))[1]:
                    gen = self._ep_written.get(name, (0, None))[0] + 1
                    tmp = self.state / "endpoints" / f".{name}.tmp"
                    tmp.write_text(f"# gen {gen}\n" + "".join(e + "\n" for e in cur))
                    os.replace(tmp, self.state / "endpoints" / name)  # rrproxy re-reads on change
                    self._ep_written[name] = (gen, list(cur))
            # published = what the proxy routes new connections to (it acknowledges each file)
            gen, cur = self._ep_written.get(name, (0, None))
            if cur is not None and cur != self._ep_published.get(name):
                try:
                    applied = int((self.state / "endpoints" / f"{name}.applied").read_text().strip() or 0)
                except (OSError, ValueError):
                    applied = 0
                if applied >= gen:
                    self._ep_published[name] = list(cur)
                    self.endpoint_history.setdefault(name, []).append((now - self.t0, list(cur)))
                    self.event(f"endpoints/{name}", "Synced", f"{len(cur)} ready: {' '.join(cur)}")

    # ------------------------------------------------------------------ configmaps
    def _reconcile_configmaps(self, now: float) -> None:
        due = [d for d in self._cm_due if d[0] <= now]
        if not due:
            return
        self._cm_due = [d for d in self._cm_due if d[0] > now]
        for _, pod_name, cm in due:
            p = self.pods.get(pod_name)
            if p is None or p.gone:
                continue
            for v in p.template["spec"].get("volumes") or []:
                if (v.get("configMap") or {}).get("name") == cm:
                    project_configmap(p.dir / "volumes" / v["name"], self.configmaps[cm], v["configMap"].get("items"))
                    self.event(p.name, "ConfigMapSynced", f"{cm} -> volume {v['name']}")

    # ------------------------------------------------------------------ the control loop
    def _loop(self) -> None:
        while not self._stop.is_set():
            with self.lock:
                now = time.monotonic()
                try:
                    self._reconcile_rollout(now)
                    self._reconcile_replicas(now)
                    self._schedule(now)
                    for p in list(self.pods.values()):
                        self.kubelet.tick(p, now)
                    self._reconcile_endpoints(now)
                    self._reconcile_configmaps(now)
                    for name in [n for n, p in self.pods.items() if p.gone]:
                        self.pods.pop(name)
                except Exception as e:  # noqa: BLE001 - keep the control plane running, record why
                    self.event("control-loop", "Error", repr(e))
                self.ticks += 1
            self._stop.wait(TICK_S)

    # ------------------------------------------------------------------ the `oc` surface
    def scale(self, replicas: int) -> None:
        """`oc scale dc/hola --replicas=N` (no new revision)."""
        with self.lock:
            self.workload["spec"]["replicas"] = int(replicas)
            self.event(f"{self.kind.lower()}/{self.name}", "Scaled", f"replicas={replicas}")

    def set_env(self, env: dict[str, str | None], container: str | None = None) -> None:
        """`oc set env dc/hola K=V` (`oc env` in the demo's era): a ConfigChange rollout."""
        with self.lock:
            self._template_changed(m.set_env(self.workload["spec"]["template"], container, env))

    def patch(self, patch: dict) -> None:
        """`oc patch dc/hola -p '<strategic merge patch>'`."""
        with self.lock:
            new = m.strategic_merge(self.workload, patch)
            self.workload["spec"]["replicas"] = new["spec"].get("replicas", self.desired)
            self._template_changed(new["spec"]["template"])

    def apply_configmap(self, name: str, data: dict[str, str]) -> None:
        """`oc apply -f configmap.yaml` for an existing ConfigMap: every pod mounting it sees
        the new files after the kubelet's sync delay."""
        with self.lock:
            self.configmaps[name] = dict(data)
            now = time.monotonic()
            for i, p in enumerate(sorted(self.pods.values(), key=lambda p: p.name)):
                if any((v.get("configMap") or {}).get("name") == name for v in p.template["spec"].get("volumes") or []):
                    # staggered over the sync period, as pods' sync loops are not aligned
                    stagger = (0.5 + 0.5 * (i % 8) / 8.0) * self.configmap_sync_s * self.time_scale
                    self._cm_due.append((now + stagger, p.name, name))
            self.event(f"configmap/{name}", "Updated", f"keys {sorted(data)}")

    def delete_pod(self, name: str, grace_s: float | None = None) -> None:
        """`oc delete pod NAME`: the controller replaces it."""
        with self.lock:
            self.kubelet.begin_delete(self.pods[name], time.monotonic(), grace_s)

    def kill_container(self, name: str, sig: int = signal.SIGKILL) -> None:
        """A crash: the container's process gets `sig`; the kubelet restarts it."""
        with self.lock:
            self.kubelet.kill_container(self.pods[name], sig)
            self.event(name, "Signal", f"sent {signal.Signals(sig).name} to the container")

    def get_pods(self) -> list[dict]:
        with self.lock:
            return [p.summary() for p in sorted(self.pods.values(), key=lambda p: p.name) if not p.gone]

    def top(self, sample_s: float = 0.5) -> list[dict]:
        """`kubectl top pod`: each running container's CPU use over `sample_s` (cores) and its
        resident memory, read from /proc, with its CPU limit and throttling counters."""
        from hola_amd.kube.kubelet import _proc_cpu_s, _proc_rss

        pods = [p for p in self.get_pods() if p["pid"]]
        t0 = time.monotonic()
        c0 = {p["name"]: _proc_cpu_s(p["pid"]) for p in pods}
        time.sleep(sample_s)
        dt = time.monotonic() - t0
        out = []
        for p in pods:
            c1 = _proc_cpu_s(p["pid"])
            if c1 is None or c0[p["name"]] is None:
                continue
            out.append({"name": p["name"], "cpu_cores": round((c1 - c0[p["name"]]) / dt, 3),
                        "memory_bytes": _proc_rss(p["pid"]) or 0, "cpu_throttle": p["cpu_throttle"]})
        return out

    def endpoints(self, name: str | None = None, published: bool = True) -> list[str]:
        with self.lock:
            name = name or next(iter(self.services))
            return list((self._ep_published if published else self._ep_desired).get(name, []))

    def rollout_status(self) -> dict:
        with self.lock:
            cur = self.rcs[-1]
            live = self._live(cur)
            old = [p for rc in self.rcs[:-1] for p in self.pods.values() if p.owner == rc.name and not p.gone]
            return {"revision": cur.revision, "rc": cur.name, "desired": self.desired,
                    "updated": len(live), "ready": sum(1 for p in live if p.ready), "old_pods": len(old),
                    "complete": not old and len(live) == self.desired and all(p.ready for p in live)}

    def wait(self, pred, timeout: float, what: str = "condition") -> None:
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            if pred():
                return
            time.sleep(0.02)
        raise TimeoutError(f"timed out after {timeout:.1f}s waiting for {what}; pods: {self.get_pods()}")

    def wait_ready(self, n: int | None = None, timeout: float = 120.0) -> None:
        """Until `n` (default: the desired count) endpoints are published and no rollout is
        in progress."""
        def ok():
            st = self.rollout_status()
            want = self.desired if n is None else n
            return st["complete"] and len(self.endpoints()) == want
        self.wait(ok, timeout, f"{n or self.desired} ready endpoints")
