"""bench.py's sub-runs: measurements taken on rank 0's CPUs after the timed region, so the
headline `value` is untouched by them.

* `config2`: BASELINE config 2 (one keep-alive connection, ~30 s) against the rank's replica.
* `deployed`: the replica exactly as the image and manifests start it (deploy/Dockerfile
  ENTRYPOINT + deploy/openshift/hola-dc.yaml args and env), with its own host load; the
  `zipkin` variant ("deployed" / "unset" / a collector URL) isolates the tracing path.
* `chain`: GET /api/hola-chaining, load generator -> hola A -> hola B (B answering as aloha),
  either engineered (bulkhead widened to 128, Feign logging off: the path's capacity) or
  as shipped (A started as the manifests start it: the reference's pool of 10 from
  conf/config.properties defaults, Feign BASIC logging, ZIPKIN_SERVER_URL set), with the
  attribution the two modes of this path need: host load, accept locality of both hops
  (load generator -> A from A's /metrics, A -> B from B's) and both replicas' busy-poll
  spin / back-off counters.
* `alt_layout`: the headline again in the other SMT layout on the same physical cores, so a
  1-GPU box (smt=off) and an 8-GPU node's N = 1 (smt=pair) each carry the other's figure.

Reference: HolaResource.java:69-78,94-113 (the chained call), Dockerfile:4-6 and
src/main/resources/config.properties:17,19 (the shipped configuration), pom.xml:77-94 (the
Service and the pod).
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import time
from pathlib import Path

from hola_amd.parallel.hostmetrics import (MetricsProbe, busy_fraction, cgroup_cpu_stat, cpu_times, irq_fraction,
                                           proc_cpu_s, steal_fraction)
from hola_amd.parallel.loadgen import ControlledLoadgen
from hola_amd.server import HolaProcess
from hola_amd.utils import cpu as _cpu
from hola_amd.utils.cpu import format_cpu_list, split_mirrored, split_server_loadgen
from hola_amd.utils.net import http_get

REPO = Path(__file__).resolve().parents[2]
FALLBACK = "Aloha response (fallback)"  # HolaResource.java:111-112


# ---------------------------------------------------------------- host load / counters

def other_siblings(own, job_cpus) -> set[int]:
    """SMT siblings of `own` that the job itself did not plan (busy there = another tenant)."""
    job = set(job_cpus) | set(own)
    return {x for c in own for x in _cpu.siblings(c)} - job


def l3_neighbours(own, job_cpus) -> set[int]:
    """CPUs that share an L3 with `own`, outside the job and not SMT siblings of `own` (those
    are reported apart): busy ones are other tenants filling the cache the job works in."""
    doms = {_cpu.l3_domain(c) for c in own} - {None, -1}
    if not doms:
        return set()
    sib = {x for c in own for x in _cpu.siblings(c)}
    return {c for c in _cpu.online_cpus() if _cpu.l3_domain(c) in doms} - set(job_cpus) - set(own) - sib


def host_load(t0: dict, t1: dict, own, job_cpus) -> dict:
    """Busy share of `own`, of the SMT siblings of `own` that belong to no part of the job and
    of the other CPUs of `own`'s L3 domains (`l3_others`), plus the interrupt (hard + soft) and
    steal shares of `own` (a slow run on quiet siblings can then be told
    apart from one that lost time to IRQs, a hypervisor or a busy L3 neighbour)."""
    own = set(own)
    return {"own": busy_fraction(t0, t1, own), "siblings": busy_fraction(t0, t1, other_siblings(own, job_cpus)),
            "l3_others": busy_fraction(t0, t1, l3_neighbours(own, job_cpus)),
            "irq_own": irq_fraction(t0, t1, own), "steal_own": steal_fraction(t0, t1, own)}


def metrics_counters(port: int, host: str = "127.0.0.1", probe: MetricsProbe | None = None) -> dict:
    """The /metrics counters the sub-runs attribute with: accept locality, busy-poll spins and
    back-offs, Hystrix events, requests (empty on a failed scrape). With a kept-alive `probe`
    the scrapes add no accepted connection of their own to the locality counts."""
    if probe is not None:
        text = probe.text()
    else:
        try:
            st, _, body = http_get(host, port, "/metrics", timeout=5.0)
        except OSError:
            return {}
        if st != 200:
            return {}
        text = body.decode()
    out: dict[str, float] = {}
    for ln in text.splitlines():
        if not ln or ln[0] == "#":
            continue
        name, _, val = ln.rpartition(" ")
        if name.startswith("hola_accept_locality_total{"):
            out["locality." + name.split('"')[1]] = float(val)
        elif name.startswith("hola_busy_poll_spins_total{"):
            out["spins." + name.split('"')[1]] = float(val)
        elif name == "hola_busy_poll_backoffs_total":
            out["spins.backoffs"] = float(val)
        elif name == "hola_busy_poll_backoff_ms_total":
            out["spins.backoff_ms"] = float(val)
        elif name == "hola_busy_poll_resumes_total":
            out["spins.resumes"] = float(val)
        elif name.startswith("hola_hystrix_events_total{"):
            out["hystrix." + name.split('event="')[1].split('"')[0]] = float(val)
        elif name.startswith("hola_hystrix_circuit_transitions_total{"):
            to = name.split('to="')[1].split('"')[0]
            by = name.split('by="')[1].split('"')[0] if 'by="' in name else ""
            out["circuit." + (f"{to}_{by}" if by else to)] = float(val)
        elif name == "hola_http_requests_total":
            out["requests"] = float(val)
        elif name == "hola_loop_idle_spin_seconds_total":
            out["loop.idle_spin_s"] = float(val)
        elif name == "hola_loop_blocking_waits_total":
            out["loop.blocking_waits"] = float(val)
        elif name.startswith("hola_loop_poll_gaps_total{"):
            out["loop.gaps_over_" + name.split('"')[1]] = float(val)
        elif name == "hola_loop_poll_gap_max_seconds":
            out["gauge.gap_max_s"] = float(val)
        elif name == "hola_loop_passes_total":
            out["loop.passes"] = float(val)
        elif name == "hola_worker_user_instructions_total":
            out["pmu.instructions"] = float(val)
        elif name == "hola_worker_user_cycles_total":
            out["pmu.cycles"] = float(val)
    return out


def counter_delta(c0: dict, c1: dict, prefix: str) -> dict:
    return {k[len(prefix):]: int(c1.get(k, 0) - c0.get(k, 0)) for k in sorted(set(c0) | set(c1))
            if k.startswith(prefix)}


def locality_fraction(d: dict) -> dict:
    n = sum(d.values())
    return {k: round(v / n, 4) for k, v in d.items() if v} if n else {}


# ---------------------------------------------------------------- processes as deployed

def deployed_argv_env(port: int, hostname: str, extra_args: list[str] | None = None,
                      env_over: dict | None = None) -> tuple[list[str], dict]:
    """argv and environment of a replica started as the image and manifests start it:
    deploy/Dockerfile's ENTRYPOINT (its /app paths mapped to this tree) + the container args
    and env of deploy/openshift/hola-dc.yaml, HOSTNAME = a pod name. `extra_args` are appended
    (the listen port always; --aloha-url for the shipped chain); `env_over` replaces or (value
    None) removes variables."""
    from hola_amd import native
    from hola_amd.kube import manifests as km
    from hola_amd.kube.image import Image

    img = Image.from_dockerfile()
    dc = next(o for o in km.load_objects([REPO / "deploy/openshift/hola-dc.yaml"]) if o["kind"] == "DeploymentConfig")
    cont = dc["spec"]["template"]["spec"]["containers"][0]
    argv = [str(img.files.get(x, x)) for x in img.entrypoint] + [str(x) for x in cont.get("args") or []]
    argv[0] = str(native.binary("hola"))
    argv += ["--port", str(port)] + list(extra_args or [])
    env = {k: v for k, v in os.environ.items() if k in ("PATH", "LANG", "LD_LIBRARY_PATH")}
    env.update(img.env)
    env.update({e["name"]: str(e["value"]) for e in cont.get("env") or [] if "value" in e})
    env["HOSTNAME"] = hostname  # fieldRef metadata.name
    for k, v in (env_over or {}).items():
        if v is None:
            env.pop(k, None)
        else:
            env[k] = v
    return argv, env


def pod_loadgen_cpus(pod_cpus, load_cpus) -> list[int]:
    """The load-generator CPUs for a pod-sized replica: those of `load_cpus` in the L3 domains
    of the pod's own CPUs, where the headline places its load generator too (a client thread
    in another L3 makes every one of its connections a cross-CCD hand-off: twice the server's
    CPU per request, profiles/round6/01_pod_shape). All of `load_cpus` when none share one."""
    doms = {_cpu.l3_domain(c) for c in pod_cpus}
    same = [c for c in load_cpus if _cpu.l3_domain(c) in doms]
    return same or list(load_cpus)


def manifest_pod_cpus() -> int:
    """The pod's CPU limit in deploy/openshift/hola-dc.yaml (whole CPUs; a Guaranteed pod
    under the static CPU manager gets exactly this many exclusive CPUs)."""
    from hola_amd.kube import manifests as km

    dc = next(o for o in km.load_objects([REPO / "deploy/openshift/hola-dc.yaml"]) if o["kind"] == "DeploymentConfig")
    lim = str(dc["spec"]["template"]["spec"]["containers"][0].get("resources", {}).get("limits", {}).get("cpu", "0"))
    return max(1, int(float(lim[:-1]) / 1000) if lim.endswith("m") else int(float(lim)))


class DeployedProc:
    """A replica started from deployed_argv_env() in a cpuset (a Guaranteed pod under the
    static CPU manager); stderr to /dev/null (Feign BASIC logging writes two lines per call)."""

    def __init__(self, cpus, hostname: str, extra_args=None, env_over=None, base_port: int = 18900):
        self.cpus = list(cpus)
        self.port = free_port_block(base_port, 1)
        self.argv, self.env = deployed_argv_env(self.port, hostname, extra_args, env_over)
        self.proc: subprocess.Popen | None = None

    def __enter__(self) -> "DeployedProc":
        cpus = self.cpus
        self.proc = subprocess.Popen(self.argv, env=self.env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                                     preexec_fn=lambda: os.sched_setaffinity(0, cpus))
        deadline = time.monotonic() + 10
        while True:
            try:
                socket.create_connection(("127.0.0.1", self.port), timeout=1).close()
                return self
            except OSError:
                if self.proc.poll() is not None or time.monotonic() > deadline:
                    self.__exit__()
                    raise RuntimeError(f"deployed replica did not start (rc {self.proc.poll()})")
                time.sleep(0.02)

    def __exit__(self, *exc) -> None:
        if self.proc and self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(timeout=15)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()

    def shown_args(self) -> str:
        return " ".join(["hola"] + self.argv[1:])

    def shown_env(self, keys) -> str:
        return " ".join(f"{k}={v}" for k, v in sorted(self.env.items()) if k in keys)


def free_port_block(start: int, n: int, host: str = "127.0.0.1") -> int:
    """First base >= start such that base..base+n-1 can all be bound on `host`."""
    base = start
    for _ in range(200):
        socks = []
        try:
            for i in range(n):
                sk = socket.socket(socket.AF_INET6 if ":" in host else socket.AF_INET)
                sk.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
                sk.bind((host, base + i))
                socks.append(sk)
            return base
        except OSError:
            base += n + 7
        finally:
            for sk in socks:
                sk.close()
    return start


# ---------------------------------------------------------------- timed closed-loop runs

def timed_closed_loop(lg: ControlledLoadgen, connections: int, seconds: float, pid: int | None,
                      own, job_cpus, warm_s: float = 1.0) -> dict:
    """A closed-loop run of `seconds` after `warm_s` of warm-up, warm-up and measurement one
    continuous run of the generator (`runfor`). A series of shorter runs left every connection
    idle between them: the server's pools drained, and the first request after each gap met
    state that steady load never shows (the shipped chain's breaker tripping with no call in
    flight and staying open a whole sleep window: profiles/round5/11_shipped_breaker). Latency,
    errors, bodies, the server's CPU per request and the host load of the timed part (the CPU
    and host-load samples bracket the whole run; the warm-up is at the same load)."""
    lg.reset()
    t0, c0 = cpu_times(), proc_cpu_s(pid) if pid else 0.0
    r = lg.run_for(seconds, warm_s)
    el_ns, reqs, errs = r["elapsed_ns"], r["requests"], r["errors"]
    t1, c1 = cpu_times(), proc_cpu_s(pid) if pid else 0.0
    st = lg.stats()
    el = el_ns / 1e9
    return {"rps": reqs / el if el > 0 else 0.0, "elapsed_s": el, "requests": reqs,
            "errors": errs, "p50_ns": st["p50_ns"], "p99_ns": st["p99_ns"], "p999_ns": st.get("p999_ns", 0),
            "non2xx": st.get("non2xx", 0),
            "body_checked": st.get("body_checked", 0), "body_mismatch": st.get("body_mismatch", 0),
            "body_alt": st.get("body_alt", 0),
            # the CPU sample spans the warm-up too, at the same load: per request of the whole run
            "cpu_us_per_req": (1e6 * (c1 - c0) / max(1.0, reqs * (el + warm_s) / max(1e-9, el))) if pid else None,
            "host_load": host_load(t0, t1, own, job_cpus)}


def loop_block(m0: dict, m1: dict, reqs: float) -> dict:
    """A replica's event-loop accounting between two metrics_counters() scrapes: CPU in empty
    polls, waits that could sleep (per request), gaps between polls past 100 us / 1 ms / 10 ms
    and the longest gap since the replica started, adaptive spin outcomes."""
    d = counter_delta(m0, m1, "loop.")
    pmu = counter_delta(m0, m1, "pmu.") if "pmu.instructions" in m1 else {}
    return {"idle_spin_s": round(m1.get("loop.idle_spin_s", 0.0) - m0.get("loop.idle_spin_s", 0.0), 4),
            # the workers' own user-space instructions and cycles per request (hardware
            # counters; absent where the host does not allow them)
            "user_instr_per_req": round(pmu["instructions"] / max(1.0, reqs), 1) if pmu else None,
            "user_cycles_per_req": round(pmu["cycles"] / max(1.0, reqs), 1) if pmu else None,
            "passes_per_req": round(d.get("passes", 0) / max(1.0, reqs), 4),
            "blocking_waits_per_req": round(d.get("blocking_waits", 0) / max(1.0, reqs), 4),
            "gaps_over_100us": d.get("gaps_over_100us", 0), "gaps_over_1ms": d.get("gaps_over_1ms", 0),
            "gaps_over_10ms": d.get("gaps_over_10ms", 0),
            "gap_max_since_start_us": round(1e6 * m1.get("gauge.gap_max_s", 0.0), 1),
            "spins": counter_delta(m0, m1, "spins.")}


def loadgen_block(st: dict, cpu_s: float, reqs: float) -> dict:
    """The load generator's side of a run from its stats (since its last reset): CPU and busy
    CPU (minus empty polls) per request, how its polls ended (found work at once, after
    spinning, or ran out and slept), and its own scheduling gaps."""
    idle = st.get("idle_spin_ns", 0) / 1e9
    n = max(1.0, reqs)
    return {"cpu_us_per_req": round(1e6 * cpu_s / n, 3), "busy_cpu_us_per_req": round(1e6 * (cpu_s - idle) / n, 3),
            "user_instr_per_req": round(st["user_instructions"] / n, 1) if "user_instructions" in st else None,
            "user_cycles_per_req": round(st["user_cycles"] / n, 1) if "user_cycles" in st else None,
            "idle_spin_s": round(idle, 4),
            "polls": {"hit_at_once": st.get("poll_hits", 0), "hit_after_spin": st.get("spin_hits", 0),
                      "ran_out": st.get("spin_misses", 0)},
            "blocking_waits_per_req": round(st.get("blocking_waits", 0) / n, 4),
            "gaps_over_100us": st.get("gaps_over_100us", 0), "gaps_over_1ms": st.get("gaps_over_1ms", 0),
            "gaps_over_10ms": st.get("gaps_over_10ms", 0), "gap_max_us": round(st.get("gap_max_ns", 0) / 1e3, 1),
            "send_late_max_us": round(st.get("send_late_max_ns", 0) / 1e3, 1)}


def attributed_closed_loop(lg: ControlledLoadgen, seconds: float, pid: int, port: int, server_cpus, load_cpus,
                           job_cpus, host: str = "127.0.0.1", warm_s: float = 1.0,
                           before_connect: dict | None = None) -> dict:
    """timed_closed_loop() with the attribution a replica's CPU per request needs (VERDICT r5
    weak #1, #4): busy CPU per request (process CPU minus the loop's empty polls), the serving
    threads' CPU and context switches apart from the process's other threads, the loop's
    waits and gaps, the load generator's own CPU and poll outcomes, TCP segments per request,
    and the host load of the server's and the load generator's CPUs separately."""
    from hola_amd.parallel.hostmetrics import task_stats, task_stats_delta, tcp_counters

    probe = MetricsProbe(host, port)
    try:
        m0, ts0, tcp0, lg0 = metrics_counters(port, host, probe), task_stats(pid), tcp_counters(), proc_cpu_s(lg.proc.pid)
        t0, w0 = cpu_times(), time.perf_counter()
        r = timed_closed_loop(lg, 0, seconds, pid, list(server_cpus) + list(load_cpus), job_cpus, warm_s=warm_s)
        t1, wall = cpu_times(), time.perf_counter() - w0
        m1, ts1, tcp1, lg1 = metrics_counters(port, host, probe), task_stats(pid), tcp_counters(), proc_cpu_s(lg.proc.pid)
        st = lg.stats()
    finally:
        probe.close()
    el = r["elapsed_s"]
    # every sample spans the warm-up too, at the same load: per request of the whole run
    reqs = r["requests"] * (el + warm_s) / max(1e-9, el)
    threads = task_stats_delta(ts0, ts1)
    cpu = sum(g["cpu_s"] for g in threads.values())
    loop = loop_block(m0, m1, reqs)
    hl_server = host_load(t0, t1, server_cpus, job_cpus)
    r.update({
        "server_busy_cpu_us_per_req": round(1e6 * (cpu - loop["idle_spin_s"]) / max(1.0, reqs), 3),
        # everything the server's CPUs did per request, whoever it is charged to: the
        # replica's threads, and interrupt time there (on loopback the receive path of the
        # segments the replica sent, when the kernel runs it as a softirq)
        "server_cpus_us_per_req": (round(1e6 * hl_server["own"] * len(set(server_cpus)) * wall / max(1.0, reqs * wall / (el + warm_s)), 3)
                                   if hl_server["own"] is not None else None),
        "server_threads": {k: {**v, "vol_per_req": round(v["vol"] / max(1.0, reqs), 4),
                               "invol_per_req": round(v["invol"] / max(1.0, reqs), 4)} for k, v in threads.items()},
        "server_loop": loop,
        "loadgen": loadgen_block(st, lg1 - lg0, reqs),
        "tcp_per_req": {k: round((tcp1[k] - tcp0[k]) / max(1.0, reqs), 3) for k in tcp1 if k in tcp0},
        "host_load_server": hl_server,
        # where each connection's client ran relative to the worker serving it (from the
        # replica's counters taken before the load generator connected)
        "locality": locality_fraction(counter_delta(before_connect or {}, m1, "locality.")) if before_connect is not None
        else {},
        "host_load_loadgen": host_load(t0, t1, load_cpus, job_cpus)})
    return r


def config2(a, host: str, port: int, server_cpus, load_cpus, bodies, job_cpus) -> dict | None:
    """BASELINE config 2: one keep-alive connection against this rank's replica."""
    if a.c1_reqs <= 0 and a.c1_seconds <= 0:
        return None
    lg = ControlledLoadgen([(host, port)], 1, 1, cpu_list=str(load_cpus[0]), path=a.path,
                           busy_poll_us=a.busy_poll_us, busy_poll_pause=a.busy_poll_pause, epoll_lt=a.epoll_lt,
                           expect_bodies=bodies, verify_body=bodies is None)
    try:
        warm = lg.run(max(1000, a.c1_reqs // 10) if a.c1_reqs > 0 else 50000)
        n = a.c1_reqs
        if n <= 0:  # size the run from the warm-up rate: about --c1-seconds, within bounds
            rate = warm["requests"] / max(1e-9, warm["elapsed_ns"] / 1e9)
            n = int(min(30_000_000, max(20_000, rate * a.c1_seconds)))
        lg.reset()
        own = set(server_cpus) | {load_cpus[0]}
        t0 = cpu_times()
        r = lg.run(n)
        t1 = cpu_times()
        st = lg.stats()
    finally:
        lg.close()
    el = r["elapsed_ns"] / 1e9
    return {"rps": r["requests"] / el if el > 0 else 0.0, "requests": r["requests"], "elapsed_s": el,
            "p50_ns": st["p50_ns"], "p99_ns": st["p99_ns"], "errors": r["errors"],
            "body_checked": st.get("body_checked", 0), "client_cpu": load_cpus[0],
            "host_load": host_load(t0, t1, own, job_cpus)}


ZIPKIN_VARIANTS = ("deployed", "unset", "sink")


def deployed(a, server_cpus, load_cpus, job_cpus, zipkin: str = "deployed", seconds: float | None = None,
             loadgen_busy_poll: int | None = None, connections: int | None = None, threads: int | None = None,
             cpu_profile: str | None = None) -> dict:
    """The replica as deployed, driven by the headline's load generator for about
    --deployed-seconds, with attributed_closed_loop()'s accounting. `zipkin`: "deployed" = the
    manifests' ZIPKIN_SERVER_URL (the cluster's zipkin-query Service, which does not resolve on
    a bare host: spans are recorded and then dropped when the post fails), "unset" = no
    collector (spans dropped at the source, the headline's path), "sink" = a native discard
    collector that accepts every post. The other keywords vary one thing for the pod-shape
    study (bench/pod_shape.py): the load generator's busy-poll window (default: the
    headline's), the connections, the replica's --threads (default: as deployed, one worker
    per CPU of its cpuset), and a --cpu-profile of the replica."""
    from hola_amd.parallel.hostmetrics import start_zipkin_sink

    sink = None
    env_over: dict = {}
    if zipkin == "unset":
        env_over["ZIPKIN_SERVER_URL"] = None
    elif zipkin == "sink":
        sink = start_zipkin_sink()
        env_over["ZIPKIN_SERVER_URL"] = f"http://127.0.0.1:{sink[1]}"
    extra = (["--threads", str(threads)] if threads else []) + (["--cpu-profile", cpu_profile] if cpu_profile else [])
    lg_bp = a.busy_poll_us if loadgen_busy_poll is None else loadgen_busy_poll
    conns = connections or a.connections
    try:
        with DeployedProc(server_cpus, "hola-1-deplo", extra_args=extra, env_over=env_over) as d:
            body = ["Hola de hola-1-deplo"] if a.path == "/api/hola" else None
            pre = metrics_counters(d.port)
            lg = ControlledLoadgen([("127.0.0.1", d.port)], conns, len(load_cpus),
                                   cpu_list=",".join(map(str, load_cpus)), path=a.path, busy_poll_us=lg_bp,
                                   busy_poll_pause=a.busy_poll_pause if lg_bp else 0, epoll_lt=a.epoll_lt,
                                   expect_bodies=body, verify_body=body is None)
            try:
                r = attributed_closed_loop(lg, seconds or a.deployed_seconds, d.proc.pid, d.port, server_cpus,
                                           load_cpus, job_cpus, before_connect=pre)
            finally:
                lg.close()
            shown = d.shown_args().split()
            r.update({"args": " ".join(shown[:len(shown) - 2 - len(extra)]), "cpus": format_cpu_list(server_cpus),
                      "loadgen_cpus": format_cpu_list(load_cpus), "connections": conns,
                      "loadgen_busy_poll_us": lg_bp, "threads": threads or len(server_cpus),
                      "env": d.shown_env(set(d.env) - {"PATH", "LANG", "LD_LIBRARY_PATH"}), "zipkin": zipkin})
            return r
    finally:
        if sink:
            sink[0].terminate()
            sink[0].wait(timeout=10)


def chain(a, cpus, job_cpus, shipped: bool = False, seconds: float | None = None, loadgen_busy_poll: int = -1,
          exe: Path | None = None) -> dict:
    """GET /api/hola-chaining end to end (HolaResource.java:69-78,94-113): load generator ->
    hola A -> hola B, where B plays aloha (B's own aloha is unreachable, so B answers its
    fallback list at once: ["Hola de B", "Aloha response (fallback)"], which A decodes as the
    aloha's List<String>). Every request crosses A's pooled keep-alive client, the Hystrix
    command (breaker, bulkhead, 600 ms timer), B3 propagation and the JSON decode. The CPUs
    are split 2:1:1 (A does two hops' work) with each L3 holding a share of all three.

    Engineered (default): A's bulkhead widened to --chain-pool, Feign logging and tracing off:
    every body must be the two-hop answer. Shipped: A is started as the manifests start it
    (image ENTRYPOINT + hola-dc.yaml args and env: the reference's pool of 10, Feign BASIC
    logging on, ZIPKIN_SERVER_URL set); the only changes are the aloha URL and path (B on
    loopback instead of the aloha Service) and the listen port. A body is then either the
    two-hop answer or A's own fallback (counted apart, as body_alt). `exe`: another server
    binary for A and B (A/B runs of server builds; engineered mode)."""
    seconds = seconds or a.chain_seconds
    plan = split_mirrored(sorted(cpus), {"A": 2, "B": 1, "loadgen": 1})
    lg_bp = a.chain_loadgen_busy_poll if loadgen_busy_poll < 0 else loadgen_busy_poll
    with HolaProcess(args=["--aloha-url", "http://127.0.0.1:1/", "--feign-log", "none", "--no-tracing",
                           "--feign-retry", "off", "--log-level", "warn"], env={"HOSTNAME": "B"},
                     threads=len(plan["B"]), cpu_list=format_cpu_list(plan["B"]), exe=exe) as b:
        aloha = ["--aloha-url", f"http://127.0.0.1:{b.port}/", "--aloha-path", "api/hola-chaining"]
        if shipped:
            a_ctx = DeployedProc(plan["A"], "A", extra_args=aloha)
        else:
            a_ctx = HolaProcess(args=aloha + ["--feign-log", "none", "--hystrix-pool-size", str(a.chain_pool),
                                              "--log-level", "warn"],
                                env={"HOSTNAME": "A"}, threads=len(plan["A"]), cpu_list=format_cpu_list(plan["A"]),
                                exe=exe)
        with a_ctx as s:
            st, _, body = http_get("127.0.0.1", s.port, "/api/hola-chaining", timeout=5.0)
            want = ["Hola de A", "Hola de B", FALLBACK]
            if st != 200 or json.loads(body) != want:
                return {"error": f"unexpected first answer {st} {body[:200]!r}"}
            fallback_body = json.dumps(["Hola de A", FALLBACK], separators=(",", ":"))
            probes = MetricsProbe("127.0.0.1", s.port), MetricsProbe("127.0.0.1", b.port)
            m0 = metrics_counters(s.port, probe=probes[0]), metrics_counters(b.port, probe=probes[1])
            c0 = proc_cpu_s(s.proc.pid), proc_cpu_s(b.proc.pid)
            thr0 = cgroup_cpu_stat()
            lg = ControlledLoadgen([("127.0.0.1", s.port)], a.connections, len(plan["loadgen"]),
                                   cpu_list=format_cpu_list(plan["loadgen"]), path="/api/hola-chaining",
                                   busy_poll_us=lg_bp, expect_bodies=[body.decode()],
                                   alt_bodies=[fallback_body] if shipped else None)
            try:
                w0 = time.perf_counter()
                r = timed_closed_loop(lg, a.connections, seconds, None, cpus, job_cpus)
                wall = time.perf_counter() - w0
            finally:
                lg.close()
            c1 = proc_cpu_s(s.proc.pid), proc_cpu_s(b.proc.pid)
            thr1 = cgroup_cpu_stat()
            m1 = metrics_counters(s.port, probe=probes[0]), metrics_counters(b.port, probe=probes[1])
            for p in probes:
                p.close()
            args = s.shown_args() if shipped else None
    rps = r["rps"]
    # CPU over the whole sub-run (its warm-up included) per request at the measured rate
    busy = ((c1[0] - c0[0]) / wall, (c1[1] - c0[1]) / wall)
    # A's event loop and its workers' own hardware counters over the same span (VERDICT r5 #4:
    # an efficiency figure independent of the peer): busy CPU without the empty polls, and
    # user-space instructions and cycles per chained request
    a_loop = loop_block(m0[0], m1[0], rps * wall)
    out = {**r, "a_cpu_us_per_req": 1e6 * busy[0] / rps if rps else 0.0,
           "b_cpu_us_per_req": 1e6 * busy[1] / rps if rps else 0.0,
           "a_busy_cpu_us_per_req": (1e6 * (c1[0] - c0[0] - a_loop["idle_spin_s"]) / (rps * wall)) if rps else 0.0,
           "a_user_instr_per_req": a_loop["user_instr_per_req"], "a_user_cycles_per_req": a_loop["user_cycles_per_req"],
           "hystrix": counter_delta(m0[0], m1[0], "hystrix."),
           # A's breaker: times it opened, and closed by a trial or by a call already running
           "circuit": counter_delta(m0[0], m1[0], "circuit."),
           # where each accepted connection's client thread ran relative to the worker serving
           # it: load generator -> A (A's counters), A's pooled client -> B (B's counters)
           "locality": {"loadgen_to_a": locality_fraction(counter_delta(m0[0], m1[0], "locality.")),
                        "a_to_b": locality_fraction(counter_delta(m0[1], m1[1], "locality."))},
           # adaptive busy-polling of each replica over the sub-run: spins that found work,
           # spins that ran out, back-offs and the milliseconds spent backed off (summed over
           # workers)
           "spins": {"a": counter_delta(m0[0], m1[0], "spins."), "b": counter_delta(m0[1], m1[1], "spins.")},
           # CFS bandwidth throttling of this cgroup over the sub-run (a CPU quota that the sub-run's
           # spinning threads exceed stops them all until the next 100 ms period)
           "cgroup_throttle": {"periods": thr1.get("nr_periods", 0) - thr0.get("nr_periods", 0),
                               "throttled_periods": thr1.get("nr_throttled", 0) - thr0.get("nr_throttled", 0),
                               "throttled_ms": round((thr1.get("throttled_usec", 0) - thr0.get("throttled_usec", 0)) / 1000, 1)},
           "cpus": {k: format_cpu_list(v) for k, v in plan.items()}, "loadgen_busy_poll_us": lg_bp,
           "pool": 10 if shipped else a.chain_pool, "shipped": shipped}
    if args:
        out["args"] = args
    return out


def alt_layout(a, host: str, server_cpus, load_cpus, smt: str, job_cpus, bodies, seconds: float) -> dict:
    """The headline replica in the other SMT layout, on the rank's physical cores:
    smt=off here (1-GPU box)  -> pair on the server's physical cores (worker + its client
                                 thread on the two threads of one core), i.e. the 8-GPU node's
                                 per-replica shape at half its cores;
    smt=pair here (the node)  -> off on the same physical cores (server workers and client
                                 threads on separate cores, siblings idle): the 1-GPU box's
                                 BENCH layout when the rank has 16 physical cores."""
    if smt == "pair":
        phys = sorted({min(_cpu.siblings(c)) for c in list(server_cpus) + list(load_cpus)})
        sv, ld = split_server_loadgen(phys, max(1, len(phys) // 2))
        alt = "off"
    else:
        sv = sorted(server_cpus)
        ld = [next((x for x in _cpu.siblings(c) if x != c), c) for c in sv]
        alt = "pair"
    with HolaProcess(args=["--busy-poll-us", a.server_busy_poll] + (["--busy-poll-pause", "16"] if alt == "pair" else [])
                     + (["--no-tracing"] if a.no_tracing else []),
                     env={"HOSTNAME": "replica-0"}, threads=len(sv), cpu_list=format_cpu_list(sv),
                     log_level="warn") as s:
        lg = ControlledLoadgen([("127.0.0.1", s.port)], a.connections, len(ld), cpu_list=",".join(map(str, ld)),
                               path=a.path, busy_poll_us=a.busy_poll_us, busy_poll_pause=16 if alt == "pair" else 0,
                               expect_bodies=bodies, verify_body=bodies is None)
        try:
            r = timed_closed_loop(lg, a.connections, seconds, s.proc.pid, sv + ld, job_cpus)
        finally:
            lg.close()
    phys_n = len({min(_cpu.siblings(c)) for c in sv + ld})
    r.update({"smt": alt, "server_cpus": format_cpu_list(sv), "loadgen_cpus": format_cpu_list(ld),
              "physical_cores": phys_n, "rps_per_physical_core": r["rps"] / max(1, phys_n)})
    return r


def v4_headline(a, server_args: list[str], server_cpus, load_cpus, conn_targets, job_cpus, bodies,
                seconds: float) -> dict:
    """The headline replica and load generator again, unchanged but for the address family:
    IPv4 loopback, the transport of the image (it binds 0.0.0.0, deploy/Dockerfile) where the
    headline runs on ::1. Same CPUs, arguments, connection layout and
    busy-polling; one continuous run (`runfor`) with its warm-up."""
    args = []
    skip = False
    for x in server_args:  # drop the headline's --host (HolaProcess binds 127.0.0.1)
        if skip:
            skip = False
            continue
        if x == "--host":
            skip = True
            continue
        args.append(x)
    with HolaProcess(args=args, env={"HOSTNAME": "replica-0"}, threads=len(server_cpus),
                     cpu_list=format_cpu_list(server_cpus), log_level="warn") as s:
        lg = ControlledLoadgen([("127.0.0.1", s.port)], a.connections, len(load_cpus),
                               cpu_list=",".join(map(str, load_cpus)), path=a.path, busy_poll_us=a.busy_poll_us,
                               busy_poll_pause=a.busy_poll_pause, epoll_lt=a.epoll_lt, pipeline=a.pipeline,
                               expect_bodies=bodies, verify_body=bodies is None, conn_targets=conn_targets)
        try:
            r = timed_closed_loop(lg, a.connections, seconds, s.proc.pid, list(server_cpus) + list(load_cpus), job_cpus)
        finally:
            lg.close()
    return r


def plain_dealing_run(a, targets: list[tuple[str, int]], local_rank: int, load_cpus, bodies, seconds: float) -> dict:
    """One rank's share of the topology-blind front: this rank's load
    generator on its own cores deals its connections (i + rank) % N over every replica of the
    node, as a LoadBalancer Service (pom.xml:77-80) would without placing any client. Every
    rank runs it at once (the caller brackets it with barriers); returns the rank's counts and
    its latency histogram for merging."""
    lg = ControlledLoadgen(targets, a.connections, len(load_cpus), cpu_list=",".join(map(str, load_cpus)),
                           path=a.path, target_offset=local_rank, busy_poll_us=a.busy_poll_us,
                           busy_poll_pause=a.busy_poll_pause, epoll_lt=a.epoll_lt, pipeline=a.pipeline,
                           expect_bodies=bodies, verify_body=bodies is None)
    try:
        lg.reset()
        r = lg.run_for(seconds, 1.0)
        st = lg.stats()
    finally:
        lg.close()
    return {"requests": r["requests"], "errors": r["errors"], "elapsed_s": r["elapsed_ns"] / 1e9,
            "hist": st.get("hist", ""), "non2xx": st.get("non2xx", 0), "body_checked": st.get("body_checked", 0),
            "body_mismatch": st.get("body_mismatch", 0), "load_cpus": format_cpu_list(load_cpus)}
