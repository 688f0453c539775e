"""Host-side measurements for bench.py (BASELINE configs 2-4 on the MI355X node's EPYC cores).

Process and thread CPU time from /proc, cgroup v2 CPU throttling, namespace-wide TCP segment
counters, a replica's own /metrics counters (spans, connection placement), and the native
discard Zipkin collector used by `bench.py --zipkin-sink`. Everything here reads the host;
nothing touches a GPU.
"""
from __future__ import annotations

import json
import os
import time
from pathlib import Path


def start_zipkin_sink():
    """Native discard Zipkin collector on an ephemeral port: (process, port)."""
    import subprocess
    import tempfile

    from hola_amd.native import binary

    import atexit
    import shutil

    tmp = Path(tempfile.mkdtemp(prefix="hola_sink_"))
    pf = tmp / "port"
    proc = subprocess.Popen([str(binary("hola_zipkin_sink")), "--port", "0", "--port-file", str(pf)])

    def stop():
        if proc.poll() is None:
            proc.terminate()
            proc.wait(timeout=10)

    atexit.register(stop)  # also on an exception before main()'s cleanup runs
    try:
        deadline = time.monotonic() + 10
        while not pf.exists():
            if proc.poll() is not None or time.monotonic() > deadline:
                raise RuntimeError("hola_zipkin_sink did not start")
            time.sleep(0.01)
        return proc, int(pf.read_text())
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def sink_stats(port: int) -> dict:
    if not port:
        return {}
    from hola_amd.utils.net import http_get
    st, _, body = http_get("127.0.0.1", port, "/stats")
    return json.loads(body) if st == 200 else {}


class MetricsProbe:
    """One kept-alive connection to a replica's /metrics. Probing over it adds no accepted
    connection after the first, so the accept-placement counters taken before and after a
    run differ by exactly the run's own connections."""

    def __init__(self, host: str, port: int, timeout: float = 5.0):
        import http.client

        self._conn = http.client.HTTPConnection(host, port, timeout=timeout)

    def text(self) -> str:
        import http.client

        for _ in range(2):  # the replica may have closed the idle connection: reconnect once
            try:
                self._conn.request("GET", "/metrics")
                r = self._conn.getresponse()
                body = r.read()
                return body.decode() if r.status == 200 else ""
            except (OSError, http.client.HTTPException):
                self._conn.close()
        return ""

    def close(self) -> None:
        self._conn.close()


def _metrics_text(host: str, port: int) -> str:
    from hola_amd.utils.net import http_get
    try:
        st, _, body = http_get(host, port, "/metrics")
    except OSError:
        return ""
    return body.decode() if st == 200 else ""


def span_counters(host: str, port: int, probe: MetricsProbe | None = None) -> dict:
    """hola_spans_* counters from a replica's /metrics (empty with tracing off)."""
    out = {}
    for line in (probe.text() if probe else _metrics_text(host, port)).splitlines():
        if line.startswith("hola_spans_recorded_total "):
            out["recorded"] = int(float(line.split()[1]))
        elif line.startswith("hola_spans_reported_total "):
            out["reported"] = int(float(line.split()[1]))
        elif line.startswith("hola_spans_dropped_total{reason="):
            out["dropped_" + line.split('"')[1]] = int(float(line.rsplit(" ", 1)[1]))
    return out


def accept_locality(host: str, port: int, probe: MetricsProbe | None = None) -> dict:
    """hola_accept_locality_total from a replica's /metrics: where each accepted connection's
    client thread ran relative to the worker serving it (same_core / same_l3 / same_socket /
    cross_socket / unknown)."""
    out = {}
    for line in (probe.text() if probe else _metrics_text(host, port)).splitlines():
        if line.startswith("hola_accept_locality_total{relation="):
            out[line.split('"')[1]] = int(float(line.rsplit(" ", 1)[1]))
    return out


def thread_cpu_s(pid: int, name: str) -> float:
    """user+system CPU seconds of the thread of `pid` whose comm is `name` (0 if none)."""
    total = 0.0
    for task in Path(f"/proc/{pid}/task").glob("*"):
        try:
            if (task / "comm").read_text().strip() != name:
                continue
            fields = (task / "stat").read_text().rsplit(")", 1)[1].split()
            total += (int(fields[11]) + int(fields[12])) / os.sysconf("SC_CLK_TCK")
        except (OSError, IndexError, ValueError):
            pass
    return total


def proc_cpu_s(pid: int) -> float:
    """user+system CPU seconds of a process (all threads) from /proc/<pid>/stat."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            fields = f.read().rsplit(")", 1)[1].split()
        return (int(fields[11]) + int(fields[12])) / os.sysconf("SC_CLK_TCK")
    except (OSError, IndexError, ValueError):
        return 0.0


def cpu_times() -> dict[int, tuple[int, int, int, int]]:
    """Per-CPU (total, idle+iowait, irq+softirq, steal) jiffies from /proc/stat, host-wide
    (other tenants included). The guest columns are already inside user/nice, so they are
    left out of the total."""
    out = {}
    try:
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("cpu") and line[3].isdigit():
                    parts = line.split()
                    v = list(map(int, parts[1:9]))  # user nice system idle iowait irq softirq steal
                    v += [0] * (8 - len(v))
                    out[int(parts[0][3:])] = (sum(v), v[3] + v[4], v[5] + v[6], v[7])
    except (OSError, ValueError, IndexError):
        pass
    return out


def _share(t0: dict, t1: dict, cpus, col: int) -> float | None:
    tot = part = 0
    for c in cpus:
        if c in t0 and c in t1:
            tot += t1[c][0] - t0[c][0]
            part += t1[c][col] - t0[c][col]
    return round(part / tot, 4) if tot > 0 else None


def busy_fraction(t0: dict, t1: dict, cpus) -> float | None:
    """Busy share of `cpus` between two cpu_times() snapshots (None when unknown)."""
    idle = _share(t0, t1, cpus, 1)
    return None if idle is None else round(1.0 - idle, 4)


def irq_fraction(t0: dict, t1: dict, cpus) -> float | None:
    """Share of `cpus`' time in hard and soft interrupt context (on loopback: the receive path
    of segments this job sent, when the kernel defers it to softirq, and other devices' IRQs)."""
    return _share(t0, t1, cpus, 2)


def steal_fraction(t0: dict, t1: dict, cpus) -> float | None:
    """Share of `cpus`' time a hypervisor ran something else (0 on bare metal)."""
    return _share(t0, t1, cpus, 3)


def busy_cpu_s(t0: dict, t1: dict, cpus) -> float:
    """CPU-seconds `cpus` were busy between two cpu_times() snapshots (any task, IRQs included)."""
    tck = os.sysconf("SC_CLK_TCK")
    return sum((t1[c][0] - t0[c][0]) - (t1[c][1] - t0[c][1]) for c in cpus if c in t0 and c in t1) / tck


_KSOFTIRQD: dict[int, int] = {}


def ksoftirqd_cpu_s(cpus) -> float:
    """CPU-seconds used so far by the ksoftirqd threads of `cpus`: softirq work the kernel
    deferred to a thread (it then preempts whatever runs on that CPU)."""
    if not _KSOFTIRQD:
        for comm in Path("/proc").glob("[0-9]*/comm"):
            try:
                name = comm.read_text().strip()
            except OSError:
                continue
            if name.startswith("ksoftirqd/") and name[10:].isdigit():
                _KSOFTIRQD[int(name[10:])] = int(comm.parent.name)
    return sum(proc_cpu_s(_KSOFTIRQD[c]) for c in cpus if c in _KSOFTIRQD)


def task_stats(pid: int) -> dict[str, dict]:
    """Per thread of `pid` (by comm): CPU seconds, voluntary / involuntary context switches (a
    thread that sleeps in epoll_wait and is woken switches voluntarily; one preempted by another
    runnable task, involuntarily) and the scheduler's run_delay (ms it was runnable but waited
    for a CPU another task held; /proc/<pid>/task/<tid>/schedstat). Threads of one name are
    summed; `run_delay_max_ms` is the largest single thread's."""
    out: dict[str, dict] = {}
    tck = os.sysconf("SC_CLK_TCK")
    for task in Path(f"/proc/{pid}/task").glob("*"):
        try:
            comm = (task / "comm").read_text().strip()
            fields = (task / "stat").read_text().rsplit(")", 1)[1].split()
            vol = invol = 0
            try:
                delay_ms = int((task / "schedstat").read_text().split()[1]) / 1e6
            except (OSError, IndexError, ValueError):
                delay_ms = 0.0
            for ln in (task / "status").read_text().splitlines():
                if ln.startswith("voluntary_ctxt_switches:"):
                    vol = int(ln.split()[1])
                elif ln.startswith("nonvoluntary_ctxt_switches:"):
                    invol = int(ln.split()[1])
        except (OSError, IndexError, ValueError):
            continue
        d = out.setdefault(comm, {"cpu_s": 0.0, "vol": 0, "invol": 0, "threads": 0, "run_delay_ms": 0.0,
                                  "per_tid": {}})
        d["cpu_s"] += (int(fields[11]) + int(fields[12])) / tck
        d["vol"] += vol
        d["invol"] += invol
        d["threads"] += 1
        d["run_delay_ms"] += delay_ms
        d["per_tid"][task.name] = delay_ms
    return out


def task_stats_delta(a: dict, b: dict, group=lambda comm: "workers" if comm.startswith(("hola-w", "hola-lg"))
                     else "other") -> dict:
    """task_stats(b) - task_stats(a), summed into groups (default: the serving threads, hola-w*
    or hola-lg*, and every other thread of the process)."""
    out: dict[str, dict] = {}
    for comm, d1 in b.items():
        d0 = a.get(comm, {"cpu_s": 0.0, "vol": 0, "invol": 0, "run_delay_ms": 0.0, "per_tid": {}})
        g = out.setdefault(group(comm), {"cpu_s": 0.0, "vol": 0, "invol": 0, "run_delay_ms": 0.0,
                                         "run_delay_max_thread_ms": 0.0})
        g["cpu_s"] = round(g["cpu_s"] + d1["cpu_s"] - d0["cpu_s"], 3)
        g["vol"] += d1["vol"] - d0["vol"]
        g["invol"] += d1["invol"] - d0["invol"]
        g["run_delay_ms"] = round(g["run_delay_ms"] + d1.get("run_delay_ms", 0.0) - d0.get("run_delay_ms", 0.0), 3)
        for tid, v in d1.get("per_tid", {}).items():
            dt = v - d0.get("per_tid", {}).get(tid, 0.0)
            g["run_delay_max_thread_ms"] = round(max(g["run_delay_max_thread_ms"], dt), 3)
    return out


def cgroup_cpu_stat() -> dict[str, int]:
    """cgroup v2 cpu.stat counters of this process's cgroup (empty when unavailable)."""
    try:
        rel = next((l[3:] for l in Path("/proc/self/cgroup").read_text().splitlines() if l.startswith("0::")), "/")
        for path in (Path("/sys/fs/cgroup") / rel.lstrip("/") / "cpu.stat", Path("/sys/fs/cgroup/cpu.stat")):
            if path.exists():
                return {k: int(v) for k, v in (l.split() for l in path.read_text().splitlines() if l.strip())}
    except (OSError, IndexError, ValueError):
        pass
    return {}


def tcp_counters() -> dict[str, int]:
    """Network-namespace-wide TCP counters (/proc/net/snmp `Tcp:`, /proc/net/netstat
    `TcpExt:`): segments, and the ACK counts that show whether ACKs ride on the request and
    response segments or travel as extra pure-ACK packets through the loopback path."""
    want = {"Tcp": ("OutSegs", "InSegs", "RetransSegs"),
            "TcpExt": ("DelayedACKs", "TCPPureAcks", "TCPHPAcks", "TCPAutoCorking")}
    out: dict[str, int] = {}
    for path in ("/proc/net/snmp", "/proc/net/netstat"):
        try:
            with open(path) as f:
                lines = f.read().splitlines()
        except OSError:
            continue
        for names, vals in zip(lines[::2], lines[1::2]):
            group = names.split(":", 1)[0]
            if group not in want:
                continue
            row = dict(zip(names.split()[1:], vals.split()[1:]))
            for field in want[group]:
                if row.get(field, "").lstrip("-").isdigit():
                    out[field] = int(row[field])
    return out
