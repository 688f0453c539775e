#!/usr/bin/env python3
"""Throughput of the chaining path with a native downstream: load generator ->
hola A `/api/hola-chaining` -> hola B `/api/hola-chaining`. B plays aloha: its JSON list
(`["Hola de B", "Aloha response (fallback)"]`, its own aloha being unreachable) is what A
decodes as `List<String>`.

Every request crosses two HTTP hops, A's per-worker keep-alive client pool, the Hystrix
command (breaker + bulkhead + 600 ms timer) and B3 propagation. The bulkhead is widened
with --pool so it measures the path rather than the (intentionally tiny) default of 10.

    python bench/chain_bench.py --duration 10 [--pool 128]
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from hola_amd.parallel.loadgen import run_duration  # noqa: E402
from hola_amd.server import HolaProcess  # noqa: E402
from hola_amd.utils.cpu import format_cpu_list, plan_mirrored  # noqa: E402

ap = argparse.ArgumentParser(description=__doc__)
ap.add_argument("--duration", type=float, default=10)
ap.add_argument("--connections", type=int, default=64)
ap.add_argument("--pool", type=int, default=128, help="hystrix thread-pool (bulkhead) size on A")
ap.add_argument("--feign-log", default="none", choices=("none", "basic"),
                help="A's Feign logging; basic = the reference's ErrorLogger at Level.BASIC (two stderr "
                     "lines per call, the server's default)")
ap.add_argument("--aloha-pipeline", type=int, default=1,
                help="A's --aloha-pipeline (HTTP/1.1 pipelining of concurrent calls to B; 1 = off)")
ap.add_argument("--cpu-profile", default="",
                help="run A with --cpu-profile here (sampled call stacks; bench/cpuprof_report.py reads it)")
ap.add_argument("--out", default="")
ap.add_argument("--exe-a", default="", help="alternative hola binary for A (A/B runs)")
a = ap.parse_args()



def cpu_split(pid: int) -> tuple[float, float]:
    """(utime, stime) of a process, in seconds."""
    f = Path(f"/proc/{pid}/stat").read_text().rsplit(")", 1)[1].split()
    tck = os.sysconf("SC_CLK_TCK")
    return int(f[11]) / tck, int(f[12]) / tck


def cpu_s(pid: int) -> float:
    """utime + stime of a process, in seconds."""
    return sum(cpu_split(pid))


# Every L3 domain holds a share of A, B and the load generator (A does two hops' work), so
# accept steering keeps loadgen->A and A->B connections inside one L3 each.
plan = plan_mirrored({"A": 2, "B": 1, "loadgen": 1})
cores = [plan["A"], plan["B"], plan["loadgen"]]
# B answers /api/hola-chaining itself with its own fallback (its aloha is unreachable and its
# breaker opens), so A decodes ["Hola de B", "Aloha response (fallback)"]. B does not retry
# its refused aloha (--feign-retry off): a retrying B would answer only at its 600 ms
# timeout until its breaker opens, and A's equal timeout would fall back first.
with HolaProcess(args=["--aloha-url", "http://127.0.0.1:1/", "--feign-log", "none", "--no-tracing",
                       "--feign-retry", "off", "--log-level", "warn"], env={"HOSTNAME": "B"}, threads=len(cores[1]),
                 cpu_list=format_cpu_list(cores[1])) as b:
    with HolaProcess(args=["--aloha-url", f"http://127.0.0.1:{b.port}/", "--aloha-path", "api/hola-chaining",
                           "--feign-log", a.feign_log, "--hystrix-pool-size", str(a.pool)]
                          + (["--cpu-profile", os.path.abspath(a.cpu_profile)] if a.cpu_profile else [])
                          + (["--aloha-pipeline", str(a.aloha_pipeline)] if a.aloha_pipeline > 1 else []),
                     env={"HOSTNAME": "A"}, threads=len(cores[0]), cpu_list=format_cpu_list(cores[0]),
                     # BASIC logging writes ~150 bytes per call: at 1.5 M calls/s that would be
                     # gigabytes of log file per run, so A's stderr goes to /dev/null
                     stderr_path=os.devnull if a.feign_log == "basic" else None,
                     exe=Path(a.exe_a) if a.exe_a else None) as s:
        st, _, body = s.get("/api/hola-chaining")
        assert st == 200, body
        sample = json.loads(body)
        assert sample[1:] == ["Hola de B", "Aloha response (fallback)"], sample  # two hops, no fallback at A
        c0, w0 = (cpu_s(s.proc.pid), cpu_s(b.proc.pid)), time.perf_counter()
        u0 = (cpu_split(s.proc.pid), cpu_split(b.proc.pid))
        # every response must be the two-hop body seen above (a fallback would differ)
        res = run_duration([("127.0.0.1", s.port)], a.connections, len(cores[2]), a.duration, 2.0,
                           cpu_list=format_cpu_list(cores[2]), path="/api/hola-chaining",
                           expect_bodies=[body.decode()])
        wall = time.perf_counter() - w0
        busy = {"A": (cpu_s(s.proc.pid) - c0[0]) / wall, "B": (cpu_s(b.proc.pid) - c0[1]) / wall}
        u1 = (cpu_split(s.proc.pid), cpu_split(b.proc.pid))
        # user-space share of each process's CPU (the rest is the kernel: sockets, epoll)
        user_share = {k: round((u1[i][0] - u0[i][0]) / max(1e-9, sum(u1[i]) - sum(u0[i])), 3)
                      for i, k in enumerate(("A", "B"))}
        _, _, metrics = s.get("/metrics")
events = {l.split('event="')[1].split('"')[0]: int(l.split()[-1]) for l in metrics.decode().splitlines()
          if l.startswith("hola_hystrix_events_total")}
out = {"sample": sample, "rps": res["rps"], "p50_ms": res["latency"]["p50_ns"] / 1e6,
       "p99_ms": res["latency"]["p99_ns"] / 1e6, "errors": res["latency"]["errors"],
       "body_checked": res["latency"].get("body_checked", 0), "body_mismatch": res["latency"].get("body_mismatch", 0),
       "hystrix_events": events, "feign_log": a.feign_log, "aloha_pipeline": a.aloha_pipeline,
       # cores kept busy (warmup included) and CPU µs per request at the measured rate
       "cpus_busy": {k: round(v, 2) for k, v in busy.items()},
       "cpu_us_per_req": {k: round(v / res["rps"] * 1e6, 2) for k, v in busy.items()},
       "user_share": user_share,
       "cpu_map": {"A": format_cpu_list(cores[0]), "B": format_cpu_list(cores[1]), "loadgen": format_cpu_list(cores[2])}}
print(json.dumps(out))
if a.out:
    Path(a.out).write_text(json.dumps(out, indent=1))
