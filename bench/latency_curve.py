#!/usr/bin/env python3
"""Open-loop latency curve for GET /api/hola (wrk2-style): one pinned replica driven at fixed
request rates, latency measured from each request's *intended* send time, so queueing delay
is not hidden by coordinated omission. Complements the closed-loop headline in bench.py.

    python bench/latency_curve.py --rates 250000,1000000,2000000,3000000 --duration 8
"""
import argparse
import json
import os
import resource
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from hola_amd.parallel import subruns  # noqa: E402
from hola_amd.parallel.hostmetrics import (busy_cpu_s, cgroup_cpu_stat, cpu_times, ksoftirqd_cpu_s,  # noqa: E402
                                           task_stats, task_stats_delta)
from hola_amd.parallel.loadgen import run_duration  # noqa: E402
from hola_amd.server import HolaProcess  # noqa: E402
from hola_amd.utils.cpu import format_cpu_list, plan_node, split_server_loadgen  # noqa: E402

ap = argparse.ArgumentParser(description=__doc__)
ap.add_argument("--rates", default="250000,1000000,2000000,3000000,3500000")
ap.add_argument("--duration", type=float, default=8)
ap.add_argument("--connections", type=int, default=64)
ap.add_argument("--busy-poll-us", type=int, default=0, help="server and load generator spin in epoll this long")
ap.add_argument("--spin-us", type=int, default=1000,
                help="load generator polls instead of sleeping when its next send is this close (the default "
                     "keeps it on its CPUs: a generator that sleeps between sends leaves CPUs the scheduler "
                     "hands to other tasks, and its late wake-ups are charged to the server)")
ap.add_argument("--server-busy-poll", default="",
                help="the server's --busy-poll-us (N, auto or auto:N); default: --busy-poll-us")
ap.add_argument("--sched-slice-us", type=int, default=0,
                help="server workers and load-generator threads ask the scheduler for this time slice (0 = kernel default)")
ap.add_argument("--out", default="")
a = ap.parse_args()

cores = plan_node(1)[0]
srv, lg = split_server_loadgen(cores, max(1, len(cores) // 2))
rows = []
server_bp = a.server_busy_poll or str(a.busy_poll_us)
server_args = ["--busy-poll-us", server_bp]  # always explicit: hola's own default is auto
if a.sched_slice_us:
    server_args += ["--sched-slice-us", str(a.sched_slice_us)]
with HolaProcess(args=server_args, env={"HOSTNAME": "h"}, threads=len(srv), cpu_list=format_cpu_list(srv),
                 log_level="warn") as s:
    def server_cpu():
        with open(f"/proc/{s.proc.pid}/stat") as f:
            v = f.read().rsplit(")", 1)[1].split()
        return (int(v[11]) + int(v[12])) / os.sysconf("SC_CLK_TCK")

    job = list(srv) + list(lg)
    probe = subruns.MetricsProbe("127.0.0.1", s.port)
    for rate in [float(x) for x in a.rates.split(",")]:
        c0 = resource.getrusage(resource.RUSAGE_CHILDREN)
        s0 = server_cpu()
        # what a tail could come from, recorded per point: the replica's
        # spin / back-off / resume transitions and gaps between its polls, its workers'
        # involuntary switches (preempted by another task), CFS throttling of the cgroup, the
        # host load (IRQ time, siblings, L3 neighbours) of both sides, and the load
        # generator's own gaps and late sends
        m0, ts0, thr0, t0 = subruns.metrics_counters(s.port, probe=probe), task_stats(s.proc.pid), cgroup_cpu_stat(), cpu_times()
        k0 = ksoftirqd_cpu_s(srv)
        r = run_duration([("127.0.0.1", s.port)], a.connections, len(lg), a.duration, 2.0,
                         cpu_list=",".join(map(str, lg)), rate=rate, busy_poll_us=a.busy_poll_us,
                         spin_us=a.spin_us, verify_body=True, sched_slice_us=a.sched_slice_us)
        m1, ts1, thr1, t1 = subruns.metrics_counters(s.port, probe=probe), task_stats(s.proc.pid), cgroup_cpu_stat(), cpu_times()
        k1 = ksoftirqd_cpu_s(srv)
        c1 = resource.getrusage(resource.RUSAGE_CHILDREN)
        s1 = server_cpu()
        wall = a.duration + 2.0  # warmup included in both CPU figures
        lat = r["latency"]
        reqs = max(1.0, r["rps"] * a.duration)
        row = {"target_rps": rate, "achieved_rps": r["rps"], "p50_us": lat["p50_ns"] / 1e3,
               "p90_us": lat["p90_ns"] / 1e3, "p99_us": lat["p99_ns"] / 1e3, "p999_us": lat["p999_ns"] / 1e3,
               "max_us": lat["max_ns"] / 1e3, "errors": lat["errors"],
               # service time: each response's send() to its arrival in the client host's kernel
               # (receive timestamp), so none of the generator's own delays (a late send, a late
               # read) is in it; the open-loop figures above charge those to the server
               "service_us": ({k: lat[f"service_{k}_ns"] / 1e3 for k in ("p50", "p99", "p999", "max")}
                              if lat.get("service_count") else None),
               "server_cpus_busy": round((s1 - s0) / wall, 2),
               "loadgen_cpus_busy": round((c1.ru_utime + c1.ru_stime - c0.ru_utime - c0.ru_stime) / wall, 2),
               "server_loop": subruns.loop_block(m0, m1, reqs),
               "server_threads": task_stats_delta(ts0, ts1),
               # what else ran on the replica's CPUs: their busy CPU-seconds less the replica's
               # own (other tasks: kernel threads, other tenants), and the part of it that was
               # ksoftirqd (softirq work deferred to a thread that preempts the worker)
               "foreign_on_server_cpus_s": round(busy_cpu_s(t0, t1, srv) - (s1 - s0), 3),
               "ksoftirqd_on_server_cpus_s": round(k1 - k0, 3),
               # ... and on the load generator's CPUs (its own CPU from its rusage): a late
               # send with other tasks there was this generator waiting for its CPU
               "foreign_on_loadgen_cpus_s": round(busy_cpu_s(t0, t1, lg) - (c1.ru_utime + c1.ru_stime
                                                                         - c0.ru_utime - c0.ru_stime), 3),
               "cgroup_throttle": {"periods": thr1.get("nr_periods", 0) - thr0.get("nr_periods", 0),
                                   "throttled_periods": thr1.get("nr_throttled", 0) - thr0.get("nr_throttled", 0),
                                   "throttled_ms": round((thr1.get("throttled_usec", 0) - thr0.get("throttled_usec", 0)) / 1e3, 1)},
               "host_load_server": subruns.host_load(t0, t1, srv, job),
               "host_load_loadgen": subruns.host_load(t0, t1, lg, job),
               "loadgen": {k: lat.get(k) for k in ("gaps_over_100us", "gaps_over_1ms", "gaps_over_10ms", "gap_max_ns",
                                                   "send_late_max_ns", "sends_late_1ms", "behind_max_ns",
                                                   "blocking_waits", "run_delay_ns", "run_delay_max_thread_ns")}}
        rows.append(row)
        print(json.dumps(row), flush=True)
    probe.close()
out = {"cpu_map": {"server": format_cpu_list(srv), "loadgen": format_cpu_list(lg)}, "connections": a.connections,
       "busy_poll_us": a.busy_poll_us, "server_busy_poll": server_bp, "server_args": server_args, "spin_us": a.spin_us,
       "sched_slice_us": a.sched_slice_us, "rows": rows}
if a.out:
    Path(a.out).write_text(json.dumps(out, indent=1))
