#!/usr/bin/env python3
"""Tail attribution table of open-loop latency curves (bench/latency_curve.py output files).

For every point with p99.9 above --threshold-us it names what the point's own record shows
(VERDICT r5 weak #2):

  gaps       the replica's loops went more than 1 ms between two polls (a handler that ran
             long, or the thread descheduled: then it also has involuntary switches)
  preempted  the replica's workers were switched out involuntarily (another task on their CPU)
  cpu-wait   the scheduler's run_delay of the replica's workers: time they were runnable but
             waited for a CPU another task held (total, and the most any one worker waited)
  lg-cpu-wait the same for the load generator's threads
  throttled  CFS bandwidth throttling of the cgroup (every thread stops until the next period)
  late       the load generator sent a scheduled request more than 1 ms late although its
             connection was free at the due time: its own stall, which the open loop charges
             to the server (latency is counted from the intended time)
  behind     a connection was still waiting for the server's previous answer more than 1 ms
             past the next request's due time (the server's delay)
  foreign    other tasks (kernel threads, other tenants) used the replica's CPUs for more
             than 1 % of the point; ksoftirqd is named apart (lg-foreign: the load generator's)
  lg-gaps    the load generator's threads went more than 1 ms between polls
  irq/steal  interrupt or hypervisor time on the replica's CPUs above 5 %
  neighbours other tenants on the SMT siblings or elsewhere in the L3 above 5 %

and the point's service-time p99.9 (send() to the response's kernel receive timestamp at the
client: the server's and the network's time with none of the generator's own delays). A point
whose open-loop p99.9 is over the threshold while its service p99.9 is not had its tail made
by the load generator (a late send or a late read), not by the server.

    python bench/tail_report.py gpurun_out/r6_06_tails/curve_*.json [--threshold-us 100]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path


def causes(row: dict) -> list[str]:
    out = []
    loop = row.get("server_loop", {})
    if loop.get("gaps_over_1ms", 0):
        out.append(f"gaps({loop['gaps_over_1ms']} >1ms, {loop.get('gaps_over_10ms', 0)} >10ms)")
    invol = sum(g.get("invol", 0) for g in row.get("server_threads", {}).values())
    if invol:
        out.append(f"preempted({invol})")
    w = row.get("server_threads", {}).get("workers", {})
    if (w.get("run_delay_ms") or 0) > 1.0:
        out.append(f"cpu-wait({w['run_delay_ms']:.1f} ms, max thread {w.get('run_delay_max_thread_ms', 0):.1f} ms)")
    thr = row.get("cgroup_throttle", {})
    if thr.get("throttled_periods", 0):
        out.append(f"throttled({thr['throttled_periods']} periods, {thr.get('throttled_ms', 0)} ms)")
    lg = row.get("loadgen", {})
    if (lg.get("send_late_max_ns") or 0) > 1_000_000:
        n = lg.get("sends_late_1ms")
        out.append(f"late({lg['send_late_max_ns'] / 1e3:.0f} us" + (f", {n} sends >1ms" if n is not None else "") + ")")
    if (lg.get("behind_max_ns") or 0) > 1_000_000:
        out.append(f"behind({lg['behind_max_ns'] / 1e3:.0f} us)")
    if (lg.get("run_delay_ns") or 0) > 1_000_000:
        out.append(f"lg-cpu-wait({lg['run_delay_ns'] / 1e6:.1f} ms, max thread {(lg.get('run_delay_max_thread_ns') or 0) / 1e6:.1f} ms)")
    fs, ks = row.get("foreign_on_server_cpus_s"), row.get("ksoftirqd_on_server_cpus_s")
    if fs is not None and fs > 0.01 * 8:  # 1 % of 8 CPUs over the 8 s point
        out.append(f"foreign({fs:.2f} CPU-s" + (f", ksoftirqd {ks:.2f}" if ks else "") + ")")
    fl = row.get("foreign_on_loadgen_cpus_s")
    if fl is not None and fl > 0.01 * 8:
        out.append(f"lg-foreign({fl:.2f} CPU-s)")
    if lg.get("gaps_over_1ms", 0):
        out.append(f"lg-gaps({lg['gaps_over_1ms']} >1ms, max {lg.get('gap_max_ns', 0) / 1e3:.0f} us)")
    hl = row.get("host_load_server", {})
    for k, name in (("irq_own", "irq"), ("steal_own", "steal")):
        if (hl.get(k) or 0) > 0.05:
            out.append(f"{name}({hl[k]:.2f})")
    for k in ("siblings", "l3_others"):
        if (hl.get(k) or 0) > 0.05:
            out.append(f"neighbours-{k}({hl[k]:.2f})")
    return out


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("curves", nargs="+")
    ap.add_argument("--threshold-us", type=float, default=100.0)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    report = []
    print(f"| curve | target | achieved | p99 µs | p99.9 µs | max µs | service p99.9 µs | server CPUs | attributed to |")
    print("|---|---|---|---|---|---|---|---|---|")
    for path in a.curves:
        d = json.loads(Path(path).read_text())
        name = Path(path).stem
        for row in d["rows"]:
            tail = row["p999_us"] > a.threshold_us
            c = causes(row)
            svc = (row.get("service_us") or {}).get("p999")
            if tail and svc is not None and svc <= a.threshold_us:
                c.insert(0, f"GENERATOR (service p99.9 {svc:.1f} us)")
            report.append({"curve": name, "server_busy_poll": d.get("server_busy_poll"), "target_rps": row["target_rps"],
                           "p99_us": row["p99_us"], "p999_us": row["p999_us"], "max_us": row["max_us"],
                           "service_p999_us": svc, "over_threshold": tail,
                           "server_over_threshold": tail and (svc is None or svc > a.threshold_us), "causes": c})
            mark = "**" if tail else ""
            print(f"| {name} | {row['target_rps'] / 1e6:g} M | {row['achieved_rps'] / 1e6:.3f} M | {row['p99_us']:.1f} | "
                  f"{mark}{row['p999_us']:.1f}{mark} | {row['max_us']:.0f} | "
                  f"{'—' if svc is None else f'{svc:.1f}'} | {row['server_cpus_busy']} | "
                  f"{', '.join(c) if c else ('—' if not tail else 'nothing recorded')} |")
    if a.json:
        Path(a.json).write_text(json.dumps(report, indent=1))
    unexplained = [r for r in report if r["over_threshold"] and not r["causes"]]
    print(f"\n{sum(r['over_threshold'] for r in report)} points over {a.threshold_us:g} us, "
          f"{len(unexplained)} with nothing recorded; "
          f"{sum(r['server_over_threshold'] for r in report)} with the service time over it too")
    return 0


if __name__ == "__main__":
    sys.exit(main())
