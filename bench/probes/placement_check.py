#!/usr/bin/env python3
"""Where the threads of a miniature-plan scaling point actually run (diagnostic).

Starts N replicas and one load generator as `hola_amd.parallel.scaling --slot-cores K` plans
them, drives them for a moment, then prints each replica's worker threads with the CPU they
last ran on and their affinity, each load-generator thread likewise, and each replica's
accept-locality counters. For a point whose locality says the clients are not on their
workers' cores, this tells whether the threads are misplaced or the counters are.

    python bench/probes/placement_check.py --replicas 4 [--slots 8] [--slot-cores 1]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[2]))

from hola_amd.parallel.hostmetrics import MetricsProbe  # noqa: E402
from hola_amd.parallel.loadgen import ControlledLoadgen  # noqa: E402
from hola_amd.parallel.replicas import ReplicaSet  # noqa: E402
from hola_amd.parallel.scaling import plan_slots  # noqa: E402
from hola_amd.parallel.subruns import metrics_counters  # noqa: E402


def threads_of(pid: int) -> list[dict]:
    out = []
    for task in sorted(Path(f"/proc/{pid}/task").iterdir(), key=lambda p: int(p.name)):
        try:
            name = (task / "comm").read_text().strip()
            stat = (task / "stat").read_text().rsplit(")", 1)[1].split()
            aff = next(l.split(":", 1)[1].strip() for l in (task / "status").read_text().splitlines()
                       if l.startswith("Cpus_allowed_list"))
            out.append({"tid": int(task.name), "name": name, "last_cpu": int(stat[36]), "allowed": aff})
        except (OSError, StopIteration, IndexError, ValueError):
            pass
    return out


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--replicas", type=int, default=4)
    ap.add_argument("--slots", type=int, default=8)
    ap.add_argument("--slot-cores", type=int, default=1)
    a = ap.parse_args()
    p = plan_slots(a.replicas, a.slot_cores, a.slots, "client")
    print(json.dumps({"plan": p}))
    with ReplicaSet(a.replicas, cpu_plan=p["replicas"], args=["--busy-poll-us", "auto", "--busy-poll-pause", "16"],
                    supervise=False) as rs:
        probes = [MetricsProbe("127.0.0.1", port) for port in rs.ports]
        m0 = [metrics_counters(0, probe=pr) for pr in probes]
        lg = ControlledLoadgen(rs.targets, 64 * a.replicas, len(p["loadgen"]), cpu_list=",".join(map(str, p["loadgen"])),
                               busy_poll_us=20, busy_poll_pause=16, verify_body=True)
        try:
            for _ in range(5):
                lg.run(2000)
            print(json.dumps({"loadgen_cmd_cpu_list": ",".join(map(str, p["loadgen"])),
                              "loadgen_threads": threads_of(lg.proc.pid)}))
            for i, pr in enumerate(rs.procs):
                m1 = metrics_counters(0, probe=probes[i])
                loc = {k: int(m1[k] - m0[i].get(k, 0)) for k in m1 if k.startswith("locality.") and m1[k] - m0[i].get(k, 0)}
                print(json.dumps({"replica": i, "port": rs.ports[i], "planned_cpus": p["replicas"][i],
                                  "threads": [t for t in threads_of(pr.proc.pid) if t["name"].startswith("hola-w")],
                                  "locality": loc}))
        finally:
            lg.close()
            for pr in probes:
                pr.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
