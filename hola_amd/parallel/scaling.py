"""Replica scaling curve for GET /api/hola on one node (BASELINE.json configs 2-4).

    python -m hola_amd.parallel.scaling --replicas 1,2,4,8 --duration 10 [--lb client|proxy]

For each replica count N the host CPU budget is split into disjoint core sets: one per
replica (server event loops) plus one for the load generator (and the proxy, with
``--lb proxy``). ``--mode weak`` keeps 64 connections per replica (512 at N=8, config 4);
``--mode strong`` uses a fixed total (``--connections``). Every row records the core map and
the load-balancing mechanism, as BASELINE.md requires.
"""
from __future__ import annotations

import argparse
import json
import sys
import time

from hola_amd.parallel.loadgen import run_duration
from hola_amd.parallel.replicas import ReplicaSet, RRProxy
from hola_amd.utils.cpu import cgroup_cpu_quota, cpu_budget, format_cpu_list, physical_cores, allowed_cpus


def plan(n_replicas: int, budget: int, server_share: float, proxy_threads: int) -> dict:
    cores = physical_cores()
    if len(cores) < budget:
        cores = allowed_cpus()
    cores = cores[:budget]
    n_server = max(n_replicas, int(round(budget * server_share)))
    n_server = min(n_server, budget - 1 - proxy_threads)
    per = max(1, n_server // n_replicas)
    replica_cpus = [cores[i * per:(i + 1) * per] for i in range(n_replicas)]
    used = per * n_replicas
    proxy_cpus = cores[used:used + proxy_threads] if proxy_threads else []
    load_cpus = cores[used + proxy_threads:] or cores[-1:]
    return {"replicas": replica_cpus, "proxy": proxy_cpus, "loadgen": load_cpus}


def run_point(n: int, args) -> dict:
    budget = args.budget or cpu_budget()
    proxy_threads = args.proxy_threads if args.lb == "proxy" else 0
    p = plan(n, budget, args.server_share, proxy_threads)
    conns = args.connections_per_replica * n if args.mode == "weak" else args.connections
    extra = ["--no-tracing"] if args.no_tracing else []
    with ReplicaSet(n, cpu_plan=p["replicas"], args=extra, supervise=False) as rs:
        if args.lb == "proxy":
            with RRProxy(rs.targets, threads=proxy_threads, cpu_list=format_cpu_list(p["proxy"])) as px:
                targets = [("127.0.0.1", px.port)]
                res = run_duration(targets, conns, len(p["loadgen"]), args.duration, args.warmup,
                                   cpu_list=format_cpu_list(p["loadgen"]))
        else:
            res = run_duration(rs.targets, conns, len(p["loadgen"]), args.duration, args.warmup,
                               cpu_list=format_cpu_list(p["loadgen"]))
    lat = res["latency"]
    return {
        "replicas": n, "connections": conns, "lb": args.lb, "rps": res["rps"],
        "p50_ms": lat["p50_ns"] / 1e6, "p99_ms": lat["p99_ns"] / 1e6, "p999_ms": lat["p999_ns"] / 1e6,
        "errors": lat["errors"], "non2xx": lat["non2xx"],
        "cpu_map": {"replicas": [format_cpu_list(c) for c in p["replicas"]], "proxy": format_cpu_list(p["proxy"]),
                    "loadgen": format_cpu_list(p["loadgen"])},
        "budget": budget, "quota": cgroup_cpu_quota(), "duration_s": args.duration,
    }


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--replicas", default="1,2,4,8")
    ap.add_argument("--duration", type=float, default=10.0)
    ap.add_argument("--warmup", type=float, default=2.0)
    ap.add_argument("--mode", choices=["weak", "strong"], default="weak")
    ap.add_argument("--connections-per-replica", type=int, default=64)
    ap.add_argument("--connections", type=int, default=512)
    ap.add_argument("--lb", choices=["client", "proxy"], default="client")
    ap.add_argument("--proxy-threads", type=int, default=2)
    ap.add_argument("--budget", type=int, default=0, help="CPUs to use (default: cgroup quota / affinity)")
    ap.add_argument("--server-share", type=float, default=0.5)
    ap.add_argument("--no-tracing", action="store_true")
    ap.add_argument("--out", default="")
    args = ap.parse_args(argv)
    rows = []
    for n in [int(x) for x in args.replicas.split(",")]:
        row = run_point(n, args)
        rows.append(row)
        print(json.dumps(row), flush=True)
        time.sleep(0.5)
    base = rows[0]["rps"] / rows[0]["replicas"] if rows else 0
    table = ["| replicas | connections | LB | req/s | p50 ms | p99 ms | per-replica vs N=1 |",
             "|---|---|---|---|---|---|---|"]
    for r in rows:
        eff = (r["rps"] / r["replicas"]) / base if base else 0
        table.append(f"| {r['replicas']} | {r['connections']} | {r['lb']} | {r['rps']:.0f} | {r['p50_ms']:.3f} | "
                     f"{r['p99_ms']:.3f} | {eff:.2f} |")
    print("\n".join(table))
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"rows": rows, "table": table}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
