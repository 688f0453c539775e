"""Replica scaling curve for GET /api/hola on one node (BASELINE.json configs 2-4).

    python -m hola_amd.parallel.scaling --replicas 1,2,4,8 --duration 10 [--lb client|proxy|reuseport]
    python -m hola_amd.parallel.scaling --slot-cores 1 --slots 8 --lb client|reuseport|proxy

With ``--slot-cores K`` the plan is a miniature of the 8-GPU node's (``--slots``): replica k
runs on the first K physical cores of node slot k, placed where the node plan puts the slot
(both sockets), one server worker per core and the load-generator thread that drives it on
the core's other SMT thread; with ``--lb proxy`` the proxy gets K more physical cores of the
same slot (both SMT threads). Each N then gets exactly N times the resources of N = 1, so
the weak-scaling efficiency total(N) / (N x total(1)) is measurable inside a small CPU quota.
It is not the 8-GPU node's curve (16 cores per slot there).

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

from hola_amd.parallel.hostmetrics import MetricsProbe, busy_fraction, cpu_times, proc_cpu_s
from hola_amd.parallel.loadgen import ControlledLoadgen
from hola_amd.parallel.subruns import counter_delta, locality_fraction, metrics_counters, timed_closed_loop
from hola_amd.parallel.replicas import ReplicaSet, RRProxy
from hola_amd.utils.cpu import (cgroup_cpu_quota, cpu_budget, format_cpu_list, plan_mirrored, plan_node,
                                plan_slot_subset, sibling_of, split_server_loadgen)


def plan(n_replicas: int, budget: int, server_share: float, proxy_threads: int) -> dict:
    """Cores for N replicas + one load generator (+ proxy) inside `budget` CPUs.

    Each replica gets an equal slice of the quietest L3 domains, split between its server
    loops and the load-generator threads that drive it: the generator deals connection i to
    thread i % T and replica i % N, so thread t is placed in replica (t % N)'s L3 domain.
    """
    usable = budget - proxy_threads
    per = max(2, usable // n_replicas) if usable >= 2 * n_replicas else max(1, usable // n_replicas)
    slices = plan_node(n_replicas + (1 if proxy_threads else 0), per_rank=per)
    replica_cpus, load_by_replica = [], []
    for k in range(n_replicas):
        cores = slices[k]
        if len(cores) > 1:
            srv, lg = split_server_loadgen(cores, max(1, int(round(len(cores) * server_share))))
        else:
            srv, lg = cores, cores
        replica_cpus.append(srv)
        load_by_replica.append(lg)
    load = []
    t = 0
    while any(load_by_replica):
        k = t % n_replicas
        if load_by_replica[k]:
            load.append(load_by_replica[k].pop(0))
        t += 1
        if t > 10000:
            break
    proxy_cpus = slices[-1][:proxy_threads] if proxy_threads else []
    return {"replicas": replica_cpus, "proxy": proxy_cpus, "loadgen": load}


def plan_proxied(n_replicas: int, budget: int) -> dict:
    """Cores for load generator -> proxy -> N replicas: every L3 domain holds servers, proxy
    threads and load-generator threads in 1:2:1 (a proxied request costs the proxy two socket
    hops, about twice the server's work). The proxy hands each client connection to a thread in
    the client's L3, and that thread's backend connection lands on a server worker in its own
    L3 (accept steering), so no hop crosses an L3 domain. Server cores are dealt to replicas
    round-robin."""
    m = plan_mirrored({"server": 1, "proxy": 2, "loadgen": 1}, total=budget)
    srv = m["server"]
    replicas = [srv[k::n_replicas] or [srv[k % len(srv)]] for k in range(n_replicas)]
    return {"replicas": replicas, "proxy": m["proxy"], "loadgen": m["loadgen"]}


def plan_slots(n: int, k: int, slots: int, lb: str) -> dict:
    """The miniature node plan (see the module docstring): replicas on slot cores, load
    generator thread t on the sibling of replica (t % n)'s core t // n (connection i runs on
    thread i % T against target i % n, so thread t drives replica t % n), proxy threads on
    both SMT threads of the slot's next k cores."""
    sub = plan_slot_subset(n, slots, k, "auto", extra_cores=k if lb == "proxy" else 0)
    load = [sub[t % n]["loadgen"][t // n] for t in range(n * k)]
    proxy = []
    for p in sub:
        for c in p["extra"]:
            proxy += [c] + ([sibling_of(c)] if sibling_of(c) is not None else [])
    return {"replicas": [p["server"] for p in sub], "proxy": proxy, "loadgen": load,
            "slots": [p["slot"] for p in sub], "smt": sub[0]["smt"] if sub else "pair"}


def _measure(targets, conns: int, load_cpus: list[int], args, verify: bool,
             conn_targets: list[int] | None = None) -> dict:
    """A closed-loop run of args.duration after args.warmup, in the load generator's control
    mode: every connection is made before any request is sent (as bench.py runs it), then
    warm-up and measurement run as one continuous run (`runfor`). In wrk-style duration mode
    each thread started sending as soon as its own connections were up, and connections made
    while others were already loaded were placed off their client's core (per-replica locality
    all `same_socket` in some runs, profiles/round5/04_scale_mini)."""
    lg = ControlledLoadgen(targets, conns, len(load_cpus), cpu_list=",".join(map(str, load_cpus)),
                           busy_poll_us=args.busy_poll_us, busy_poll_pause=args.busy_poll_pause, verify_body=verify,
                           conn_targets=conn_targets)
    try:
        r = timed_closed_loop(lg, conns, args.duration, None, [], [], warm_s=args.warmup)
    finally:
        lg.close()
    return {"rps": r["rps"], "latency": {"p50_ns": r["p50_ns"], "p99_ns": r["p99_ns"], "p999_ns": r.get("p999_ns", 0),
                                         "errors": r["errors"], "non2xx": r["non2xx"],
                                         "body_mismatch": r["body_mismatch"]}}


def run_point(n: int, args) -> dict:
    budget = args.budget or cpu_budget()
    if args.slot_cores:
        p = plan_slots(n, args.slot_cores, args.slots, args.lb)
        proxy_threads = len(p["proxy"])
    elif args.lb == "proxy" and not args.proxy_threads:
        p = plan_proxied(n, budget)
        proxy_threads = len(p["proxy"])
    else:
        proxy_threads = args.proxy_threads if args.lb == "proxy" else 0
        p = plan(n, budget, args.server_share, proxy_threads)
    conns = args.connections_per_replica * n if args.mode == "weak" else args.connections
    extra = ["--no-tracing"] if args.no_tracing else []
    server_bp = args.server_busy_poll or (str(args.busy_poll_us) if args.busy_poll_us else "")
    if server_bp and server_bp != "0":
        extra += ["--busy-poll-us", server_bp]
        if args.busy_poll_pause:
            extra += ["--busy-poll-pause", str(args.busy_poll_pause)]
    shared = 0 if args.lb == "reuseport" else None
    reuseport_cpu = args.reuseport_cpu
    if reuseport_cpu == "auto":  # the client runs on the worker's SMT sibling in the pair plan
        reuseport_cpu = "sibling" if args.slot_cores and p.get("smt") == "pair" else "none"
    if shared is not None and reuseport_cpu != "none":
        extra += ["--reuseport-cpu", reuseport_cpu]
    hints = args.proxy_hints == "on" or (args.proxy_hints == "auto" and bool(args.slot_cores))
    with ReplicaSet(n, cpu_plan=p["replicas"], args=extra, supervise=False, shared_port=shared) as rs:
        # per replica: requests served and where each accepted connection's client ran, read
        # over kept-alive /metrics connections (reuseport: one shared port, so no per-replica view)
        probes = [MetricsProbe("127.0.0.1", port) for port in rs.ports] if shared is None else []
        m0 = [metrics_counters(0, probe=pr) for pr in probes]
        cpu0 = [proc_cpu_s(pr.proc.pid) for pr in rs.procs]
        t0 = cpu_times()
        if args.lb == "proxy":
            with RRProxy(rs.targets, threads=proxy_threads, cpu_list=format_cpu_list(p["proxy"]),
                         busy_poll_us=args.busy_poll_us if args.proxy_busy_poll_us < 0 else args.proxy_busy_poll_us,
                         exe=args.proxy_exe or None, backend_cpus=p["replicas"] if hints else None) as px:
                res = _measure([("127.0.0.1", px.port)], conns, p["loadgen"], args, verify=False)
        elif args.lb == "plain":
            # topology-blind round-robin on the same cores: connection i runs on thread i % T
            # and goes to replica (i // T) % n, so every thread deals its connections over all
            # replicas wherever they run, as a LoadBalancer Service deals them (pom.xml:77-80)
            nthreads = len(p["loadgen"])
            res = _measure(rs.targets, conns, p["loadgen"], args, verify=True,
                           conn_targets=[(i // nthreads) % n for i in range(conns)])
        else:
            # client-side round-robin: one target per replica, so each target's body is fixed
            res = _measure(rs.targets, conns, p["loadgen"], args, verify=args.lb == "client")
        m1 = [metrics_counters(0, probe=pr) for pr in probes]
        cpu1 = [proc_cpu_s(pr.proc.pid) for pr in rs.procs]
        t1 = cpu_times()
        for pr in probes:
            pr.close()
    # Per replica, over warm-up and timed run: requests, where its clients ran, its process's CPU
    # time, its busy-poll spins / back-offs, and how busy its server CPUs and the CPUs of the
    # client threads that drive it (slot plans: thread t drives replica t % n) were (/proc/stat: every task and interrupt on them). A replica
    # whose CPUs read busier than its own CPU time shares them with something else.
    drivers = [[c for t, c in enumerate(p["loadgen"]) if t % n == r] for r in range(n)]
    per_replica = [{"requests": int(b.get("requests", 0) - a.get("requests", 0)),
                    "locality": locality_fraction(counter_delta(a, b, "locality.")),
                    "cpu_s": round(c1 - c0, 3), "spins": counter_delta(a, b, "spins."),
                    "server_cpus_busy": busy_fraction(t0, t1, set(p["replicas"][r])),
                    "client_cpus_busy": (busy_fraction(t0, t1, set(drivers[r]))
                                         if args.lb == "client" and args.slot_cores else None)}
                   for r, (a, b, c0, c1) in enumerate(zip(m0, m1, cpu0, cpu1))]
    lat = res["latency"]
    return {
        "replicas": n, "connections": conns, "lb": args.lb, "rps": res["rps"],
        "p50_ms": lat["p50_ns"] / 1e6, "p99_ms": lat["p99_ns"] / 1e6, "p999_ms": lat["p999_ns"] / 1e6,
        "errors": lat["errors"], "non2xx": lat["non2xx"], "body_mismatch": lat.get("body_mismatch", 0),
        "cpu_map": {"replicas": [format_cpu_list(c) for c in p["replicas"]], "proxy": format_cpu_list(p["proxy"]),
                    "loadgen": format_cpu_list(p["loadgen"])},
        "budget": budget, "quota": cgroup_cpu_quota(), "duration_s": args.duration, "per_replica": per_replica,
        "lb_detail": ({"reuseport_cpu": reuseport_cpu} if args.lb == "reuseport" else
                      {"topology_hints": hints} if args.lb == "proxy" else
                      {"dealing": "thread t -> every replica, blind to topology"} if args.lb == "plain" else
                      {"dealing": "thread t -> replica t"}),
        **({"slot_cores": args.slot_cores, "node_slots": p["slots"], "layout": f"miniature node plan ({p['smt']})"}
           if args.slot_cores else {}),
    }


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--replicas", default="1,2,4,8")
    ap.add_argument("--duration", type=float, default=10.0)
    ap.add_argument("--warmup", type=float, default=2.0)
    ap.add_argument("--mode", choices=["weak", "strong"], default="weak")
    ap.add_argument("--connections-per-replica", type=int, default=64)
    ap.add_argument("--connections", type=int, default=512)
    ap.add_argument("--lb", choices=["client", "plain", "proxy", "reuseport"], default="client",
                    help="client: load generator round-robins over replica ports, each thread next to the "
                         "replica it drives; plain: the same dealing blind to topology (every thread over "
                         "every replica); proxy: hola_rrproxy; reuseport: one shared port, the kernel spreads "
                         "connections")
    ap.add_argument("--proxy-threads", type=int, default=0,
                    help="0 = half the CPU budget, mirrored with the servers and the load generator "
                         "in every L3 domain")
    ap.add_argument("--proxy-exe", default="", help="alternative hola_rrproxy binary (A/B runs)")
    ap.add_argument("--busy-poll-us", type=int, default=0,
                    help="busy-poll window of the replicas, the load generator and the proxy")
    ap.add_argument("--server-busy-poll", default="",
                    help="the replicas' own --busy-poll-us (N, auto, auto:N); default --busy-poll-us")
    ap.add_argument("--busy-poll-pause", type=int, default=0,
                    help="PAUSE instructions between empty polls (replicas and load generator)")
    ap.add_argument("--reuseport-cpu", choices=("auto", "none", "self", "sibling"), default="auto",
                    help="--lb reuseport: the replicas' --reuseport-cpu (auto = sibling on the miniature "
                         "pair plan, where each client thread runs on its worker's SMT sibling; else none)")
    ap.add_argument("--proxy-hints", choices=("auto", "on", "off"), default="auto",
                    help="--lb proxy: give hola_rrproxy each replica's CPUs (topology hints; auto = on "
                         "with --slot-cores)")
    ap.add_argument("--slot-cores", type=int, default=0,
                    help="miniature node plan: K physical cores per replica at the node slots' places")
    ap.add_argument("--slots", type=int, default=8, help="node slots of the miniature plan (GPUs on the node)")
    ap.add_argument("--proxy-busy-poll-us", type=int, default=-1, help="-1 = --busy-poll-us")
    ap.add_argument("--budget", type=int, default=0, help="CPUs to use (default: cgroup quota / affinity)")
    ap.add_argument("--server-share", type=float, default=0.5)
    ap.add_argument("--no-tracing", action="store_true")
    ap.add_argument("--out", default="")
    args = ap.parse_args(argv)
    rows = []
    for n in [int(x) for x in args.replicas.split(",")]:
        row = run_point(n, args)
        rows.append(row)
        if args.slot_cores and rows[0]["rps"]:  # weak scaling: N times the N = 1 resources
            row["efficiency"] = round(row["rps"] / (rows[0]["rps"] * n / rows[0]["replicas"]), 4)
        print(json.dumps(row), flush=True)
        time.sleep(0.5)
    base = rows[0]["rps"] if rows else 0
    weak = bool(args.slot_cores)
    table = ["| replicas | connections | LB | req/s | p50 ms | p99 ms | " +
             ("efficiency = total / (N x N=1) |" if weak else "total vs N=1 (same CPU budget) |"),
             "|---|---|---|---|---|---|---|"]
    for r in rows:
        eff = r["rps"] / (base * (r["replicas"] / rows[0]["replicas"] if weak else 1)) if base else 0
        if not weak:
            r["vs_first"] = round(eff, 4)
        table.append(f"| {r['replicas']} | {r['connections']} | {r['lb']} | {r['rps']:.0f} | {r['p50_ms']:.3f} | "
                     f"{r['p99_ms']:.3f} | {eff:.3f} |")
    print("\n".join(table))
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"rows": rows, "table": table}, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
