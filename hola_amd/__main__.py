"""Command line entry point: ``python -m hola_amd <command>``.

  build [--preset P]                         compile the native artefacts in-tree (P: release,
                                             debug, tsan, asan, or a release-* flag variant)
  serve [hola args...]                       run the service (same flags as the binary)
  cluster --replicas N [--port P] [--lb L]   N pinned replicas on P: behind the round-robin
                                             proxy (--lb proxy) or one SO_REUSEPORT group
                                             spread by the kernel (--lb reuseport)
  scaling [...]                              replica scaling curve (hola_amd.parallel.scaling)
  bench [...]                                the headline benchmark (bench.py)
  info                                       host CPU topology / quota / plan for this node
  units --replicas N --out DIR [--lb L]      systemd units: N pinned replicas + proxy on :8080
                                             (or --lb reuseport: replicas share :8080)
  apply -f MANIFEST... [--replicas N]        run deploy/openshift/*.yaml on this node: pods from
                                             the image's ENTRYPOINT, probe-gated Service, ConfigMaps
  oc get|scale|set env|patch|apply|delete|rollout ...   control a running `apply`

The local equivalents of the reference's `mvn wildfly-swarm:run` (Readme.md:13) and
`mvn clean package docker:build fabric8:json fabric8:apply` (Readme.md:24) are
`python -m hola_amd serve` and deploy/Dockerfile + deploy/openshift/*.yaml, which
`python -m hola_amd apply` executes on one node (hola_amd/kube).
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time
from pathlib import Path

from hola_amd import native


_STOP_SIGNALS = (signal.SIGTERM, signal.SIGINT, signal.SIGHUP)


def _serve(argv: list[str]) -> int:
    exe = native.binary("hola")
    # Runs as a child (never exec from a process that might have touched a GPU). Termination
    # signals sent to this wrapper (systemd, a container runtime, Ctrl-C) go to the server, which
    # drains and exits; the wrapper then exits with its status.
    p = subprocess.Popen([str(exe), *argv])
    for s in _STOP_SIGNALS:
        signal.signal(s, lambda sig, _frame: p.send_signal(sig))
    return p.wait()


class _Stop(Exception):
    pass


def _raise_stop(sig, _frame):
    raise _Stop(sig)


def _cluster(argv: list[str]) -> int:
    from hola_amd.parallel.replicas import ReplicaSet, RRProxy
    from hola_amd.utils.cpu import format_cpu_list, plan_node

    ap = argparse.ArgumentParser(prog="python -m hola_amd cluster")
    ap.add_argument("--replicas", type=int, default=2)
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--host", default="127.0.0.1",
                    help="address of the front (the proxy, or the replicas' shared port); pass the "
                         "address clients reach it on to serve beyond this host. Replicas behind the "
                         "proxy always listen on 127.0.0.1")
    ap.add_argument("--cores-per-replica", type=int, default=0)
    ap.add_argument("--proxy-threads", type=int, default=2)
    ap.add_argument("--lb", choices=["proxy", "reuseport"], default="proxy",
                    help="proxy: hola_rrproxy health-checks /api/health and round-robins connections; "
                         "reuseport: replicas share the port and the kernel spreads connections (no hop)")
    ap.add_argument("hola_args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)

    def wait():
        # SIGTERM/SIGHUP/SIGINT unwind the `with` blocks below, which stop the proxy and every
        # replica (each drains); otherwise they would outlive this process.
        try:
            while True:
                time.sleep(1)
        except (KeyboardInterrupt, _Stop):
            for s in _STOP_SIGNALS:  # a second signal must not interrupt the teardown
                signal.signal(s, signal.SIG_IGN)

    for s in _STOP_SIGNALS:
        signal.signal(s, _raise_stop)

    if a.lb == "reuseport":
        plan = plan_node(a.replicas, a.cores_per_replica or None)
        with ReplicaSet(a.replicas, cpu_plan=plan, args=[*a.hola_args, "--host", a.host], supervise=True,
                        shared_port=a.port) as rs:
            print(f"hola cluster: {a.replicas} replicas sharing :{rs.shared_port} (SO_REUSEPORT; Ctrl-C to stop)",
                  flush=True)
            wait()
        return 0
    plan = plan_node(a.replicas + 1, a.cores_per_replica or None)
    with ReplicaSet(a.replicas, cpu_plan=plan[:a.replicas], args=a.hola_args, supervise=True) as rs:
        with RRProxy(rs.targets, port=a.port, threads=a.proxy_threads, host=a.host,
                     cpu_list=format_cpu_list(plan[-1][:a.proxy_threads])) as px:
            print(f"hola cluster: {a.replicas} replicas on ports {rs.ports} behind :{px.port} (Ctrl-C to stop)",
                  flush=True)
            wait()
    return 0


def _info() -> int:
    from hola_amd.utils.cpu import (allowed_cpus, cgroup_cpu_quota, cpu_budget, format_cpu_list, l3_domain, package_of,
                                    physical_cores, plan_node)

    try:
        from hola_amd.native import binary

        r = subprocess.run([str(binary("hola", build_if_missing=False)), "--version"], capture_output=True,
                           text=True, timeout=10)
        print(f"build          : {r.stdout.strip() or r.stderr.strip()}")
    except Exception as e:  # noqa: BLE001 - a report, not a check
        print(f"build          : not built ({e})")
    phys = physical_cores()
    doms: dict[int, list[int]] = {}
    for c in phys:
        doms.setdefault(l3_domain(c), []).append(c)
    print(f"allowed cpus   : {format_cpu_list(allowed_cpus())}")
    print(f"physical cores : {len(phys)} in {len(doms)} L3 domains")
    print(f"cgroup quota   : {cgroup_cpu_quota() or 'unlimited'}  -> budget {cpu_budget()} CPUs")
    # Host load per L3 domain (both SMT threads of its cores, other tenants included): what
    # the bench's planner ranks when it takes the quietest domains first.
    from hola_amd.utils.cpu import cpu_busy, siblings

    busy = cpu_busy(0.5)
    dom_load = {d: sum(busy.get(x, 0.0) for c in cs for x in siblings(c)) for d, cs in doms.items()}
    print("L3 load (CPUs busy, 0.5 s): " + ", ".join(f"{d}:{v:.1f}" for d, v in sorted(dom_load.items())))
    for n in (1, 2, 4, 8):
        print(f"plan x{n}: {[format_cpu_list(p) for p in plan_node(n, avoid_busy=False)]}")
    # What bench.py would decide on this node (one replica per GPU slot, weak scaling).
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))  # bench.py at the repo root
    from bench import _gpu_slots
    from hola_amd.utils.cpu import slot_cores, smt_fits

    slots = max(1, _gpu_slots())
    cores = slot_cores(slots)
    print(f"gpu slots      : {slots} (KFD topology) -> {cores} physical cores per replica")
    print(f"bench --smt auto: {'pair' if smt_fits(slots, cores) else 'off'}")
    # The bench's per-N layout: server and load-generator CPUs, and which replicas each
    # load-generator thread drives (connection dealing), as bench.py would plan them.
    from hola_amd.utils.cpu import plan_replicas_with_loadgen

    budget = cpu_budget()
    for n in (1, 2, 4, 8):
        # bench.py plans N ranks as max(N, GPU slots) slots, so a node with fewer GPUs than
        # ranks (a rehearsal on the 1-GPU box) splits its budget further
        s = max(n, slots)
        per_rank = min(slot_cores(s), max(1, budget // n))
        smt = "pair" if smt_fits(s, per_rank) else "off"
        try:
            plans = plan_replicas_with_loadgen(n, per_rank, avoid_busy=False, smt=smt)
        except (IndexError, ValueError) as e:
            print(f"bench N={n}: no plan ({e})")
            continue
        print(f"bench N={n}: {per_rank} cores/replica, smt {smt}, {plans[0]['dealing']}")
        for r, p in enumerate(plans):
            socks = sorted({package_of(c) for c in p["server"]})
            print(f"  rank{r}: server {format_cpu_list(p['server'])} loadgen {format_cpu_list(p['loadgen'])} "
                  f"threads->replicas {p['thread_targets']} server socket(s) {socks}")
    return 0


def main(argv: list[str] | None = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("-h", "--help"):
        print(__doc__)
        return 0
    cmd, rest = argv[0], argv[1:]
    if cmd == "build":
        ap = argparse.ArgumentParser(prog="python -m hola_amd build")
        ap.add_argument("--preset", default="release", choices=sorted(native.PRESETS))
        a = ap.parse_args(rest)
        d = native.build(a.preset, quiet=False)
        print(f"built {a.preset} -> {d}")
        return 0
    if cmd == "serve":
        return _serve(rest)
    if cmd == "cluster":
        return _cluster(rest)
    if cmd == "scaling":
        from hola_amd.parallel import scaling

        return scaling.main(rest)
    if cmd == "bench":
        root = Path(__file__).resolve().parent.parent
        return subprocess.call([sys.executable, str(root / "bench.py"), *rest])
    if cmd == "info":
        return _info()
    if cmd == "apply":
        from hola_amd.kube.cli import apply_main

        return apply_main(rest)
    if cmd == "oc":
        from hola_amd.kube.cli import oc_main

        return oc_main(rest)
    if cmd == "units":
        from hola_amd.deploy import write_units

        ap = argparse.ArgumentParser(prog="python -m hola_amd units")
        ap.add_argument("--replicas", type=int, default=8)
        ap.add_argument("--out", required=True)
        ap.add_argument("--prefix", default="/opt/hola")
        ap.add_argument("--port", type=int, default=8080)
        ap.add_argument("--cores-per-replica", type=int, default=0)
        ap.add_argument("--lb", choices=["proxy", "reuseport"], default="proxy")
        a = ap.parse_args(rest)
        for p in write_units(a.out, replicas=a.replicas, prefix=a.prefix, public_port=a.port,
                             cores_per_replica=a.cores_per_replica or None, lb=a.lb):
            print(p)
        return 0
    print(f"unknown command {cmd!r}\n{__doc__}", file=sys.stderr)
    return 2


if __name__ == "__main__":
    sys.exit(main())
