#!/usr/bin/env python3
"""Headline benchmark: HTTP req/s + p50/p99 latency of GET /api/hola (BASELINE.json).

One rank per "GPU slot" of the node = one hola replica. Every rank:
  * starts a `hola` replica pinned to its own share of the host cores (the GPUs stay idle:
    the reference has no tensor work — SURVEY.md §0),
  * drives it with the native closed-loop load generator on disjoint cores; the generator's
    64 keep-alive connections per replica are dealt round-robin over the replicas of the
    node (client-side round-robin, BASELINE.json config 4: "512 connections against 8
    replicas behind round-robin"; N=1 is config 3: 64 connections, 1 replica), each
    load-generator thread on the L3 (or SMT sibling core) of the replicas it drives.
A step = connections x `--reqs-per-conn` requests per replica, drawn by the connections from
a shared budget (weak scaling: the work per replica is fixed). W warmup steps, then exactly
K timed steps between barriers; the elapsed time is the MAX over ranks, `value` is the
node-wide total req/s, and p50/p99 come from the merged latency histograms of all ranks.
Every response body in the timed region is compared with the greeting of the replica behind
its connection (a mismatch is an error). After the timed region rank 0 runs BASELINE config
2 (one connection, 30 s) and reports it as c1_* keys with the host load of that run, then the
as-deployed replica (the image's exact ENTRYPOINT + the manifests' args and env:
`--shutdown-delay-ms 5000 --busy-poll-us auto`; deployed_* keys), then the chaining endpoint
(load generator -> hola A -> hola B as aloha; chain_* keys); the JSON also carries span
accounting
(`tracing`, with a native collector under --zipkin-sink), connection placement (`locality`)
and how busy the replicas' cores and their idle SMT siblings were (`host_load`: other
tenants on the siblings are what moves the number between runs on a shared host).

  python bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))

from hola_amd.native import ensure_built  # noqa: E402
from hola_amd.parallel.hostmetrics import (  # noqa: E402
    MetricsProbe, accept_locality, busy_fraction, cgroup_cpu_stat, cpu_times, proc_cpu_s, sink_stats, span_counters,
    start_zipkin_sink, tcp_counters, thread_cpu_s)
from hola_amd.parallel.loadgen import ControlledLoadgen, decode_hist, merge_hists, percentile  # noqa: E402
from hola_amd.server import HolaProcess  # noqa: E402
from hola_amd.utils.cpu import (  # noqa: E402
    cgroup_cpu_quota, connection_targets, cpu_budget, format_cpu_list, plan_replicas_with_loadgen, siblings,
    slot_cores, smt_fits)

METRIC = "HTTP req/sec + p50/p99 latency, GET /api/hola at 1/2/4/8 replicas"
BASELINE_VALUE = None  # the reference publishes no numbers


def parse_args():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1, help="replicas on this node (one per rank)")
    # A step is sized so that the driver's `--steps 20` times ~30 s at ~4.1 M req/s, the length
    # of BASELINE configs 3/4 (30 s wrk runs): 20 x 64 x 96,000 requests.
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--connections", type=int, default=64, help="keep-alive connections per replica")
    ap.add_argument("--reqs-per-conn", type=int, default=96000, help="requests per connection per step")
    ap.add_argument("--cores", type=int, default=0,
                    help="physical host cores per replica (server + load generator); 0 = one GPU "
                         "slot's share of the node: min(CPU budget, physical cores) / GPUs on the node "
                         "(16 on the 16-CPU box and on a 2x64-core 8-GPU node), decided per node, so "
                         "every N runs each replica on the same resources (weak scaling)")
    ap.add_argument("--server-threads", type=int, default=0, help="0 = half of the rank's cores")
    ap.add_argument("--base-port", type=int, default=int(os.environ.get("HOLA_BENCH_PORT", "18400")))
    ap.add_argument("--path", default="/api/hola")
    ap.add_argument("--host", default="auto",
                    help="loopback address of the replicas; auto = ::1 when IPv6 loopback works (2.6%% "
                         "more req/s than 127.0.0.1 on the box, profiles/round1/r20_v6), else 127.0.0.1")
    ap.add_argument("--no-tracing", action="store_true", help="run replicas with tracing off")
    ap.add_argument("--zipkin-sink", action="store_true",
                    help="the deployed tracing configuration (ZIPKIN_SERVER_URL is set in the image, "
                         "Dockerfile:6): start a native discard Zipkin collector (hola_zipkin_sink) and "
                         "point every replica at it; the JSON gains a `tracing` block with spans "
                         "recorded/reported/dropped per second and the reporter thread's CPU")
    ap.add_argument("--zipkin-url", default="",
                    help="the replicas' collector URL as given (e.g. the image's http://zipkin-query:9411, "
                         "which does not resolve on a bare host); --zipkin-sink starts a real one instead")
    ap.add_argument("--trace-queue", type=int, default=-1,
                    help="replicas' --trace-queue (spans exported per flush interval; -1 = server "
                         "default 1000, Brave 3's collector queue; 0 = bounded only by the rings)")
    ap.add_argument("--profile-dir", default="",
                    help="run replicas with --profile and write their stage histograms here")
    ap.add_argument("--cpu-profile-dir", default="",
                    help="run replicas and load generators with --cpu-profile (sampled call stacks of "
                         "their threads; bench/cpuprof_report.py symbolises them) and write them here")
    ap.add_argument("--plain-dealing", action="store_true",
                    help="deal every rank's connections (i + rank) %% N over all replicas from its own "
                         "cores, instead of giving each load-generator thread the replicas of its L3 "
                         "(A/B of the planner's locality)")
    ap.add_argument("--no-avoid-busy", action="store_true",
                    help="take cores in id order instead of the quietest L3 domains first")
    ap.add_argument("--per-conn-quota", action="store_true",
                    help="every connection does exactly --reqs-per-conn per step (default: the step's "
                         "connections x reqs-per-conn requests are shared, so no connection idles at the end)")
    ap.add_argument("--smt", choices=("auto", "off", "split", "pair"), default="auto",
                    help="use the SMT sibling of each planned physical core: off = idle, split = "
                         "same side, pair = server worker + its load-generator thread on one core "
                         "(1.55x req/s per physical core, profiles/round1/r16_smt); auto = pair when one GPU "
                         "slot's CPU share (budget / GPUs on the node) holds both threads of --cores "
                         "cores, else off. Decided per node, so every N runs replicas alike")
    ap.add_argument("--epoll-lt", action="store_true",
                    help="level-triggered epoll for connection sockets on both sides (default: edge)")
    ap.add_argument("--busy-poll-pause", type=int, default=-1,
                    help="PAUSE instructions between empty polls while busy-polling (both sides); "
                         "-1 = 16 with --smt pair (+6%% req/s: the spinning sibling leaves issue slots "
                         "to the working one, profiles/round1/r19_pause), else 0")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="requests per connection sent back to back before waiting for their "
                         "responses (wrk's pipeline.lua, as in the TechEmpower plaintext test); "
                         "1 = wrk's default and the headline (BASELINE configs 2-4)")
    ap.add_argument("--c1-seconds", type=float, default=30.0,
                    help="after the timed region, rank 0 drives its own replica over ONE connection for "
                         "about this long (BASELINE config 2: 30 s) and reports c1_rps/c1_p50_ms/c1_p99_ms "
                         "with the host load of that run; 0 = skip. Outside the timed region: `value` is "
                         "untouched")
    ap.add_argument("--c1-reqs", type=int, default=0,
                    help="config-2 request count instead of --c1-seconds (0 = sized from a warm-up "
                         "run to last --c1-seconds)")
    ap.add_argument("--deployed-seconds", type=float, default=3.0,
                    help="after the timed region, rank 0 also drives a replica started exactly as the image "
                         "and manifests start it (deploy/Dockerfile ENTRYPOINT + deploy/openshift args and "
                         "env) on its server CPUs, with the same load generator, for about "
                         "this long; reported as deployed_*. 0 = skip. `value` is untouched")
    ap.add_argument("--chain-seconds", type=float, default=5.0,
                    help="after the timed region, rank 0 also measures GET /api/hola-chaining: load generator "
                         "-> hola A -> hola B (B answering as aloha), 64 connections, about this long, on "
                         "the rank's CPUs; reported as chain_* (rps, latency, A's CPU per request, Hystrix "
                         "events: fallbacks must be 0). 0 = skip. `value` is untouched")
    ap.add_argument("--chain-pool", type=int, default=128,
                    help="hola A's Hystrix thread-pool (bulkhead) size in the chain sub-run: the reference's "
                         "10 would turn most of 64 concurrent calls into fallbacks (SURVEY.md D2)")
    ap.add_argument("--server-busy-poll", default="",
                    help="the replica's own --busy-poll-us (N, auto or auto:N); default: adaptive with the "
                         "load generator's N (`auto`, as the manifests start the replica), 0 when that is 0")
    ap.add_argument("--gpu-slots", type=int, default=0,
                    help="rehearsal only: plan as if the node had this many GPUs (replica slots) instead "
                         "of the ones it has (0 = detect)")
    ap.add_argument("--ignore-quota", action="store_true",
                    help="rehearsal only: plan on the whole affinity mask, ignoring the cgroup CPU quota "
                         "(the 1-GPU box is a 16-CPU quota over a 256-CPU host: with --gpu-slots 8 this "
                         "plans the unconstrained 8-GPU node's layout on its real topology)")
    ap.add_argument("--plan-only", action="store_true",
                    help="print the core plan of every slot of the node (one JSON line) and exit")
    ap.add_argument("--busy-poll-us", type=int, default=20,
                    help="spin this long in epoll before sleeping (the load generator; the replica spins "
                         "adaptively up to this long); 20 us measured best on the box "
                         "(profiles/round1/r11_box_session), 0 = off")
    a = ap.parse_args()
    if not a.server_busy_poll:
        # the manifests' setting: at saturation equal to a fixed spin (profiles/round3/10_auto)
        a.server_busy_poll = ("auto" if a.busy_poll_us == 20 else f"auto:{a.busy_poll_us}") if a.busy_poll_us else "0"
    return a


def main() -> int:
    a = parse_args()
    if a.ignore_quota:
        os.environ["HOLA_IGNORE_QUOTA"] = "1"  # read by cpu_budget(); inherited by every rank
    if a.plan_only:
        return _plan_only(a)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world != a.gpus:
        print(f"bench: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)

    dist = None
    if world > 1:
        import torch.distributed as dist  # gloo: replicas exchange only a few numbers (no device data)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        with _stdout_to_stderr():  # gloo prints "[Gloo] Rank N is connected..." on fd 1
            dist.init_process_group("gloo", rank=rank, world_size=world)

    ensure_built("release")  # file-locked: concurrent ranks build once

    # ---- core plan: disjoint physical cores per rank, quietest L3 domains first (computed
    # once on rank 0 and broadcast, since load measurements differ between processes);
    # within a rank, server worker t and loadgen thread t share an L3 domain. ----
    plan = [None]
    sink = None
    if rank == 0 and a.zipkin_sink and not a.no_tracing:
        sink = start_zipkin_sink()
    if rank == 0:
        slots = max(local_world, a.gpu_slots or _gpu_slots())
        cores = a.cores or slot_cores(slots)
        per_rank = min(cores, max(1, cpu_budget() // local_world))
        host = a.host if a.host != "auto" else ("::1" if _can_bind("::1") else "127.0.0.1")
        smt = a.smt
        if smt == "auto":
            smt = "pair" if smt_fits(slots, per_rank) else "off"
        plan = [{"cores": plan_replicas_with_loadgen(local_world, per_rank, a.server_threads,
                                                     avoid_busy=not a.no_avoid_busy, smt=smt),
                 "smt": smt, "gpu_slots": slots,
                 "host": host,
                 "base_port": _free_port_block(a.base_port, local_world, host),
                 "sink_port": sink[1] if sink else 0}]
        # the rank's own load-generator cores, for --plain-dealing (the r42 layout)
        plan[0]["own_loadgen"] = _own_loadgen(plan[0]["cores"])
    if dist:
        dist.broadcast_object_list(plan, src=0)
    server_cpus, load_cpus = plan[0]["cores"][local_rank]["server"], plan[0]["cores"][local_rank]["loadgen"]
    thread_targets = plan[0]["cores"][local_rank].get("thread_targets")
    # Each load-generator thread drives only replicas in its own L3 (see
    # plan_replicas_with_loadgen); None = plain (i + rank) % N dealing.
    conn_targets = connection_targets(thread_targets, a.connections) if thread_targets else None
    if a.plain_dealing:
        conn_targets = None
        load_cpus = plan[0]["own_loadgen"][local_rank]
    s_threads = len(server_cpus)
    smt = plan[0]["smt"]
    if a.busy_poll_pause < 0:
        a.busy_poll_pause = 16 if smt == "pair" else 0
    base_port = plan[0]["base_port"]
    port = base_port + local_rank
    host = plan[0]["host"]
    targets = [(host, base_port + i) for i in range(local_world)]

    env = {"HOSTNAME": f"replica-{rank}"}
    # Every response body is checked by the load generator (a mismatch is an error): the
    # replica behind target i answers "Hola de replica-<node's first rank + i>".
    first_rank = rank - local_rank
    bodies = _expected_bodies(a.path, [first_rank + i for i in range(local_world)])
    args = ["--no-tracing"] if a.no_tracing else []
    if plan[0]["sink_port"]:
        args += ["--zipkin-url", f"http://127.0.0.1:{plan[0]['sink_port']}/"]
    elif a.zipkin_url and not a.no_tracing:
        args += ["--zipkin-url", a.zipkin_url]
    if a.trace_queue >= 0:
        args += ["--trace-queue", str(a.trace_queue)]
    if host != "127.0.0.1":
        args += ["--host", host]
    if a.epoll_lt:
        args += ["--epoll-lt"]
    server_bp = a.server_busy_poll
    if server_bp != "0":
        args += ["--busy-poll-us", server_bp]
        if a.busy_poll_pause:
            args += ["--busy-poll-pause", str(a.busy_poll_pause)]
    if a.profile_dir:
        os.makedirs(a.profile_dir, exist_ok=True)
        args += ["--profile", "--profile-out", os.path.join(os.path.abspath(a.profile_dir),
                                                            f"server_profile_rank{rank}.json")]
    if a.cpu_profile_dir:
        os.makedirs(a.cpu_profile_dir, exist_ok=True)
        args += ["--cpu-profile", os.path.join(os.path.abspath(a.cpu_profile_dir), f"server_cpu_rank{rank}.prof")]
    server = HolaProcess(args=args, env=env, port=port, threads=s_threads, cpu_list=format_cpu_list(server_cpus),
                         log_level="warn")
    server.start()
    loadgen = None
    # /metrics over one kept-alive connection: the placement counters before the load
    # generator connects and after the timed region then differ by exactly its connections
    probe = MetricsProbe(host, port)
    locality0 = accept_locality(host, port, probe)
    try:
        if dist:
            dist.barrier()  # every replica is listening before any connection is made
        loadgen = ControlledLoadgen(targets, a.connections, len(load_cpus), cpu_list=",".join(map(str, load_cpus)),
                                    path=a.path, target_offset=local_rank, busy_poll_us=a.busy_poll_us,
                                    busy_poll_pause=a.busy_poll_pause, epoll_lt=a.epoll_lt,
                                    per_conn_quota=a.per_conn_quota, pipeline=a.pipeline,
                                    expect_bodies=bodies, verify_body=bodies is None, conn_targets=conn_targets,
                                    cpu_profile=os.path.join(os.path.abspath(a.cpu_profile_dir),
                                                             f"loadgen_cpu_rank{rank}.prof") if a.cpu_profile_dir else None)
        for _ in range(a.warmup):
            loadgen.run(a.reqs_per_conn)
        loadgen.reset()

        cuda = _cuda_sync_fn(local_rank)
        if dist:
            dist.barrier()
        cuda()
        span0 = span_counters(host, port, probe)
        sink0 = sink_stats(plan[0]["sink_port"]) if local_rank == 0 else {}
        tracer0 = thread_cpu_s(server.proc.pid, "hola-tracer")
        cpu0 = (proc_cpu_s(server.proc.pid), proc_cpu_s(loadgen.proc.pid))
        tcp0 = tcp_counters()
        thr0 = cgroup_cpu_stat()
        times0 = cpu_times()
        t0 = time.perf_counter()
        reqs = errs = 0
        for _ in range(a.steps):
            r = loadgen.run(a.reqs_per_conn)
            reqs += r["requests"]
            errs += r["errors"]
        if dist:
            dist.barrier()
        cuda()
        elapsed = time.perf_counter() - t0
        cpu1 = (proc_cpu_s(server.proc.pid), proc_cpu_s(loadgen.proc.pid))
        tracer1 = thread_cpu_s(server.proc.pid, "hola-tracer")
        span1 = span_counters(host, port, probe)
        locality1 = accept_locality(host, port, probe)
        locality = {k: v - locality0.get(k, 0) for k, v in locality1.items()}
        sink1 = sink_stats(plan[0]["sink_port"]) if local_rank == 0 else {}
        tcp1 = tcp_counters()
        thr1 = cgroup_cpu_stat()
        times1 = cpu_times()
        own = set(server_cpus) | set(load_cpus)
        sibs = {x for c in own for x in siblings(c)} - own
        st = loadgen.stats()
        mem = server.memory_kb()
        c1 = _config2_subrun(a, host, port, server_cpus, load_cpus, bodies and [bodies[local_rank]]) if local_rank == 0 else None

        local = {"elapsed": elapsed, "requests": reqs, "errors": errs, "hist": st.get("hist", ""),
                 "non2xx": st.get("non2xx", 0), "body_checked": st.get("body_checked", 0),
                 "body_mismatch": st.get("body_mismatch", 0), "c1": c1,
                 "spans": {k: span1[k] - span0.get(k, 0) for k in span1},
                 "sink": {k: sink1[k] - sink0.get(k, 0) for k in sink1},
                 "tracer_cpu_s": tracer1 - tracer0,
                 "locality": locality,
                 "server_cpus": format_cpu_list(server_cpus),
                 "load_cpus": format_cpu_list(load_cpus),
                 "server_cpu_s": cpu1[0] - cpu0[0], "loadgen_cpu_s": cpu1[1] - cpu0[1],
                 "startup_ms": server.startup_ms, "rss_peak_kb": mem.get("VmHWM", 0),
                 "tcp": {k: tcp1[k] - tcp0[k] for k in tcp1 if k in tcp0},
                 "cgroup": {k: thr1[k] - thr0[k] for k in thr1 if k in thr0},
                 # host-wide busy share over the timed region of this rank's CPUs and of their
                 # SMT siblings that it leaves idle (busy there = another tenant sharing our cores)
                 "host_load": {"own": busy_fraction(times0, times1, own),
                               "siblings": busy_fraction(times0, times1, sibs)}}
        if dist:
            gathered = [None] * world
            dist.all_gather_object(gathered, local)
        else:
            gathered = [local]
    finally:
        probe.close()
        if loadgen:
            loadgen.close()
        server.stop()
    # The as-deployed replica, then the chaining path, on the same CPUs once the headline
    # replica is gone (rank 0).
    deployed = chain = None
    if local_rank == 0 and a.deployed_seconds > 0:
        try:
            deployed = _deployed_subrun(a, server_cpus, load_cpus)
        except Exception as e:  # noqa: BLE001 - reported in the JSON; the other ranks must not hang
            deployed = {"error": f"{type(e).__name__}: {e}"}
    if local_rank == 0 and a.chain_seconds > 0:
        try:
            chain = _chain_subrun(a, list(server_cpus) + list(load_cpus))
        except Exception as e:  # noqa: BLE001 - as above
            chain = {"error": f"{type(e).__name__}: {e}"}
    if dist:
        both = [None] * world
        dist.all_gather_object(both, (deployed, chain))
        deployed, chain = both[0]
        if sink:
            sink[0].terminate()
            sink[0].wait(timeout=10)

    if rank == 0:
        t = max(g["elapsed"] for g in gathered)
        total = sum(g["requests"] for g in gathered)
        hist = merge_hists([decode_hist(g["hist"]) for g in gathered])
        value = total / t if t > 0 else 0.0
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "req/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(t * 1000.0 / a.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None if BASELINE_VALUE is None else round(value / BASELINE_VALUE, 4),
            "dtype": "n/a (host-CPU HTTP service; no tensor compute)",
            "data": "synthetic closed-loop HTTP load (native loadgen, keep-alive, "
                    + ("1 request in flight per connection" if a.pipeline == 1 else
                       f"{a.pipeline} pipelined requests in flight per connection")
                    + ", every response body verified)",
            "p50_ms": round(percentile(hist, 50) / 1e6, 4),
            "p99_ms": round(percentile(hist, 99) / 1e6, 4),
            "p999_ms": round(percentile(hist, 99.9) / 1e6, 4),
            "requests": total,
            # host CPU time per request (user+sys, all threads) over the timed region
            "server_cpu_us_per_req": round(1e6 * sum(g["server_cpu_s"] for g in gathered) / max(1, total), 3),
            "loadgen_cpu_us_per_req": round(1e6 * sum(g["loadgen_cpu_s"] for g in gathered) / max(1, total), 3),
            # replica footprint: exec -> listening, and peak resident memory (max over ranks)
            "server_startup_ms": round(max(g["startup_ms"] or 0 for g in gathered), 1),
            "server_rss_peak_mb": round(max(g["rss_peak_kb"] for g in gathered) / 1024.0, 1),
            # loopback TCP segments per request over the timed region (the network namespace
            # is shared by all ranks, so rank 0's delta covers the node): ~2 = one request and
            # one response segment with the ACKs piggybacked
            "tcp_per_req": {k: round(v / max(1, total), 3) for k, v in gathered[0]["tcp"].items()},
            # CFS bandwidth throttling of this cgroup over the timed region (cgroup v2
            # cpu.stat; shared by all ranks of one container): with a CPU quota, threads that
            # exceed it in a 100 ms period all stop until the next one
            "cgroup_throttle": {"periods": gathered[0]["cgroup"].get("nr_periods", 0),
                                "throttled_periods": gathered[0]["cgroup"].get("nr_throttled", 0),
                                "throttled_ms": round(gathered[0]["cgroup"].get("throttled_usec", 0) / 1000.0, 1)},
            "errors": sum(g["errors"] for g in gathered),
            "non2xx": sum(g["non2xx"] for g in gathered),
            # every 2xx body of the timed region compared byte for byte with the expected one
            "body_checked": sum(g["body_checked"] for g in gathered),
            "body_mismatch": sum(g["body_mismatch"] for g in gathered),
            # BASELINE config 2 (1 connection, 1 replica), measured after the timed region
            **_c1_keys(gathered[0]["c1"]),
            # the replica as the image and manifests run it (--shutdown-delay-ms 5000
            # --busy-poll-us auto), same load generator
            **_deployed_keys(deployed),
            # GET /api/hola-chaining through two replicas (the endpoint with real work behind it)
            **_chain_keys(chain),
            # span accounting over the timed region, all replicas (per second)
            "tracing": _tracing_block(a, gathered, t, plan[0]["sink_port"]),
            # client thread vs. serving worker placement of every accepted connection
            "locality": _locality_block(gathered),
            # busy share of the replicas' CPUs and of the SMT siblings they leave idle, per rank,
            # over the timed region: siblings kept busy by other tenants slow our threads
            "host_load": [g["host_load"] for g in gathered],
            "config": {
                "model": "hola GET /api/hola (native C++ replica, default greeting, "
                         + ("tracing off" if a.no_tracing else
                            "B3 tracing on, spans posted to a native discard Zipkin collector "
                            "(hola_zipkin_sink) as the deployed ZIPKIN_SERVER_URL does" if plan[0]["sink_port"] else
                            f"B3 tracing on, collector URL {a.zipkin_url}" if a.zipkin_url else
                            "B3 tracing on without a collector: spans counted and dropped, as Brave "
                            "does with ZIPKIN_SERVER_URL unset")
                         + (f", --busy-poll-us {a.server_busy_poll}" if a.server_busy_poll != "0" else "") + ")",
                "global_batch": a.connections * world,
                "seq_len": 1,
                "parallelism": f"replicas{world}",
                "connections_per_replica": a.connections,
                "reqs_per_conn_per_step": a.reqs_per_conn,
                "pipeline": a.pipeline,
                "lb": "client-side " + ("round-robin over all replicas from the rank's own cores" if a.plain_dealing
                                        else plan[0]["cores"][local_rank].get("dealing", "round-robin")),
                "loopback": host,
                "cores_per_replica": len({min(siblings(c)) for c in list(server_cpus) + list(load_cpus)}),
                "server_threads_per_replica": s_threads,
                "loadgen_threads_per_replica": len(load_cpus),
                "busy_poll_us": a.busy_poll_us,
                "server_busy_poll": a.server_busy_poll,
                "busy_poll_pause": a.busy_poll_pause,
                "epoll": "level" if a.epoll_lt else "edge",
                "smt": smt,
                "layout_note": _layout_note(plan[0]["gpu_slots"], smt, server_cpus, load_cpus),
                "gpu_slots_on_node": plan[0]["gpu_slots"],
                "cpus_per_replica": len(set(server_cpus) | set(load_cpus)),
                "step_budget": "per-connection" if a.per_conn_quota else "shared",
                "cpu_map": {f"rank{i}": {"server": g["server_cpus"], "loadgen": g["load_cpus"]}
                            for i, g in enumerate(gathered)},
                "cpu_budget": cpu_budget(),
                "cgroup_quota": cgroup_cpu_quota(),
            },
        }
        print(json.dumps(out), flush=True)
    if dist:
        with _stdout_to_stderr():
            dist.barrier()
            dist.destroy_process_group()
    return 0


def _plan_only(a) -> int:
    """The core plan of a whole node (one replica per GPU slot), as rank 0 computes it, without
    starting anything: the cpu map an N = slots run would use."""
    from hola_amd.utils.cpu import l3_domain, package_of, physical_cores

    slots = a.gpu_slots or max(1, _gpu_slots())
    cores = a.cores or slot_cores(slots)
    per_rank = min(cores, max(1, cpu_budget() // slots))
    smt = a.smt
    if smt == "auto":
        smt = "pair" if smt_fits(slots, per_rank) else "off"
    plan = plan_replicas_with_loadgen(slots, per_rank, a.server_threads, avoid_busy=False, smt=smt)
    print(json.dumps({"gpu_slots": slots, "cores_per_slot": per_rank, "smt": smt, "cpu_budget": cpu_budget(),
                      "cgroup_quota": cgroup_cpu_quota(), "physical_cores": len(physical_cores()),
                      "ranks": [{"server": p["server"], "loadgen": p["loadgen"], "thread_targets": p["thread_targets"],
                                 "dealing": p["dealing"],
                                 "server_sockets": sorted({package_of(c) for c in p["server"]}),
                                 "server_l3": sorted({l3_domain(c) for c in p["server"]}),
                                 "loadgen_sockets": sorted({package_of(c) for c in p["loadgen"]}),
                                 "siblings": {str(c): siblings(c) for c in p["server"] + p["loadgen"]}}
                                for p in plan]}), flush=True)
    return 0


def _own_loadgen(cores: list[dict]) -> list[list[int]]:
    """Load-generator CPUs regrouped so that each rank runs on the CPUs planned next to its
    own replica (no cross-rank swap): rank r takes the CPUs whose L3 is its server's."""
    from hola_amd.utils.cpu import l3_domain
    pool = sorted({c for p in cores for c in p["loadgen"]})
    out = []
    for p in cores:
        doms = {l3_domain(c) for c in p["server"]}
        mine = [c for c in pool if l3_domain(c) in doms][:len(p["loadgen"])]
        for c in mine:
            pool.remove(c)
        out.append(mine if len(mine) == len(p["loadgen"]) else p["loadgen"])
    return out


def _locality_block(gathered: list[dict]) -> dict:
    """Node-wide and per-replica fractions of accepted connections by client/worker
    relation, counted over the load generator's own connections (made before the timed
    region): the placement of every timed request's connection."""
    def frac(d: dict) -> dict:
        n = sum(d.values())
        return {k: round(v / n, 4) for k, v in d.items()} if n else {}
    total: dict[str, int] = {}
    for g in gathered:
        for k, v in g["locality"].items():
            total[k] = total.get(k, 0) + v
    return {"accepted": sum(total.values()), "fraction": frac(total),
            "per_replica": [frac(g["locality"]) for g in gathered]}


def _tracing_block(a, gathered: list[dict], t: float, sink_port: int) -> dict:
    if a.no_tracing:
        return {"mode": "off"}
    spans: dict[str, int] = {}
    for g in gathered:
        for k, v in g["spans"].items():
            spans[k] = spans.get(k, 0) + v
    per_s = {k: round(v / t, 1) for k, v in sorted(spans.items())} if t > 0 else {}
    out = {"mode": "collector: native discard sink (hola_zipkin_sink)" if sink_port else
           f"collector URL {a.zipkin_url} (as given)" if a.zipkin_url else
           "no collector (ZIPKIN_SERVER_URL unset): spans counted and dropped at the source",
           "trace_queue_per_flush": a.trace_queue if a.trace_queue >= 0 else 1000,
           "spans_per_s": per_s,
           # reporter thread CPU (drain rings, encode Zipkin JSON, POST), % of one core, summed
           "reporter_cpu_pct": round(100.0 * sum(g["tracer_cpu_s"] for g in gathered) / t, 2) if t > 0 else 0.0}
    if sink_port and gathered[0]["sink"]:
        s = gathered[0]["sink"]
        out["sink_received_spans_per_s"] = round(s.get("spans", 0) / t, 1) if t > 0 else 0.0
        out["sink_posts"] = s.get("posts", 0)
        out["sink_bad"] = s.get("bad", 0)
    return out


def _expected_bodies(path: str, ranks: list[int]) -> list[str] | None:
    """Exact body each target must answer, or None to learn it from the first response."""
    if path.split("?")[0] in ("/api/hola", "/api/hola/"):
        return [f"Hola de replica-{r}" for r in ranks]  # default greeting (HolaResource.java:60,65)
    if path.split("?")[0] == "/api/health":
        return ["I'm ok"] * len(ranks)
    return None


def _config2_subrun(a, host: str, port: int, server_cpus, load_cpus, bodies) -> dict | None:
    """BASELINE config 2: one keep-alive connection against this rank's replica, run after
    the timed region (so the headline is unaffected)."""
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
        sibs = {x for c in own for x in siblings(c)} - own
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
            # as for the headline: busy share of the replica's + client's CPUs and of their idle
            # SMT siblings over this run (another tenant on a sibling slows the one connection)
            "host_load": {"own": busy_fraction(t0, t1, own), "siblings": busy_fraction(t0, t1, sibs)}}


def _layout_note(slots: int, smt: str, server_cpus, load_cpus) -> str:
    """One line that tells a SCALE_rNN.json reader why its N=1 point differs from BENCH."""
    phys = len({min(siblings(c)) for c in list(server_cpus) + list(load_cpus)})
    how = ("each physical core runs a server worker on one SMT thread and its load-generator "
           "thread on the other (--smt pair)" if smt == "pair" else
           "server workers and load-generator threads on separate physical cores, SMT siblings idle")
    return (f"{slots} GPU slot(s) on this node: each replica's share is {phys} physical cores "
            f"({len(set(server_cpus) | set(load_cpus))} CPUs); {how}. The 1-GPU box (16-CPU quota) runs "
            f"smt=off and an unconstrained 8-GPU node smt=pair, so BENCH and SCALE's N=1 differ by layout, "
            f"not by code; compare config.smt before reading a difference as a regression.")


def _deployed_subrun(a, server_cpus, load_cpus) -> dict | None:
    """The replica exactly as deployed: deploy/Dockerfile's ENTRYPOINT (its /app paths mapped
    to this tree) + the container args and env of deploy/openshift/hola-dc.yaml, in a cpuset of
    this rank's server CPUs (a Guaranteed pod under the static CPU manager), HOSTNAME = a pod
    name. Only the listen port differs (a free one instead of 8080). Same load generator as the
    headline, about --deployed-seconds long."""
    import socket
    import subprocess

    from hola_amd import native
    from hola_amd.kube import manifests as km
    from hola_amd.kube.image import Image

    img = Image.from_dockerfile()
    dc = next(o for o in km.load_objects([Path(__file__).resolve().parent / "deploy/openshift/hola-dc.yaml"])
              if o["kind"] == "DeploymentConfig")
    cont = dc["spec"]["template"]["spec"]["containers"][0]
    argv = [str(img.files.get(x, x)) for x in img.entrypoint] + [str(x) for x in cont.get("args") or []]
    argv[0] = str(native.binary("hola"))
    port = _free_port_block(18900, 1)
    argv += ["--port", str(port)]
    env = {k: v for k, v in os.environ.items() if k in ("PATH", "LANG", "LD_LIBRARY_PATH")}
    env.update(img.env)
    env.update({e["name"]: str(e["value"]) for e in cont.get("env") or [] if "value" in e})
    env["HOSTNAME"] = "hola-1-deplo"  # fieldRef metadata.name
    cpus = list(server_cpus)
    proc = subprocess.Popen(argv, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                            preexec_fn=lambda: os.sched_setaffinity(0, cpus))
    try:
        deadline = time.monotonic() + 10
        while True:
            try:
                socket.create_connection(("127.0.0.1", port), timeout=1).close()
                break
            except OSError:
                if proc.poll() is not None or time.monotonic() > deadline:
                    return {"error": f"deployed replica did not start (rc {proc.poll()})"}
                time.sleep(0.02)
        body = ["Hola de hola-1-deplo"] if a.path == "/api/hola" else None
        lg = ControlledLoadgen([("127.0.0.1", port)], a.connections, len(load_cpus),
                               cpu_list=",".join(map(str, load_cpus)), path=a.path, busy_poll_us=a.busy_poll_us,
                               busy_poll_pause=a.busy_poll_pause, epoll_lt=a.epoll_lt,
                               expect_bodies=body, verify_body=body is None)
        try:
            warm = lg.run(2000)
            rate = warm["requests"] / max(1e-9, warm["elapsed_ns"] / 1e9)
            per_conn = int(min(200_000, max(2_000, rate * a.deployed_seconds / a.connections)))
            lg.reset()
            c0 = proc_cpu_s(proc.pid)
            r = lg.run(per_conn)
            c1 = proc_cpu_s(proc.pid)
            st = lg.stats()
        finally:
            lg.close()
    finally:
        proc.terminate()
        try:
            proc.wait(timeout=15)
        except subprocess.TimeoutExpired:
            proc.kill()
    el = r["elapsed_ns"] / 1e9
    return {"rps": r["requests"] / el if el > 0 else 0.0, "p50_ns": st["p50_ns"], "p99_ns": st["p99_ns"],
            "requests": r["requests"], "errors": r["errors"], "non2xx": st.get("non2xx", 0),
            "cpu_us_per_req": 1e6 * (c1 - c0) / max(1, r["requests"]),
            "args": " ".join(["hola"] + argv[1:-2]), "cpus": format_cpu_list(cpus),
            "env": " ".join(f"{k}={v}" for k, v in sorted(env.items()) if k in img.env or k == "HOSTNAME")}


def _chain_subrun(a, cpus: list[int]) -> dict:
    """GET /api/hola-chaining end to end (HolaResource.java:69-78,94-113): load generator ->
    hola A -> hola B, where B plays aloha (B's own aloha is unreachable, so B answers its
    fallback list at once: ["Hola de B", "Aloha response (fallback)"], which A decodes as the
    aloha's List<String>). Every request crosses A's pooled keep-alive client, the Hystrix
    command (breaker, bulkhead, 600 ms timer), B3 propagation and the JSON decode. Each body is
    checked; an A-side fallback would differ from the expected body. The CPUs are the rank's
    own, split 2:1:1 (A does two hops' work) with each L3 holding a share of all three."""
    from hola_amd.parallel.loadgen import run_duration
    from hola_amd.utils.cpu import split_mirrored

    plan = split_mirrored(sorted(cpus), {"A": 2, "B": 1, "loadgen": 1})
    with HolaProcess(args=["--aloha-url", "http://127.0.0.1:1/", "--feign-log", "none", "--no-tracing",
                           "--feign-retry", "off", "--log-level", "warn"], env={"HOSTNAME": "B"},
                     threads=len(plan["B"]), cpu_list=format_cpu_list(plan["B"])) as b:
        with HolaProcess(args=["--aloha-url", f"http://127.0.0.1:{b.port}/", "--aloha-path", "api/hola-chaining",
                               "--feign-log", "none", "--hystrix-pool-size", str(a.chain_pool), "--log-level", "warn"],
                         env={"HOSTNAME": "A"}, threads=len(plan["A"]), cpu_list=format_cpu_list(plan["A"])) as s:
            st, _, body = s.get("/api/hola-chaining")
            want = json.dumps(["Hola de A", "Hola de B", "Aloha response (fallback)"], separators=(",", ":"))
            if st != 200 or json.loads(body) != json.loads(want):
                return {"error": f"unexpected first answer {st} {body[:200]!r}"}
            ev0 = _hystrix_events(s)
            c0 = proc_cpu_s(s.proc.pid), proc_cpu_s(b.proc.pid)
            w0 = time.perf_counter()
            res = run_duration([("127.0.0.1", s.port)], a.connections, len(plan["loadgen"]), a.chain_seconds, 1.0,
                               cpu_list=format_cpu_list(plan["loadgen"]), path="/api/hola-chaining",
                               expect_bodies=[body.decode()])
            wall = time.perf_counter() - w0
            c1 = proc_cpu_s(s.proc.pid), proc_cpu_s(b.proc.pid)
            ev1 = _hystrix_events(s)
    lat = res["latency"]
    rps = res["rps"]
    # CPU over the whole run (its 1 s warm-up included) per request at the measured rate
    busy = ((c1[0] - c0[0]) / wall, (c1[1] - c0[1]) / wall)
    return {"rps": rps, "p50_ns": lat["p50_ns"], "p99_ns": lat["p99_ns"], "requests": lat.get("count", 0),
            "errors": lat["errors"], "non2xx": lat.get("non2xx", 0), "body_checked": lat.get("body_checked", 0),
            "body_mismatch": lat.get("body_mismatch", 0),
            "a_cpu_us_per_req": 1e6 * busy[0] / rps if rps else 0.0,
            "b_cpu_us_per_req": 1e6 * busy[1] / rps if rps else 0.0,
            "hystrix": {k: ev1.get(k, 0) - ev0.get(k, 0) for k in sorted(set(ev0) | set(ev1))},
            "cpus": {k: format_cpu_list(v) for k, v in plan.items()}, "pool": a.chain_pool}


def _hystrix_events(s: HolaProcess) -> dict:
    _, _, metrics = s.get("/metrics")
    return {ln.split('event="')[1].split('"')[0]: int(float(ln.split()[-1])) for ln in metrics.decode().splitlines()
            if ln.startswith("hola_hystrix_events_total")}


def _chain_keys(c: dict | None) -> dict:
    if not c:
        return {}
    if "error" in c:
        return {"chain_error": c["error"]}
    h = c["hystrix"]
    return {"chain_rps": round(c["rps"], 1), "chain_p50_ms": round(c["p50_ns"] / 1e6, 4),
            "chain_p99_ms": round(c["p99_ns"] / 1e6, 4), "chain_requests": c["requests"],
            "chain_errors": c["errors"], "chain_non2xx": c["non2xx"], "chain_body_checked": c["body_checked"],
            "chain_body_mismatch": c["body_mismatch"],
            # hola A's own CPU per chained request (it serves the client and calls B)
            "chain_a_cpu_us_per_req": round(c["a_cpu_us_per_req"], 3),
            "chain_b_cpu_us_per_req": round(c["b_cpu_us_per_req"], 3),
            # A's Hystrix command over the run (1 s warm-up included): all SUCCESS, no FALLBACK / TIMEOUT
            "chain_hystrix_success": h.get("SUCCESS", 0), "chain_hystrix_fallback": h.get("FALLBACK_SUCCESS", 0),
            "chain_hystrix_timeout": h.get("TIMEOUT", 0), "chain_hystrix_events": h,
            "chain_cpus": c["cpus"], "chain_pool": c["pool"]}


def _deployed_keys(d: dict | None) -> dict:
    if not d:
        return {}
    if "error" in d:
        return {"deployed_error": d["error"]}
    return {"deployed_rps": round(d["rps"], 1), "deployed_p50_ms": round(d["p50_ns"] / 1e6, 4),
            "deployed_p99_ms": round(d["p99_ns"] / 1e6, 4), "deployed_requests": d["requests"],
            "deployed_errors": d["errors"], "deployed_non2xx": d["non2xx"],
            "deployed_server_cpu_us_per_req": round(d["cpu_us_per_req"], 3),
            "deployed_args": d["args"], "deployed_cpus": d["cpus"],
            # ZIPKIN_SERVER_URL names the cluster's zipkin-query Service, which does not resolve
            # on a bare host: spans are recorded and dropped, as Brave does without a collector
            "deployed_env": d["env"]}


def _c1_keys(c1: dict | None) -> dict:
    if not c1:
        return {}
    return {"c1_rps": round(c1["rps"], 1), "c1_p50_ms": round(c1["p50_ns"] / 1e6, 4),
            "c1_p99_ms": round(c1["p99_ns"] / 1e6, 4), "c1_requests": c1["requests"],
            "c1_errors": c1["errors"], "c1_body_checked": c1["body_checked"],
            "c1_elapsed_s": round(c1["elapsed_s"], 2), "c1_host_load": c1.get("host_load"),
            # the client's CPU: with --smt pair it is the SMT sibling of a server worker, and the
            # connection is served on that same physical core (r18: slower for one connection)
            "c1_client_cpu": c1["client_cpu"]}


class _stdout_to_stderr:
    """Points file descriptor 1 at stderr for a block, so native libraries that print to
    stdout cannot break the one-JSON-line contract of this script."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def _can_bind(host: str) -> bool:
    import socket

    try:
        with socket.socket(socket.AF_INET6 if ":" in host else socket.AF_INET) as sk:
            sk.bind((host, 0))
        return True
    except OSError:
        return False


def _free_port_block(start: int, n: int, host: str = "127.0.0.1") -> int:
    """First base >= start such that base..base+n-1 can all be bound on `host`."""
    import socket

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


def _gpu_slots() -> int:
    """GPUs on this node (one replica slot each), visible to this process or not: the KFD
    topology lists every GPU agent (gpu_id != 0), whatever HIP_VISIBLE_DEVICES says; falls
    back to torch.cuda.device_count() (which does not initialise HIP)."""
    n = 0
    for gid in Path("/sys/class/kfd/kfd/topology/nodes").glob("*/gpu_id"):
        try:
            n += int(gid.read_text().strip() or "0") != 0
        except (OSError, ValueError):
            pass
    if n:
        return n
    try:
        import torch
        return int(torch.cuda.device_count())
    except Exception:
        return 0


def _cuda_sync_fn(local_rank: int):
    """torch.cuda.synchronize bracket required by the bench contract. The service launches
    no device work, so this is a no-op fence; it only runs when a GPU is present (and after
    every child process has been started)."""
    if os.environ.get("HOLA_BENCH_CUDA_SYNC", "1") != "1":
        return lambda: None
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
            return torch.cuda.synchronize
    except Exception:
        pass
    return lambda: None


if __name__ == "__main__":
    sys.exit(main())
