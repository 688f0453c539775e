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
A step = connections x R requests per replica, drawn by the connections from a shared budget
(weak scaling: the work per replica is fixed); R is sized from the last warmup step so that the
driver's 20 steps time the 30 s of BASELINE configs 3/4 (or fixed with --reqs-per-conn). W
warmup steps, then exactly K timed steps between barriers; the elapsed time is the MAX over
ranks, `value` is the node-wide total req/s, and p50/p99 come from the merged latency
histograms of all ranks. Every response body in the timed region is compared with the
greeting of the replica behind its connection (a mismatch is an error).

After the timed region rank 0 runs BASELINE config 2 (one connection, 30 s; c1_* keys), and at
N = 1 the per-node sub-runs of hola_amd/parallel/subruns.py: the as-deployed replica (the
image's ENTRYPOINT + the manifests' args and env: `--shutdown-delay-ms 5000 --busy-poll-us
auto`, ZIPKIN_SERVER_URL set; deployed_*), GET /api/hola-chaining
engineered (chain_*) and as shipped (pool of 10, Feign BASIC logging; chain_shipped_*), and
the headline in the other SMT layout (alt_*: BENCH and SCALE's N = 1 each carry the other's
figure). Each sub-run is one continuous run of the load generator with its warm-up inside it
(`runfor`): no idle gaps for pools and breakers to drain in. The JSON also names the server
binary measured (`build`: release, source revision, x86-64 level) and carries span accounting (`tracing`, with a native collector under
--zipkin-sink), connection placement (`locality`) and how busy the replicas' cores and the
SMT siblings outside the job were (`host_load`: other tenants on the siblings are what moves
the number between runs on a shared host).

  python bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))

from hola_amd.native import binary, ensure_built  # noqa: E402
from hola_amd.parallel.hostmetrics import (  # noqa: E402
    MetricsProbe, accept_locality, cgroup_cpu_stat, cpu_times, proc_cpu_s, sink_stats, span_counters,
    start_zipkin_sink, tcp_counters, thread_cpu_s)
from hola_amd.parallel import subruns  # noqa: E402
from hola_amd.parallel.loadgen import ControlledLoadgen, decode_hist, merge_hists, percentile  # noqa: E402
from hola_amd.server import HolaProcess  # noqa: E402
from hola_amd.utils.cpu import (  # noqa: E402
    cgroup_cpu_quota, connection_targets, cpu_budget, format_cpu_list, physical_cores, plan_replicas_with_loadgen,
    plan_slot_subset, sibling_of, siblings, slot_cores, smt_fits)

METRIC = "HTTP req/sec + p50/p99 latency, GET /api/hola at 1/2/4/8 replicas"
BASELINE_VALUE = None  # the reference publishes no numbers


def parse_args():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1, help="replicas on this node (one per rank)")
    # BASELINE configs 3/4 are 30 s wrk runs: the driver's `--steps 20` is sized to time ~30 s.
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--connections", type=int, default=64, help="keep-alive connections per replica")
    ap.add_argument("--reqs-per-conn", type=int, default=0,
                    help="requests per connection per step; 0 = sized from the last warmup step so that a "
                         "step lasts --step-seconds (every rank takes the smallest size any rank computed, "
                         "so each replica does the same work; `requests` stays exact)")
    ap.add_argument("--step-seconds", type=float, default=1.55,
                    help="target length of one timed step with --reqs-per-conn 0: 20 steps time the 30 s of "
                         "BASELINE configs 3/4 (the timed steps run 0-4 %% faster than the last warmup step "
                         "they are sized from: 28.8-30.2 s at 1.5 s on the box)")
    ap.add_argument("--warmup-reqs-per-conn", type=int, default=96000,
                    help="requests per connection of each warmup step with --reqs-per-conn 0")
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
                         "cores, else off. Decided per node, so every N runs replicas alike. A forced pair "
                         "in a budget too small for both threads pairs half the cores")
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
    ap.add_argument("--deployed-seconds", type=float, default=10.0,
                    help="after the timed region, rank 0 also drives a replica started exactly as the image "
                         "and manifests start it (deploy/Dockerfile ENTRYPOINT + deploy/openshift args and "
                         "env) on its server CPUs, with the same load generator, for about "
                         "this long; reported as deployed_* with its own host load. 0 = skip. `value` is "
                         "untouched. N = 1 only (a per-node figure)")
    ap.add_argument("--deployed-zipkin", choices=("deployed", "unset", "sink"), default="deployed",
                    help="the deployed sub-run's ZIPKIN_SERVER_URL: as the manifests set it (the cluster's "
                         "zipkin-query, unresolvable on a bare host), unset, or a native discard collector")
    ap.add_argument("--chain-seconds", type=float, default=10.0,
                    help="after the timed region, rank 0 also measures GET /api/hola-chaining: load generator "
                         "-> hola A -> hola B (B answering as aloha), 64 connections, about this long, on "
                         "the rank's CPUs; reported as chain_* (rps, latency, A's CPU per request, Hystrix "
                         "events: fallbacks must be 0; host load, accept locality of both hops, busy-poll "
                         "counters of both replicas). 0 = skip. `value` is untouched. N = 1 only")
    ap.add_argument("--chain-shipped-seconds", type=float, default=10.0,
                    help="then the same chain with hola A started exactly as the manifests start it (pool of "
                         "10, Feign BASIC logging, ZIPKIN_SERVER_URL set): chain_shipped_* (rps, latency, "
                         "fallback fraction, Hystrix SUCCESS count). 0 = skip. N = 1 only")
    ap.add_argument("--chain-loadgen-busy-poll", type=int, default=0,
                    help="the chain sub-runs' load generator busy-poll window in us (0 = sleep in epoll_wait)")
    ap.add_argument("--alt-seconds", type=float, default=10.0,
                    help="N = 1 only: the headline replica again in the other SMT layout for about this long "
                         "(alt_* keys): pair on a 1-GPU box, off on an 8-GPU node, so BENCH and SCALE's N = 1 "
                         "each carry a figure in the other's layout. 0 = skip")
    ap.add_argument("--v4-seconds", type=float, default=10.0,
                    help="N = 1 only: the headline replica and load generator again over IPv4 loopback (the "
                         "image binds 0.0.0.0) for about this long, when the headline ran on ::1 (v4_* keys). "
                         "0 = skip")
    ap.add_argument("--plain-seconds", type=float, default=10.0,
                    help="N > 1 only: after the timed region every rank's load generator runs this long from its "
                         "own cores dealing its connections over all replicas, with no client placement, as a "
                         "LoadBalancer Service deals them (plain_* keys; `value` is untouched). 0 = skip")
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
                    help="print the core plan (one JSON line) and exit: of every slot of the node, or of "
                         "--replicas N replicas as an N-rank run would plan them")
    ap.add_argument("--replicas", type=int, default=0,
                    help="with --plan-only: plan this many replicas (ranks) on the node (0 = one per slot)")
    ap.add_argument("--slot-cores", type=int, default=0,
                    help="miniature node layout: rank r runs on only the first K physical cores of node slot "
                         "r (slots placed as the --gpu-slots node plan places them, across both sockets); "
                         "with --smt pair (the default here) each core carries a server worker and, on its "
                         "sibling, the load-generator thread driving it. 0 = off")
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
        host = a.host if a.host != "auto" else ("::1" if _can_bind("::1") else "127.0.0.1")
        plan = [{**_plan(a, local_world, avoid_busy=not a.no_avoid_busy),
                 "host": host,
                 "base_port": subruns.free_port_block(a.base_port, local_world, host),
                 "sink_port": sink[1] if sink else 0}]
        # the rank's own load-generator cores, for --plain-dealing (the r42 layout)
        plan[0]["own_loadgen"] = (_own_loadgen(plan[0]["cores"]) if not a.slot_cores
                                  else [p["loadgen"] for p in plan[0]["cores"]])
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
    # every CPU this job planned (all ranks' servers and load generators): a busy SMT sibling
    # outside this set is another tenant's
    job_cpus = sorted({c for p in plan[0]["cores"] for c in p["server"] + p["loadgen"]})
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
        per_conn = a.reqs_per_conn or a.warmup_reqs_per_conn
        w = None
        for _ in range(a.warmup):
            w = loadgen.run(per_conn)
        loadgen.reset()
        if not a.reqs_per_conn:
            # size the timed steps from the last warmup step: each step lasts about
            # --step-seconds; every rank takes the smallest size (the same work per replica)
            per_conn = 108000
            if w and w["elapsed_ns"] > 0:
                rate = w["requests"] / (w["elapsed_ns"] / 1e9)
                per_conn = max(100, int(rate * a.step_seconds / a.connections))
            if dist:
                sizes = [None] * world
                dist.all_gather_object(sizes, per_conn)
                per_conn = min(sizes)

        cuda = _cuda_sync_fn(local_rank)
        if dist:
            dist.barrier()
        cuda()
        span0 = span_counters(host, port, probe)
        m0 = subruns.metrics_counters(port, host, probe)
        sink0 = sink_stats(plan[0]["sink_port"]) if local_rank == 0 else {}
        tracer0 = thread_cpu_s(server.proc.pid, "hola-tracer")
        cpu0 = (proc_cpu_s(server.proc.pid), proc_cpu_s(loadgen.proc.pid))
        tcp0 = tcp_counters()
        thr0 = cgroup_cpu_stat()
        times0 = cpu_times()
        t0 = time.perf_counter()
        reqs = errs = 0
        for _ in range(a.steps):
            r = loadgen.run(per_conn)
            reqs += r["requests"]
            errs += r["errors"]
        if dist:
            dist.barrier()
        cuda()
        elapsed = time.perf_counter() - t0
        cpu1 = (proc_cpu_s(server.proc.pid), proc_cpu_s(loadgen.proc.pid))
        tracer1 = thread_cpu_s(server.proc.pid, "hola-tracer")
        span1 = span_counters(host, port, probe)
        m1 = subruns.metrics_counters(port, host, probe)
        locality1 = accept_locality(host, port, probe)
        locality = {k: v - locality0.get(k, 0) for k, v in locality1.items()}
        sink1 = sink_stats(plan[0]["sink_port"]) if local_rank == 0 else {}
        tcp1 = tcp_counters()
        thr1 = cgroup_cpu_stat()
        times1 = cpu_times()
        own = set(server_cpus) | set(load_cpus)
        st = loadgen.stats()
        mem = server.memory_kb()
        plain = None
        if dist and a.plain_seconds > 0 and not a.plain_dealing:
            # the topology-blind front on the same replicas, every rank at once (after the timed
            # region: `value` is untouched)
            loc_p0 = accept_locality(host, port, probe)
            dist.barrier()
            try:
                plain = subruns.plain_dealing_run(a, targets, local_rank, plan[0]["own_loadgen"][local_rank], bodies,
                                                  a.plain_seconds)
            except Exception as e:  # noqa: BLE001 - reported in the JSON
                plain = {"error": f"{type(e).__name__}: {e}"}
            dist.barrier()
            loc_p1 = accept_locality(host, port, probe)
            plain["locality"] = {k: v - loc_p0.get(k, 0) for k, v in loc_p1.items()}
        c1 = subruns.config2(a, host, port, server_cpus, load_cpus, bodies and [bodies[local_rank]],
                             job_cpus) if local_rank == 0 else None

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
                 # where the replica's and the load generator's time went
                 "server_loop": subruns.loop_block(m0, m1, reqs),
                 "loadgen_loop": subruns.loadgen_block(st, cpu1[1] - cpu0[1], reqs),
                 "startup_ms": server.startup_ms, "rss_peak_kb": mem.get("VmHWM", 0),
                 "tcp": {k: tcp1[k] - tcp0[k] for k in tcp1 if k in tcp0},
                 "cgroup": {k: thr1[k] - thr0[k] for k in thr1 if k in thr0},
                 "per_conn": per_conn, "plain": plain,
                 # host-wide busy share over the timed region of this rank's CPUs and of those of
                 # their SMT siblings that no part of this job uses (busy there = another tenant)
                 "host_load": subruns.host_load(times0, times1, own, job_cpus)}
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
    # Per-node sub-runs at N = 1 (BENCH and SCALE's first point), on the rank's CPUs once the
    # headline replica is gone: the as-deployed replica, the chaining path engineered and as
    # shipped, and the headline in the other SMT layout. Each is reported in the JSON (an
    # exception included) without touching `value`.
    subs: dict[str, dict | None] = {}
    if world == 1:
        rank_cpus = list(server_cpus) + list(load_cpus)
        pod_cpus = sorted(server_cpus)[:subruns.manifest_pod_cpus()]
        for key, secs, fn in (
                # the headline on the image's address family, when it ran on ::1
                ("v4", a.v4_seconds if host != "127.0.0.1" else 0,
                 lambda: subruns.v4_headline(a, args, server_cpus, load_cpus, conn_targets, job_cpus,
                                             bodies and [bodies[0]], a.v4_seconds)),
                ("deployed", a.deployed_seconds,
                 lambda: subruns.deployed(a, server_cpus, load_cpus, job_cpus, zipkin=a.deployed_zipkin)),
                # the same, sized as the manifests size one pod (limits.cpu: a 2-CPU cpuset), its
                # load generator on the rank's load-generator CPUs in the pod's L3 (as the
                # headline's is placed) ...
                ("deployed_pod", a.deployed_seconds,
                 lambda: subruns.deployed(a, pod_cpus, subruns.pod_loadgen_cpus(pod_cpus, load_cpus), job_cpus,
                                          zipkin=a.deployed_zipkin)),
                # ... and on all of them, across two L3s (round 5's deployed_pod_*): what clients
                # in another cache domain cost the pod (profiles/round6/01_pod_shape)
                ("deployed_pod_spanning", a.deployed_seconds / 2,
                 lambda: subruns.deployed(a, pod_cpus, load_cpus, job_cpus, zipkin=a.deployed_zipkin,
                                          seconds=a.deployed_seconds / 2)),
                ("chain", a.chain_seconds, lambda: subruns.chain(a, rank_cpus, job_cpus)),
                ("chain_shipped", a.chain_shipped_seconds,
                 lambda: subruns.chain(a, rank_cpus, job_cpus, shipped=True, seconds=a.chain_shipped_seconds)),
                ("alt", a.alt_seconds,
                 lambda: subruns.alt_layout(a, host, server_cpus, load_cpus, smt, job_cpus,
                                            bodies and [bodies[0]], a.alt_seconds))):
            if secs > 0:
                try:
                    subs[key] = fn()
                except Exception as e:  # noqa: BLE001 - reported in the JSON
                    subs[key] = {"error": f"{type(e).__name__}: {e}"}
    if dist and sink:
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
            # ... less the CPU both spent in polls that found nothing (spinning): the CPU that
            # did work, an efficiency figure that does not follow the spin (at saturation both
            # raw figures are the CPUs' wall time over the request count: equal by construction)
            **_busy_keys(gathered, total),
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
            # the server binary measured: release, source revision, x86-64 level, compiler
            "build": _build_line(),
            # every 2xx body of the timed region compared byte for byte with the expected one
            "body_checked": sum(g["body_checked"] for g in gathered),
            "body_mismatch": sum(g["body_mismatch"] for g in gathered),
            # BASELINE config 2 (1 connection, 1 replica), measured after the timed region
            **_c1_keys(gathered[0]["c1"]),
            # N = 1 only: the replica as the image and manifests run it (--shutdown-delay-ms 5000
            # --busy-poll-us auto, ZIPKIN_SERVER_URL set), same load generator
            **_deployed_keys(subs.get("deployed")),
            # ... in one pod's CPU limit (deploy/openshift: limits.cpu 2): what one pod of
            # BASELINE config 5 serves on its own, with the attribution of its CPU per request
            **_deployed_keys(subs.get("deployed_pod"), "deployed_pod", full=False),
            **{k: v for k, v in _deployed_keys(subs.get("deployed_pod_spanning"), "deployed_pod_spanning",
                                               full=False).items()
               if k.rsplit("deployed_pod_spanning_", 1)[-1] in (
                   "rps", "p99_ms", "server_cpu_us_per_req", "server_busy_cpu_us_per_req", "loadgen_cpus", "locality",
                   "error", "errors", "body_mismatch")},
            # N = 1 only: GET /api/hola-chaining through two replicas (the endpoint with real work
            # behind it), engineered (pool 128, logging off) and as shipped (pool 10, BASIC logging)
            **_chain_keys(subs.get("chain"), "chain"),
            **_chain_keys(subs.get("chain_shipped"), "chain_shipped"),
            # N = 1 only: the headline in the other SMT layout (BENCH <-> SCALE N = 1 comparison)
            **_alt_keys(subs.get("alt")),
            # N = 1 only: the headline over IPv4 loopback (the image's transport)
            **_v4_keys(subs.get("v4"), value),
            # N > 1 only: the same replicas behind a topology-blind front (no client placement)
            **_plain_keys([g["plain"] for g in gathered], value),
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
                "reqs_per_conn_per_step": gathered[0]["per_conn"],
                "step_sizing": (f"sized from the last warmup step to ~{a.step_seconds:g} s per step" if not a.reqs_per_conn
                                else "fixed (--reqs-per-conn)"),
                "pipeline": a.pipeline,
                "lb": ("client-side round-robin over all replicas from the rank's own cores, no client placement"
                       if a.plain_dealing else
                       "client-side, clients placed: " + plan[0]["cores"][local_rank].get("dealing", "round-robin")
                       + ". Each load-generator thread is pinned next to the replica(s) it drives; a LoadBalancer "
                         "Service places no client (the topology-blind figure is plain_* at N > 1)"),
                "loopback": host,
                # physical cores under the replica's server workers (with smt=pair the load
                # generator runs on their siblings; with smt=off on as many separate cores)
                "cores_per_replica": _phys_count(server_cpus),
                "physical_cores_per_slot": plan[0]["cores_per_slot"] if not a.slot_cores else a.slot_cores,
                "server_threads_per_replica": s_threads,
                "loadgen_threads_per_replica": len(load_cpus),
                "busy_poll_us": a.busy_poll_us,
                "server_busy_poll": a.server_busy_poll,
                "busy_poll_pause": a.busy_poll_pause,
                "epoll": "level" if a.epoll_lt else "edge",
                "smt": smt,
                "layout_note": _layout_note(plan[0]["gpu_slots"], smt, server_cpus, load_cpus, a.slot_cores),
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


def _plan(a, n: int, avoid_busy: bool = True) -> dict:
    """Core plan of `n` co-located replicas (one per rank) on this node, as rank 0 computes it.

    Each replica gets one GPU slot's share of the node: slot_cores(slots) physical cores
    (16 on the 16-CPU box and on a 2 x 64-core 8-GPU node), the SMT layout decided per node
    (pair when the node's CPU budget holds both threads of every slot's cores), so every N
    runs each replica on the same resources (weak scaling). With --slot-cores K each replica
    gets only the first K cores of its node slot (plan_slot_subset)."""
    slots = max(n, a.gpu_slots or _gpu_slots())
    if a.slot_cores:
        sub = plan_slot_subset(n, slots, a.slot_cores, a.smt if a.smt in ("off", "pair") else "auto")
        smt = sub[0]["smt"]
        cores = [{"server": p["server"], "loadgen": p["loadgen"], "thread_targets": [[r]] * len(p["loadgen"]),
                  "dealing": "round-robin over the replicas: each client thread drives the replica whose worker "
                             "shares its physical core (the node plan's per-connection placement)" if smt == "pair"
                             else "each client thread drives the replica in its own node slot"}
                 for r, p in enumerate(sub)]
        return {"cores": cores, "smt": smt, "gpu_slots": slots, "cores_per_slot": a.slot_cores}
    per_rank = min(a.cores or slot_cores(slots), max(1, cpu_budget() // n))
    smt = a.smt
    if smt == "auto":
        smt = "pair" if smt_fits(slots, per_rank) else "off"
    elif smt == "pair" and not smt_fits(slots, per_rank) and any(sibling_of(c) is not None
                                                                  for c in physical_cores()[:1]):
        # forced pairing inside a CPU budget that cannot hold both threads of every core: half
        # the physical cores, both threads each (a 16-CPU quota: 8 paired cores, as alt_* runs),
        # instead of 32 busy CPUs that the quota throttles to half speed
        per_rank = min(per_rank, max(1, cpu_budget() // (2 * n)))
    return {"cores": plan_replicas_with_loadgen(n, per_rank, a.server_threads, avoid_busy=avoid_busy, smt=smt),
            "smt": smt, "gpu_slots": slots, "cores_per_slot": per_rank}


def _plan_only(a) -> int:
    """The core plan of a whole node (one replica per GPU slot), or of --replicas N replicas,
    as rank 0 computes it, without starting anything: the cpu map such a run would use."""
    from hola_amd.utils.cpu import l3_domain, package_of, physical_cores

    slots = a.gpu_slots or max(1, _gpu_slots())
    n = a.replicas or slots
    p = _plan(a, n, avoid_busy=False)
    print(json.dumps({"gpu_slots": p["gpu_slots"], "replicas": n, "cores_per_slot": p["cores_per_slot"],
                      "smt": p["smt"], "cpu_budget": cpu_budget(),
                      "cgroup_quota": cgroup_cpu_quota(), "physical_cores": len(physical_cores()),
                      "ranks": [{"server": r["server"], "loadgen": r["loadgen"], "thread_targets": r["thread_targets"],
                                 "dealing": r["dealing"],
                                 "server_physical_cores": _phys_count(r["server"]),
                                 "server_sockets": sorted({package_of(c) for c in r["server"]}),
                                 "server_l3": sorted({l3_domain(c) for c in r["server"]}),
                                 "loadgen_sockets": sorted({package_of(c) for c in r["loadgen"]}),
                                 "siblings": {str(c): siblings(c) for c in r["server"] + r["loadgen"]}}
                                for r in p["cores"]]}), flush=True)
    return 0


def _phys_count(cpus) -> int:
    """Physical cores under a CPU list (SMT siblings counted once)."""
    return len({min(siblings(c)) for c in cpus})


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


def _layout_note(slots: int, smt: str, server_cpus, load_cpus, slot_cores_k: int = 0) -> str:
    """One line that tells a SCALE_rNN.json reader why its N=1 point differs from BENCH."""
    srv = _phys_count(server_cpus)
    if smt == "pair":
        how = (f"{srv} physical cores, each running a server worker on one SMT thread and the "
               f"load-generator thread that drives it on the other (--smt pair)")
    else:
        how = (f"{srv} physical cores of server workers and {_phys_count(load_cpus)} more of load-generator "
               f"threads, SMT siblings idle (--smt off)")
    mini = (f" Miniature layout (--slot-cores {slot_cores_k}): only the first {slot_cores_k} core(s) of each "
            f"node slot are used; this is not the 8-GPU node's curve." if slot_cores_k else "")
    return (f"{slots} GPU slot(s) on this node; each replica runs on {how}.{mini} The 1-GPU box (16-CPU quota) "
            f"runs smt=off and an unconstrained 8-GPU node smt=pair, so BENCH and SCALE's N=1 differ by layout, "
            f"not by code: at N=1 each carries the other layout's figure (alt_* keys).")


def _build_line() -> str:
    """`hola --version` of the server binary the replicas ran (HOLA_SERVER_BIN included)."""
    try:
        r = subprocess.run([str(binary("hola")), "--version"], capture_output=True, text=True, timeout=10)
        return r.stdout.strip() or r.stderr.strip()
    except Exception as e:  # noqa: BLE001 - reported, not fatal
        return f"unknown ({type(e).__name__})"


def _busy_keys(gathered: list[dict], total: int) -> dict:
    """server_/loadgen_busy_cpu_us_per_req and the loop accounting of the timed region, over
    all ranks: waits that could sleep per request, gaps between polls past 100 us / 1 ms /
    10 ms, the longest gap (replica: since start; load generator: in the timed region)."""
    n = max(1, total)
    srv = [g["server_loop"] for g in gathered]
    lg = [g["loadgen_loop"] for g in gathered]

    def loop_sum(rows, key):
        return sum(r.get(key, 0) for r in rows)

    def per_req(rows, key):  # a per-request figure of every rank, weighted by its requests
        if any(r.get(key) is None for r in rows):
            return None
        return round(sum(r[key] * g["requests"] for r, g in zip(rows, gathered)) / n, 1)

    return {
        "server_busy_cpu_us_per_req": round(1e6 * (sum(g["server_cpu_s"] for g in gathered) - loop_sum(srv, "idle_spin_s")) / n, 3),
        "loadgen_busy_cpu_us_per_req": round(1e6 * (sum(g["loadgen_cpu_s"] for g in gathered) - loop_sum(lg, "idle_spin_s")) / n, 3),
        # each side's own user-space instructions and cycles per request (hardware counters of
        # the serving threads; null where the host does not allow them): independent of each
        # other, where the CPU-time figures of two saturated peers are not
        "server_user_instr_per_req": per_req(srv, "user_instr_per_req"),
        "server_user_cycles_per_req": per_req(srv, "user_cycles_per_req"),
        "loadgen_user_instr_per_req": per_req(lg, "user_instr_per_req"),
        "loadgen_user_cycles_per_req": per_req(lg, "user_cycles_per_req"),
        "server_loop": {"idle_spin_s": round(loop_sum(srv, "idle_spin_s"), 3),
                        "blocking_waits_per_req": round(sum(r["blocking_waits_per_req"] for r in srv) / len(srv), 4),
                        "gaps_over_100us": loop_sum(srv, "gaps_over_100us"), "gaps_over_1ms": loop_sum(srv, "gaps_over_1ms"),
                        "gaps_over_10ms": loop_sum(srv, "gaps_over_10ms"),
                        "gap_max_since_start_us": max(r["gap_max_since_start_us"] for r in srv)},
        "loadgen_loop": {"idle_spin_s": round(loop_sum(lg, "idle_spin_s"), 3),
                         "polls": {k: sum(r["polls"][k] for r in lg) for k in lg[0]["polls"]},
                         "blocking_waits_per_req": round(sum(r["blocking_waits_per_req"] for r in lg) / len(lg), 4),
                         "gaps_over_100us": loop_sum(lg, "gaps_over_100us"), "gaps_over_1ms": loop_sum(lg, "gaps_over_1ms"),
                         "gaps_over_10ms": loop_sum(lg, "gaps_over_10ms"), "gap_max_us": max(r["gap_max_us"] for r in lg)}}


def _chain_keys(c: dict | None, p: str) -> dict:
    """chain_* (engineered) or chain_shipped_* keys of a chain sub-run."""
    if not c:
        return {}
    if "error" in c:
        return {f"{p}_error": c["error"]}
    h = c["hystrix"]
    n = max(1, c["body_checked"])
    out = {f"{p}_rps": round(c["rps"], 1), f"{p}_p50_ms": round(c["p50_ns"] / 1e6, 4),
           f"{p}_p99_ms": round(c["p99_ns"] / 1e6, 4), f"{p}_requests": c["requests"],
           f"{p}_elapsed_s": round(c["elapsed_s"], 2),
           f"{p}_errors": c["errors"], f"{p}_non2xx": c["non2xx"], f"{p}_body_checked": c["body_checked"],
           f"{p}_body_mismatch": c["body_mismatch"],
           # hola A's own CPU per chained request (it serves the client and calls B)
           f"{p}_a_cpu_us_per_req": round(c["a_cpu_us_per_req"], 3),
           f"{p}_b_cpu_us_per_req": round(c["b_cpu_us_per_req"], 3),
           # ... and what of it was work: without A's empty polls, and A's workers' own user-space
           # instructions and cycles (hardware counters; null where the host refuses them; they
           # include the empty polls' instructions, which bench/instr_ab.py's figure, measured
           # with busy-polling off, does not)
           f"{p}_a_busy_cpu_us_per_req": round(c["a_busy_cpu_us_per_req"], 3),
           f"{p}_a_user_instr_per_req": c["a_user_instr_per_req"], f"{p}_a_user_cycles_per_req": c["a_user_cycles_per_req"],
           # A's Hystrix command over the sub-run (its warm-up included)
           f"{p}_hystrix_success": h.get("SUCCESS", 0), f"{p}_hystrix_fallback": h.get("FALLBACK_SUCCESS", 0),
           f"{p}_hystrix_timeout": h.get("TIMEOUT", 0), f"{p}_hystrix_events": h,
           # A's circuit breaker: openings, and closings by the sleep window's trial or by a call
           # that was already running when it opened
           f"{p}_circuit": c.get("circuit", {}),
           # busy share of the sub-run's CPUs and of their SMT siblings outside the job
           f"{p}_host_load": c["host_load"],
           # client thread vs serving worker of every connection accepted in the sub-run, per hop
           f"{p}_locality": c["locality"],
           # adaptive busy-polling of A and B: spins that found work / ran out, back-offs, ms backed off
           f"{p}_spins": c["spins"], f"{p}_loadgen_busy_poll_us": c["loadgen_busy_poll_us"],
           f"{p}_cgroup_throttle": c["cgroup_throttle"],
           f"{p}_cpus": c["cpus"], f"{p}_pool": c["pool"]}
    if c.get("shipped"):
        # the timed responses that were A's own fallback (the pool of 10 or an open circuit)
        out[f"{p}_fallback_fraction"] = round(c["body_alt"] / n, 4)
        out[f"{p}_fallback_bodies"] = c["body_alt"]
        out[f"{p}_args"] = c.get("args", "")
    return out


def _v4_keys(r: dict | None, value: float) -> dict:
    if not r:
        return {}
    if "error" in r:
        return {"v4_error": r["error"]}
    return {"v4_rps": round(r["rps"], 1), "v4_p50_ms": round(r["p50_ns"] / 1e6, 4), "v4_p99_ms": round(r["p99_ns"] / 1e6, 4),
            "v4_p999_ms": round(r["p999_ns"] / 1e6, 4), "v4_requests": r["requests"], "v4_errors": r["errors"],
            "v4_body_checked": r["body_checked"], "v4_body_mismatch": r["body_mismatch"],
            "v4_elapsed_s": round(r["elapsed_s"], 2), "v4_server_cpu_us_per_req": round(r["cpu_us_per_req"], 3),
            "v4_vs_value": round(r["rps"] / value, 4) if value else None, "v4_host_load": r["host_load"]}


def _plain_keys(rows: list, value: float) -> dict:
    """plain_* over all ranks: node-wide req/s (requests / the longest rank's elapsed time),
    merged latency, errors, and where the connections' clients ran relative to the workers."""
    rows = [r for r in rows if r]
    if not rows:
        return {}
    errs = [r["error"] for r in rows if "error" in r]
    if errs:
        return {"plain_error": errs[0]}
    t = max(r["elapsed_s"] for r in rows)
    total = sum(r["requests"] for r in rows)
    hist = merge_hists([decode_hist(r["hist"]) for r in rows])
    loc: dict[str, int] = {}
    for r in rows:
        for k, v in r["locality"].items():
            loc[k] = loc.get(k, 0) + v
    n = sum(loc.values())
    rps = total / t if t > 0 else 0.0
    return {"plain_rps": round(rps, 1), "plain_p50_ms": round(percentile(hist, 50) / 1e6, 4),
            "plain_p99_ms": round(percentile(hist, 99) / 1e6, 4), "plain_requests": total,
            "plain_elapsed_s": round(t, 2), "plain_errors": sum(r["errors"] for r in rows),
            "plain_non2xx": sum(r["non2xx"] for r in rows), "plain_body_checked": sum(r["body_checked"] for r in rows),
            "plain_body_mismatch": sum(r["body_mismatch"] for r in rows),
            "plain_vs_value": round(rps / value, 4) if value else None,
            "plain_locality": {k: round(v / n, 4) for k, v in loc.items()} if n else {},
            "plain_loadgen_cpus": [r["load_cpus"] for r in rows]}


def _alt_keys(r: dict | None) -> dict:
    if not r:
        return {}
    if "error" in r:
        return {"alt_error": r["error"]}
    return {"alt_smt": r["smt"], "alt_rps": round(r["rps"], 1), "alt_p50_ms": round(r["p50_ns"] / 1e6, 4),
            "alt_p99_ms": round(r["p99_ns"] / 1e6, 4), "alt_requests": r["requests"], "alt_errors": r["errors"],
            "alt_body_checked": r["body_checked"], "alt_body_mismatch": r["body_mismatch"],
            "alt_elapsed_s": round(r["elapsed_s"], 2), "alt_physical_cores": r["physical_cores"],
            "alt_rps_per_physical_core": round(r["rps_per_physical_core"], 1),
            "alt_server_cpu_us_per_req": round(r["cpu_us_per_req"], 3), "alt_host_load": r["host_load"],
            "alt_cpus": {"server": r["server_cpus"], "loadgen": r["loadgen_cpus"]}}


def _deployed_keys(d: dict | None, p: str = "deployed", full: bool = True) -> dict:
    """deployed_* (or deployed_pod_*) keys of a deployed sub-run, with the attribution of its
    server CPU per request (subruns.attributed_closed_loop)."""
    if not d:
        return {}
    if "error" in d:
        return {f"{p}_error": d["error"]}
    out = {f"{p}_rps": round(d["rps"], 1), f"{p}_p50_ms": round(d["p50_ns"] / 1e6, 4),
           f"{p}_p99_ms": round(d["p99_ns"] / 1e6, 4), f"{p}_requests": d["requests"],
           f"{p}_elapsed_s": round(d["elapsed_s"], 2),
           f"{p}_errors": d["errors"], f"{p}_non2xx": d["non2xx"],
           f"{p}_body_checked": d["body_checked"], f"{p}_body_mismatch": d["body_mismatch"],
           # the replica's threads' CPU per request; ... less its loop's empty polls; and all
           # that its CPUs did per request (interrupt time included)
           f"{p}_server_cpu_us_per_req": round(d["cpu_us_per_req"], 3),
           f"{p}_server_busy_cpu_us_per_req": d["server_busy_cpu_us_per_req"],
           f"{p}_server_cpus_us_per_req": d["server_cpus_us_per_req"],
           # serving threads apart from the rest (tracer, logger), with context switches
           f"{p}_server_threads": d["server_threads"], f"{p}_server_loop": d["server_loop"],
           f"{p}_loadgen": d["loadgen"], f"{p}_tcp_per_req": d["tcp_per_req"],
           f"{p}_host_load": d["host_load"], f"{p}_host_load_server": d["host_load_server"],
           f"{p}_host_load_loadgen": d["host_load_loadgen"],
           f"{p}_locality": d["locality"],
           f"{p}_cpus": d["cpus"], f"{p}_loadgen_cpus": d["loadgen_cpus"], f"{p}_connections": d["connections"],
           f"{p}_loadgen_busy_poll_us": d["loadgen_busy_poll_us"]}
    if full:
        out.update({
            f"{p}_args": d["args"],
            # the image binds 0.0.0.0, as a pod on an IPv4 pod network: the client connects over
            # IPv4 loopback, where the headline uses ::1 (2.6 % apart, profiles/round1/r20_v6), which
            # is the in-bench gap between the two (profiles/round5/03_deployed_ab)
            f"{p}_loopback": "127.0.0.1",
            # ZIPKIN_SERVER_URL names the cluster's zipkin-query Service, which does not resolve
            # on a bare host: spans are recorded and dropped when the post fails
            f"{p}_env": d["env"], f"{p}_zipkin": d["zipkin"]})
    return out


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
