"""Checks that run on the MI355X box (marked `gpu`): the headline benchmark end to end on the
real host, and that the native artefacts are the code under test."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.gpu
def test_native_module_loaded_from_tree(native):
    # The tests exercise the in-tree C++ core, not a Python stand-in.
    assert Path(native.__file__).resolve().parent == ROOT / "hola_amd"
    assert native.java_format("Hola de %s", ["x"]) == b"Hola de x"


@pytest.mark.gpu
def test_bench_json_contract_on_host():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "3", "--warmup", "1",
                        "--reqs-per-conn", "200", "--c1-seconds", "2", "--deployed-seconds", "2",
                        "--chain-seconds", "2", "--chain-shipped-seconds", "2", "--alt-seconds", "2",
                        "--v4-seconds", "2"],
                       capture_output=True, text=True, timeout=600, env={**os.environ, "HOLA_BENCH_PORT": "18700"})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout[-2000:]  # the driver's contract: ONE JSON line
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out
    assert out["n_gpus"] == 1 and out["steps"] == 3 and out["warmup"] == 1
    assert out["errors"] == 0 and out["non2xx"] == 0
    assert out["value"] > 10000  # a pinned native replica on EPYC cores does far more than this
    assert out["p50_ms"] > 0 and out["p99_ms"] >= out["p50_ms"]
    # every timed response body was compared with the replica's greeting
    assert out["body_checked"] == out["requests"] and out["body_mismatch"] == 0
    # BASELINE config 2 ran after the timed region, and placement was reported
    assert out["c1_errors"] == 0 and out["c1_rps"] > 10000 and out["c1_body_checked"] == out["c1_requests"]
    # ... and the replica exactly as the image and manifests start it (adaptive busy-polling)
    assert out["deployed_errors"] == 0 and out["deployed_non2xx"] == 0 and out["deployed_rps"] > 10000
    assert "--shutdown-delay-ms 5000" in out["deployed_args"] and "--busy-poll-us auto" in out["deployed_args"]
    assert out["config"]["smt"] in ("off", "split", "pair") and "GPU slot" in out["config"]["layout_note"]
    assert abs(sum(out["locality"]["fraction"].values()) - 1.0) < 1e-3
    # config 2 carries its own host load
    hl_keys = {"own", "siblings", "l3_others", "irq_own", "steal_own"}
    assert set(out["c1_host_load"]) == hl_keys
    # ... and GET /api/hola-chaining through two replicas: every call a Hystrix SUCCESS, no
    # fallback or timeout, every body (three greetings, two hops) checked
    assert out["chain_errors"] == 0 and out["chain_non2xx"] == 0 and out["chain_rps"] > 10000, out
    assert out["chain_body_checked"] == out["chain_requests"] and out["chain_body_mismatch"] == 0
    assert out["chain_hystrix_fallback"] == 0 and out["chain_hystrix_timeout"] == 0
    assert out["chain_hystrix_success"] >= out["chain_requests"]  # its warm-up counts too
    assert out["chain_a_cpu_us_per_req"] > 0
    # A's own work per chained request, independent of the peer: busy CPU without empty polls,
    # and its workers' user-space instructions from hardware counters (the box allows them)
    assert 0 < out["chain_a_busy_cpu_us_per_req"] <= out["chain_a_cpu_us_per_req"] + 0.05
    assert out["chain_a_user_instr_per_req"] and 1000 < out["chain_a_user_instr_per_req"] < 20000, out
    # ... with what separates its two modes: host load, per-hop accept locality, spin counters
    assert set(out["chain_locality"]) == {"loadgen_to_a", "a_to_b"} and out["chain_spins"]["a"]
    assert set(out["chain_host_load"]) == hl_keys and set(out["deployed_host_load"]) == hl_keys
    # ... and as shipped (pool of 10, BASIC logging): every body is the two-hop answer or A's
    # fallback, the fraction is reported
    assert out["chain_shipped_pool"] == 10 and out["chain_shipped_body_mismatch"] == 0
    assert 0.0 <= out["chain_shipped_fallback_fraction"] <= 1.0
    # ... and the other SMT layout on the rank's cores (BENCH <-> SCALE N = 1)
    assert out["alt_errors"] == 0 and out["alt_smt"] != out["config"]["smt"] and out["alt_rps"] > 10000
    # the independent efficiency figure, the pod's attribution and the IPv4 headline
    assert 0 < out["server_busy_cpu_us_per_req"] <= out["server_cpu_us_per_req"]
    assert out["deployed_pod_server_busy_cpu_us_per_req"] > 0 and out["deployed_pod_tcp_per_req"]["OutSegs"] >= 1.9
    if out["config"]["loopback"] != "127.0.0.1":
        assert out["v4_errors"] == 0 and out["v4_rps"] > 10000


@pytest.mark.gpu
def test_bench_two_ranks_on_host():
    """The multi-replica path (torchrun, gloo barriers, client-side round-robin across
    replicas, cross-rank L3-aware load-generator placement) on the real host."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29517", str(ROOT / "bench.py"),
                        "--gpus", "2", "--steps", "3", "--warmup", "1", "--reqs-per-conn", "500",
                        "--c1-seconds", "1", "--deployed-seconds", "0", "--chain-seconds", "0",
                        "--plain-seconds", "2"],
                       capture_output=True, text=True, timeout=600,
                       env={**os.environ, "HOLA_BENCH_PORT": "18760"})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout[-2000:]  # gloo's "[Gloo] Rank N is connected" goes to stderr
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "replicas2"
    assert out["requests"] == 2 * 64 * 500 * 3
    assert out["errors"] == 0 and out["non2xx"] == 0
    assert set(out["config"]["cpu_map"]) == {"rank0", "rank1"}
    assert out["body_checked"] == out["requests"] and out["body_mismatch"] == 0
    # the planner keeps each load-generator thread in the L3 of the replica it drives
    loc = out["locality"]["fraction"]
    assert loc["same_core"] + loc["same_l3"] > 0.8, loc
    # ... and the same replicas behind a topology-blind front
    assert out["plain_errors"] == 0 and out["plain_body_mismatch"] == 0
    assert out["plain_body_checked"] == out["plain_requests"] > 0 and out["plain_rps"] > 10000
    assert abs(sum(out["plain_locality"].values()) - 1.0) < 1e-3 and "places no client" in out["config"]["lb"]


@pytest.mark.gpu
def test_tracing_as_deployed_on_host():
    """`bench.py --zipkin-sink`: a native collector attached, as ZIPKIN_SERVER_URL is in the
    reference image. Spans beyond the Brave-parity budget are dropped and counted, the rest
    reach the collector, and the request path does not slow down."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "4", "--warmup", "1",
                        "--reqs-per-conn", "20000", "--c1-seconds", "0", "--deployed-seconds", "0",
                        "--chain-seconds", "0", "--chain-shipped-seconds", "0", "--alt-seconds", "0", "--zipkin-sink",
                        "--v4-seconds", "0"],
                       capture_output=True, text=True, timeout=600, env={**os.environ, "HOLA_BENCH_PORT": "18720"})
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    tr = out["tracing"]
    assert out["errors"] == 0 and tr["mode"].startswith("collector")
    assert tr["sink_bad"] == 0 and tr["spans_per_s"]["reported"] > 0
    assert tr["spans_per_s"]["dropped_queue_full"] > 0
    assert out["value"] > 10000


@pytest.mark.gpu
def test_pipelined_bench_on_host():
    """`bench.py --pipeline 16` on the real host: 16 requests share each loopback segment."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--pipeline", "16", "--steps", "2", "--warmup", "1",
                        "--reqs-per-conn", "16000", "--c1-seconds", "0", "--deployed-seconds", "0",
                        "--chain-seconds", "0", "--chain-shipped-seconds", "0", "--alt-seconds", "0",
                        "--v4-seconds", "0"],
                       capture_output=True, text=True, timeout=300,
                       env={**os.environ, "HOLA_BENCH_PORT": "18780"})
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["errors"] == 0 and out["non2xx"] == 0 and out["requests"] == 64 * 16000 * 2
    assert out["config"]["pipeline"] == 16
    assert out["value"] > 1_000_000  # a loaded box still does several times this
    if out["tcp_per_req"]:
        assert out["tcp_per_req"]["OutSegs"] < 0.5


@pytest.mark.gpu
def test_proxy_front_on_host():
    """The L4 round-robin proxy between the load generator and a replica, in the mirrored core
    plan on the real host's L3 domains."""
    import contextlib
    import io

    from hola_amd.parallel import scaling

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        scaling.main(["--replicas", "1", "--lb", "proxy", "--duration", "2", "--warmup", "0.5"])
    row = json.loads(next(l for l in buf.getvalue().splitlines() if l.startswith("{")))
    assert row["errors"] == 0 and row["non2xx"] == 0 and row["lb"] == "proxy"
    assert row["rps"] > 100_000


@pytest.mark.gpu
def test_manifests_execute_on_host():
    """BASELINE config 5 on the real host, at 0.1x the probe timings: hola-dc.yaml + the
    translation ConfigMap + patch as 8 pods behind the Service, a rollout under 512
    connections with the manifests' shutdown delay (0 errors), a SIGKILLed pod rejoining, a
    ConfigMap edit reaching every pod (bench/kube_rollout.py; profiles/round3/01_kube has the
    run at real timings)."""
    out_dir = ROOT / "gpurun_out" / "pytest_kube"
    r = subprocess.run([sys.executable, str(ROOT / "bench" / "kube_rollout.py"), "--out", str(out_dir),
                        "--time-scale", "0.1", "--configmap-sync-s", "5", "--policy", "none"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["greetings_seen"] == 8 and res["greetings_match_pods"]
    assert res["rollout_with_delay"]["errors"] == 0 and res["rollout_with_delay"]["non2xx"] == 0
    assert res["rollout_with_delay"]["requests"] > 10000
    assert res["sigkill"]["restarts"] == 1
    assert res["configmap_edit_all_pods_s"] < 60


def _node_plan(slots: int, replicas: int = 0) -> dict:
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--plan-only", "--gpu-slots", str(slots),
                        "--ignore-quota", "--replicas", str(replicas)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
def test_eight_slot_plan_on_the_real_topology():
    """The 8-GPU node's layout (SCALE N = 8), planned on this host's real topology with the
    box's CPU quota set aside: 8 replica slots of 16 physical cores,
    every CPU used once; each replica's server workers inside one socket, on L3 domains no
    other replica's workers use; and with --smt pair every load-generator thread on the other
    SMT thread of a core of the replica it drives (the client and the worker serving its
    connections share that physical core)."""
    from hola_amd.utils.cpu import physical_cores

    if len(physical_cores()) < 128:
        pytest.skip("the 8-slot layout needs the node's 2 x 64 physical cores")
    plan = _node_plan(8)
    ranks = plan["ranks"]
    assert plan["gpu_slots"] == 8 and len(ranks) == 8 and plan["smt"] == "pair", plan["smt"]
    assert plan["cores_per_slot"] == 16
    used = [c for r in ranks for c in r["server"] + r["loadgen"]]
    assert len(used) == len(set(used)) == 256, "a CPU planned twice"
    l3_owner: dict[int, int] = {}
    for i, r in enumerate(ranks):
        assert len(r["server"]) == len(r["loadgen"]) == 16
        assert len(r["server_sockets"]) == 1, (i, r["server_sockets"])
        for d in r["server_l3"]:
            assert l3_owner.setdefault(d, i) == i, f"L3 {d} holds workers of replicas {l3_owner[d]} and {i}"
    for i, r in enumerate(ranks):
        assert r["thread_targets"], i
        for t, l_cpu in enumerate(r["loadgen"]):
            target = ranks[r["thread_targets"][t][0]]
            sib = set(r["siblings"][str(l_cpu)]) - {l_cpu}
            assert sib & set(target["server"]), (i, t, l_cpu)
    out = ROOT / "gpurun_out" / "plan8.json"
    out.parent.mkdir(exist_ok=True)
    out.write_text(json.dumps(plan, indent=1))


@pytest.mark.gpu
def test_node_plan_gives_every_n_the_same_replica_shape():
    """SCALE's weak-scaling curve on the 8-GPU node: at N = 1, 2, 4 and 8 (--plan-only
    --replicas N, planned on this host's real topology with the quota set aside) every
    replica gets the same shape: 16 physical cores of server workers, smt=pair, its workers
    inside one socket, and every load-generator thread on the other SMT thread of a core of
    the replica it drives."""
    from hola_amd.utils.cpu import physical_cores

    if len(physical_cores()) < 128:
        pytest.skip("the 8-slot layout needs the node's 2 x 64 physical cores")
    shapes = {}
    for n in (1, 2, 4, 8):
        plan = _node_plan(8, n)
        ranks = plan["ranks"]
        assert plan["replicas"] == n and len(ranks) == n and plan["smt"] == "pair", (n, plan["smt"])
        used = [c for r in ranks for c in r["server"] + r["loadgen"]]
        assert len(used) == len(set(used)) == 32 * n, n
        for i, r in enumerate(ranks):
            assert r["server_physical_cores"] == 16 and len(r["loadgen"]) == 16, (n, i)
            assert len(r["server_sockets"]) == 1, (n, i, r["server_sockets"])
            for t, l_cpu in enumerate(r["loadgen"]):
                target = ranks[r["thread_targets"][t][0]]
                assert (set(r["siblings"][str(l_cpu)]) - {l_cpu}) & set(target["server"]), (n, i, t)
        shapes[n] = plan
    out = ROOT / "gpurun_out" / "plans_by_n.json"
    out.parent.mkdir(exist_ok=True)
    out.write_text(json.dumps(shapes, indent=1))


@pytest.mark.gpu
def test_eight_ranks_run_under_the_node_plan():
    """The N = 8 torchrun command under the 8-slot plan for a couple of tiny steps. Inside
    the box's 16-CPU quota the 256 threads are squeezed, so the throughput means nothing (no
    scaling curve is measured here); what is checked is that the layout runs end to end with
    no errors, and that accept steering puts each connection on the worker that shares its
    client thread's physical core."""
    from hola_amd.utils.cpu import physical_cores

    if len(physical_cores()) < 128:
        pytest.skip("the 8-slot layout needs the node's 2 x 64 physical cores")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", "29537", str(ROOT / "bench.py"),
                        "--gpus", "8", "--gpu-slots", "8", "--ignore-quota", "--steps", "2", "--warmup", "1",
                        "--reqs-per-conn", "200", "--busy-poll-us", "0", "--c1-seconds", "0",
                        "--deployed-seconds", "0", "--chain-seconds", "0", "--plain-seconds", "0"],
                       capture_output=True, text=True, timeout=300,
                       env={**os.environ, "HOLA_BENCH_PORT": "18800", "HOLA_BENCH_CUDA_SYNC": "0"})
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / "n8_plan_run.json").write_text(json.dumps(out, indent=1))
    assert out["n_gpus"] == 8 and out["config"]["smt"] == "pair" and out["config"]["gpu_slots_on_node"] == 8
    assert out["requests"] == 8 * 64 * 200 * 2
    assert out["errors"] == 0 and out["non2xx"] == 0 and out["body_mismatch"] == 0
    assert out["locality"]["fraction"]["same_core"] >= 0.9, out["locality"]
    # labels: each replica is 16 physical cores of server workers; its SMT siblings are the
    # job's own load-generator threads, so no sibling load is charged to other tenants
    assert out["config"]["cores_per_replica"] == 16 and "16 physical cores" in out["config"]["layout_note"]
    assert all(h["siblings"] is None for h in out["host_load"]), out["host_load"]


@pytest.mark.gpu
def test_steering_keeps_one_l3s_clients_in_their_l3():
    """Accept steering on the real topology: a replica with two workers in each of two L3
    domains, and 24 connections opened from one client CPU of the first domain (a pool warming
    up one L3 first). Every connection is served in the client's L3: the balance rule lets a
    worker take up to twice its fair share (+8) before it refuses a steered connection; the
    old rule (the least loaded worker + 8) sent a third of them across."""
    import socket

    from hola_amd.server import HolaProcess
    from hola_amd.utils.cpu import allowed_cpus, l3_domain, physical_cores

    by_dom: dict[int, list[int]] = {}
    for c in physical_cores(allowed_cpus()):
        by_dom.setdefault(l3_domain(c), []).append(c)
    doms = [d for d, cs in by_dom.items() if len(cs) >= 3][:2]
    if len(doms) < 2:
        pytest.skip("needs two L3 domains with three cores each")
    x, y = by_dom[doms[0]], by_dom[doms[1]]
    server_cpus = [x[0], x[1], y[0], y[1]]
    with HolaProcess(threads=4, cpu_list=",".join(map(str, server_cpus)), env={"HOSTNAME": "s"},
                     log_level="warn") as s:
        old = os.sched_getaffinity(0)
        os.sched_setaffinity(0, {x[2]})
        try:
            conns = []
            for _ in range(24):
                c = socket.create_connection(("127.0.0.1", s.port), timeout=5)
                c.sendall(b"GET /api/hola HTTP/1.1\r\nHost: x\r\n\r\n")
                assert c.recv(4096).startswith(b"HTTP/1.1 200")
                conns.append(c)
        finally:
            os.sched_setaffinity(0, old)
        metrics = s.get("/metrics")[2].decode()
        for c in conns:
            c.close()
    loc = {l.split('"')[1]: int(float(l.split()[-1])) for l in metrics.splitlines()
           if l.startswith("hola_accept_locality_total{")}
    assert loc.get("same_l3", 0) + loc.get("same_core", 0) >= 24, loc


def _two_l3s(n: int = 3):
    from hola_amd.utils.cpu import allowed_cpus, l3_domain, physical_cores

    by_dom: dict[int, list[int]] = {}
    for c in physical_cores(allowed_cpus()):
        by_dom.setdefault(l3_domain(c), []).append(c)
    doms = [d for d, cs in by_dom.items() if len(cs) >= n][:2]
    if len(doms) < 2:
        pytest.skip(f"needs two L3 domains with {n} cores each")
    return by_dom[doms[0]], by_dom[doms[1]]


@pytest.mark.gpu
def test_proxy_topology_hints_keep_sessions_in_the_clients_l3():
    """hola_rrproxy with topology hints (backend h:p@cpus): a session accepted by the proxy
    thread in the client's L3 goes to the replica in that L3, so client, proxy and server share
    one cache domain (without hints the round-robin crosses L3s for half of them)."""
    import socket

    from hola_amd.parallel.replicas import RRProxy
    from hola_amd.server import HolaProcess

    x, y = _two_l3s()
    with HolaProcess(threads=1, cpu_list=str(x[0]), env={"HOSTNAME": "x"}, log_level="warn") as a, \
            HolaProcess(threads=1, cpu_list=str(y[0]), env={"HOSTNAME": "y"}, log_level="warn") as b, \
            RRProxy([("127.0.0.1", a.port), ("127.0.0.1", b.port)], threads=2, cpu_list=f"{x[1]},{y[1]}",
                    backend_cpus=[[x[0]], [y[0]]]) as px:
        old = os.sched_getaffinity(0)
        bodies = []
        try:
            for cpu, want in ((x[2], b"Hola de x"), (y[2], b"Hola de y")):
                os.sched_setaffinity(0, {cpu})
                for _ in range(16):
                    with socket.create_connection(("127.0.0.1", px.port), timeout=5) as c:
                        c.sendall(b"GET /api/hola HTTP/1.1\r\nHost: x\r\nConnection: close\r\n\r\n")
                        data = b""
                        while b"\r\n\r\n" not in data or not data.endswith(want):
                            chunk = c.recv(4096)
                            if not chunk:
                                break
                            data += chunk
                    bodies.append((cpu, data.split(b"\r\n\r\n", 1)[-1] == want))
        finally:
            os.sched_setaffinity(0, old)
    assert all(ok for _, ok in bodies), bodies
