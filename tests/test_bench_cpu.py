"""bench.py's output contract, exercised on CPU with a tiny run (1 rank, and 2 ranks over
gloo) — the same code path the driver runs on the MI355X node."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config")


def run(cmd, port):
    # the IPv4 and topology-blind sub-runs (10 s each by default) only where a test asks for them
    for flag in ("--v4-seconds", "--plain-seconds"):
        if flag not in cmd:
            cmd = cmd + [flag, "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env={**os.environ, "HOLA_BENCH_PORT": str(port)})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout  # exactly one JSON line on stdout
    return json.loads(lines[0])


def test_bench_one_rank():
    out = run([sys.executable, str(ROOT / "bench.py"), "--steps", "2", "--warmup", "1", "--reqs-per-conn", "100",
               "--c1-reqs", "3000", "--deployed-seconds", "0", "--chain-seconds", "0", "--chain-shipped-seconds", "0", "--alt-seconds", "0"], 18800)
    for k in KEYS:
        assert k in out
    assert out["metric"] == json.loads((ROOT / "BASELINE.json").read_text())["metric"]
    assert out["n_gpus"] == 1 and out["steps"] == 2 and out["warmup"] == 1
    assert out["requests"] == 64 * 100 * 2 and out["errors"] == 0
    # every timed response body was compared with "Hola de replica-0"
    assert out["body_checked"] == out["requests"] and out["body_mismatch"] == 0
    # BASELINE config 2 sub-run (1 connection), outside the timed region
    assert out["c1_requests"] == 3000 and out["c1_errors"] == 0 and out["c1_body_checked"] == 3000
    assert out["c1_rps"] > 0 and 0 < out["c1_p50_ms"] <= out["c1_p99_ms"]
    assert out["scaling"] == "weak" and out["higher_is_better"] is True and out["vs_baseline"] is None
    assert out["build"].startswith("hola 0.0.1-SNAPSHOT (revision ")  # the binary measured
    assert out["config"]["global_batch"] == 64 and out["config"]["parallelism"] == "replicas1"
    assert abs(out["value"] - out["requests"] / (out["ms_per_step"] * out["steps"] / 1000)) / out["value"] < 0.01
    # loopback TCP: at least one request and one response segment per request
    if out["tcp_per_req"]:
        assert out["tcp_per_req"]["OutSegs"] >= 1.9


def test_bench_auto_steps_and_node_subruns():
    """--reqs-per-conn 0 (the default): the timed steps are sized from the last warmup step
    and the JSON says how big they were; at N = 1 the per-node sub-runs report the deployed
    replica with its host load, the chain engineered and as shipped (fallbacks counted apart,
    per-hop accept locality, both replicas' busy-poll counters) and the other SMT layout."""
    out = run([sys.executable, str(ROOT / "bench.py"), "--steps", "2", "--warmup", "2", "--warmup-reqs-per-conn",
               "200", "--step-seconds", "0.2", "--c1-seconds", "0", "--deployed-seconds", "0.5",
               "--chain-seconds", "0.5", "--chain-shipped-seconds", "0.5", "--alt-seconds", "0.5",
               "--v4-seconds", "0.5"], 18870)
    per = out["config"]["reqs_per_conn_per_step"]
    assert per >= 100 and out["requests"] == 64 * per * 2 and out["errors"] == 0
    assert out["config"]["step_sizing"].startswith("sized from the last warmup step")
    # the replica's own cores, not its load generator's
    from hola_amd.utils.cpu import parse_cpu_list, siblings
    srv = parse_cpu_list(out["config"]["cpu_map"]["rank0"]["server"])
    assert out["config"]["cores_per_replica"] == len({min(siblings(c)) for c in srv})
    assert out["deployed_errors"] == 0 and out["deployed_body_checked"] == out["deployed_requests"] > 0
    hl_keys = {"own", "siblings", "l3_others", "irq_own", "steal_own"}
    assert set(out["deployed_host_load"]) == hl_keys and out["deployed_zipkin"] == "deployed"
    assert set(out["host_load"][0]) == hl_keys
    assert out["deployed_loopback"] == "127.0.0.1"  # the image binds 0.0.0.0: IPv4, as a pod
    # every sub-run is one continuous run of its length, its warm-up uncounted
    assert abs(out["deployed_elapsed_s"] - 0.5) < 0.1 and abs(out["chain_elapsed_s"] - 0.5) < 0.1
    assert set(out["chain_circuit"]) == {"open", "closed_trial", "closed_inflight"}
    # ... and sized as the manifests size a pod (limits.cpu 2)
    assert len(parse_cpu_list(out["deployed_pod_cpus"])) == 2 and out["deployed_pod_errors"] == 0
    assert out["deployed_pod_rps"] > 0
    # ... with the attribution of its CPU per request
    assert 0 < out["deployed_pod_server_busy_cpu_us_per_req"] <= out["deployed_pod_server_cpu_us_per_req"] + 0.05
    assert set(out["deployed_pod_server_threads"]) <= {"workers", "other"} and "workers" in out["deployed_pod_server_threads"]
    assert {"blocking_waits_per_req", "gaps_over_100us", "spins"} <= set(out["deployed_pod_server_loop"])
    assert {"polls", "busy_cpu_us_per_req", "blocking_waits_per_req"} <= set(out["deployed_pod_loadgen"])
    assert set(out["deployed_pod_host_load_server"]) == hl_keys and out["deployed_pod_connections"] == 64
    # the headline's independent efficiency figures
    assert 0 < out["server_busy_cpu_us_per_req"] <= out["server_cpu_us_per_req"]
    assert 0 < out["loadgen_busy_cpu_us_per_req"] <= out["loadgen_cpu_us_per_req"]
    assert {"idle_spin_s", "blocking_waits_per_req", "gap_max_since_start_us"} <= set(out["server_loop"])
    assert {"polls", "gap_max_us"} <= set(out["loadgen_loop"])
    # the headline again over IPv4 loopback, when the headline ran on ::1
    if out["config"]["loopback"] != "127.0.0.1":
        assert out["v4_errors"] == 0 and out["v4_body_checked"] == out["v4_requests"] > 0
        assert out["v4_vs_value"] > 0
    assert out["chain_errors"] == 0 and out["chain_hystrix_fallback"] == 0 and out["chain_pool"] == 128
    assert 0 < out["chain_a_busy_cpu_us_per_req"] <= out["chain_a_cpu_us_per_req"] + 0.05
    assert "chain_a_user_instr_per_req" in out and "chain_a_user_cycles_per_req" in out
    assert set(out["chain_locality"]) == {"loadgen_to_a", "a_to_b"}
    assert abs(sum(out["chain_locality"]["a_to_b"].values()) - 1.0) < 1e-3
    assert {"hit", "miss", "backoffs", "backoff_ms"} <= set(out["chain_spins"]["a"])
    # as shipped: every body is the two-hop answer or A's own fallback, and both are counted
    assert out["chain_shipped_pool"] == 10 and out["chain_shipped_errors"] == 0
    assert out["chain_shipped_body_mismatch"] == 0 and 0.0 <= out["chain_shipped_fallback_fraction"] <= 1.0
    assert "--shutdown-delay-ms 5000" in out["chain_shipped_args"]
    assert out["chain_shipped_hystrix_success"] + out["chain_shipped_hystrix_fallback"] >= out["chain_shipped_requests"]
    assert out["alt_smt"] == ("pair" if out["config"]["smt"] == "off" else "off") and out["alt_errors"] == 0
    assert out["alt_body_checked"] == out["alt_requests"] > 0


def test_plan_only_replicas():
    """--plan-only --replicas N: the plan an N-rank run would use (here on the container's CPUs)."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--plan-only", "--replicas", "2", "--gpu-slots", "2"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    plan = json.loads(r.stdout.strip().splitlines()[-1])
    assert plan["replicas"] == 2 and len(plan["ranks"]) == 2
    used = [c for rk in plan["ranks"] for c in rk["server"]]
    assert len(used) == len(set(used))
    assert all(rk["server_physical_cores"] >= 1 for rk in plan["ranks"])


def test_bench_two_ranks_gloo():
    out = run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", "29561", str(ROOT / "bench.py"), "--gpus", "2",
               "--steps", "2", "--warmup", "1", "--reqs-per-conn", "100", "--c1-reqs", "2000",
               "--plain-seconds", "0.5"], 18820)
    assert out["n_gpus"] == 2 and out["requests"] == 2 * 64 * 100 * 2
    # the topology-blind front after the timed region: every body checked
    assert out["plain_errors"] == 0 and out["plain_body_checked"] == out["plain_requests"] > 0
    assert out["plain_body_mismatch"] == 0 and out["plain_rps"] > 0 and len(out["plain_loadgen_cpus"]) == 2
    assert abs(sum(out["plain_locality"].values()) - 1.0) < 1e-3
    assert "places no client" in out["config"]["lb"]
    # connections are dealt over both replicas; each body must name the replica behind it
    assert out["body_checked"] == out["requests"] and out["body_mismatch"] == 0 and out["errors"] == 0
    assert out["c1_requests"] == 2000 and out["c1_errors"] == 0
    assert out["config"]["global_batch"] == 128


def test_bench_four_ranks_gloo():
    """N=4 (BASELINE config 4 shape, scaled down): every rank's load generator deals its 64
    connections over all 4 replicas; the JSON line reports the node-wide total."""
    out = run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
               "--master-addr", "127.0.0.1", "--master-port", "29563", str(ROOT / "bench.py"), "--gpus", "4",
               "--steps", "2", "--warmup", "1", "--reqs-per-conn", "50", "--c1-seconds", "0"], 18840)
    assert out["n_gpus"] == 4 and out["requests"] == 4 * 64 * 50 * 2
    assert out["errors"] == 0 and out["non2xx"] == 0
    assert out["body_checked"] == out["requests"] and "c1_rps" not in out
    # every accepted connection's client/worker placement is reported, per replica
    loc = out["locality"]
    assert loc["accepted"] >= 4 * 64 and len(loc["per_replica"]) == 4
    assert abs(sum(loc["fraction"].values()) - 1.0) < 1e-3
    assert out["config"]["global_batch"] == 256 and out["config"]["parallelism"] == "replicas4"
    from hola_amd.utils.cpu import parse_cpu_list
    cpus = [c for r in out["config"]["cpu_map"].values() for side in r.values() for c in parse_cpu_list(side)]
    assert len(cpus) == len(set(cpus))  # disjoint core sets across ranks


def test_bench_pipelined():
    """--pipeline 16 (wrk's pipeline.lua): a step still completes connections x reqs-per-conn
    requests, every response is counted and checked, and the setting is recorded."""
    out = run([sys.executable, str(ROOT / "bench.py"), "--steps", "2", "--warmup", "1", "--reqs-per-conn", "160",
               "--pipeline", "16", "--c1-seconds", "0", "--deployed-seconds", "0", "--chain-seconds", "0", "--chain-shipped-seconds", "0", "--alt-seconds", "0"], 18860)
    assert out["requests"] == 64 * 160 * 2 and out["errors"] == 0 and out["non2xx"] == 0
    assert out["config"]["pipeline"] == 16 and "16 pipelined" in out["data"]
    # 16 requests per segment each way: far fewer than 2 segments per request
    if out["tcp_per_req"]:
        assert out["tcp_per_req"]["OutSegs"] < 1.0


def test_loadgen_counts_wrong_bodies_as_errors():
    """A server answering 200 with the wrong bytes must not count as good throughput."""
    from hola_amd.parallel.loadgen import run_duration
    from hola_amd.server import HolaProcess

    with HolaProcess(env={"HOSTNAME": "hx"}, threads=1) as s:
        good = run_duration([("127.0.0.1", s.port)], 2, 1, 0.3, warmup_s=0.1, expect_bodies=["Hola de hx"])
        bad = run_duration([("127.0.0.1", s.port)], 2, 1, 0.3, warmup_s=0.1, expect_bodies=["Hola de hy"])
        learned = run_duration([("127.0.0.1", s.port)], 2, 1, 0.3, warmup_s=0.1, verify_body=True)
    assert good["latency"]["body_mismatch"] == 0 and good["latency"]["errors"] == 0
    assert good["latency"]["body_checked"] == good["latency"]["count"] > 0
    assert bad["latency"]["body_mismatch"] == bad["latency"]["count"] > 0
    assert bad["latency"]["errors"] >= bad["latency"]["body_mismatch"]
    assert learned["latency"]["body_mismatch"] == 0 and learned["latency"]["body_checked"] > 0


def test_loadgen_conn_targets_pin_connections_to_replicas():
    """--conn-targets fixes each connection's replica (the planner's L3 groups); an index
    outside --targets is rejected before any connection is made."""
    import subprocess

    from hola_amd.native import binary
    from hola_amd.parallel.loadgen import run_duration
    from hola_amd.server import HolaProcess

    with HolaProcess(env={"HOSTNAME": "a"}, threads=1) as a, HolaProcess(env={"HOSTNAME": "b"}, threads=1) as b:
        targets = [("127.0.0.1", a.port), ("127.0.0.1", b.port)]
        # all 4 connections on replica 1: every body must be b's greeting
        out = run_duration(targets, 4, 2, 0.3, warmup_s=0.1, expect_bodies=["Hola de a", "Hola de b"])
        assert out["latency"]["body_mismatch"] == 0
        cmd = [str(binary("hola_loadgen")), "--targets", f"127.0.0.1:{a.port},127.0.0.1:{b.port}", "-c", "4",
               "-t", "2", "--duration", "0.3", "--conn-targets", "1,1,1,1", "--expect-body", "Hola de b",
               "--expect-body", "Hola de b"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=60)
        assert r.returncode == 0, r.stderr
        lat = json.loads(r.stdout.strip().splitlines()[-1])["latency"]
        assert lat["body_mismatch"] == 0 and lat["body_checked"] == lat["count"] > 0
        bad = subprocess.run(cmd[:-4] + ["--conn-targets", "0,2"], capture_output=True, text=True, timeout=60)
        assert bad.returncode == 2 and "out of range" in bad.stderr


def test_loadgen_alt_body_counted_apart():
    """--alt-body: a response equal to an accepted second answer (the shipped chain's Hystrix
    fallback) is counted in body_alt, not as a mismatch; anything else still is one."""
    from hola_amd.parallel.loadgen import run_duration
    from hola_amd.server import HolaProcess

    with HolaProcess(env={"HOSTNAME": "hx"}, threads=1) as s:
        alt = run_duration([("127.0.0.1", s.port)], 2, 1, 0.3, warmup_s=0.1, expect_bodies=["Hola de hy"],
                           alt_bodies=["Hola de hz", "Hola de hx"])
        bad = run_duration([("127.0.0.1", s.port)], 2, 1, 0.3, warmup_s=0.1, expect_bodies=["Hola de hy"],
                           alt_bodies=["Hola de hz"])
    assert alt["latency"]["body_mismatch"] == 0 and alt["latency"]["errors"] == 0
    assert alt["latency"]["body_alt"] == alt["latency"]["body_checked"] == alt["latency"]["count"] > 0
    assert bad["latency"]["body_alt"] == 0 and bad["latency"]["body_mismatch"] == bad["latency"]["count"] > 0


def test_loadgen_runfor_counts_only_after_its_warm_up():
    """`runfor MS WARM_MS`: one continuous run whose first WARM_MS go uncounted; the reply's
    requests, the histogram and the body counts cover the measured part only, and elapsed is
    that part's length. A plain `run` after it counts everything again."""
    import time

    from hola_amd.parallel.loadgen import ControlledLoadgen
    from hola_amd.server import HolaProcess

    with HolaProcess(env={"HOSTNAME": "hx"}, threads=1) as s:
        lg = ControlledLoadgen([("127.0.0.1", s.port)], 4, 1, expect_bodies=["Hola de hx"])
        try:
            lg.reset()
            t0 = time.monotonic()
            r = lg.run_for(0.6, 0.4)
            wall = time.monotonic() - t0
            st = lg.stats()
            lg.reset()
            plain = lg.run(50)
        finally:
            lg.close()
    assert r["errors"] == 0 and r["requests"] > 0
    assert 0.55e9 <= r["elapsed_ns"] <= 0.8e9 and wall >= 0.95  # the warm-up ran, uncounted
    assert st["count"] == st["body_checked"] == r["requests"] and st["body_mismatch"] == 0
    assert plain["requests"] == 4 * 50 and plain["errors"] == 0


def test_bench_slot_cores_miniature_two_ranks():
    """--slot-cores 1: each rank runs on the first physical core of its node slot (the
    miniature weak-scaling layout), and the JSON says so rather than passing for the node's."""
    out = run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", "29565", str(ROOT / "bench.py"), "--gpus", "2",
               "--gpu-slots", "4", "--slot-cores", "1", "--steps", "2", "--warmup", "1", "--reqs-per-conn", "50",
               "--c1-seconds", "0"], 18880)
    assert out["n_gpus"] == 2 and out["errors"] == 0 and out["requests"] == 2 * 64 * 50 * 2
    c = out["config"]
    assert c["cores_per_replica"] == 1 and c["physical_cores_per_slot"] == 1
    assert "Miniature layout (--slot-cores 1)" in c["layout_note"] and "not the 8-GPU node's curve" in c["layout_note"]


def test_scaling_miniature_weak_efficiency():
    """hola_amd.parallel.scaling --slot-cores: N = 1 and 2 on the miniature plan, every LB mode;
    the table reports total / (N x N=1)."""
    import contextlib
    import io

    from hola_amd.parallel import scaling

    for lb in ("client", "reuseport", "proxy"):
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            scaling.main(["--slot-cores", "1", "--slots", "2", "--replicas", "1,2", "--lb", lb, "--duration", "0.4",
                          "--warmup", "0.1"])
        rows = [json.loads(l) for l in buf.getvalue().splitlines() if l.startswith("{")]
        assert [r["replicas"] for r in rows] == [1, 2] and all(r["errors"] == 0 for r in rows), rows
        assert rows[0]["efficiency"] == 1.0 and rows[1]["efficiency"] > 0 and rows[1]["slot_cores"] == 1
        assert "efficiency = total / (N x N=1)" in buf.getvalue()


def test_forced_smt_pair_stays_inside_the_cpu_budget(monkeypatch):
    """`--smt pair` under a budget that cannot hold both threads of a slot's cores (the 1-GPU
    box: 16 CPUs, 16 cores per slot) pairs half the cores instead of running 32 busy CPUs that
    the quota throttles to half speed; with room for both threads the slot keeps its cores,
    and a host without SMT keeps them too (pair falls back to off there)."""
    import argparse
    import importlib

    sys.path.insert(0, str(ROOT))
    bench = importlib.import_module("bench")
    seen = {}

    def fake_plan(n, per_rank, server_threads, avoid_busy=True, smt="off"):
        seen.update(n=n, per_rank=per_rank, smt=smt)
        return [{"server": [0], "loadgen": [128], "thread_targets": [[0]]}]

    monkeypatch.setattr(bench, "plan_replicas_with_loadgen", fake_plan)
    monkeypatch.setattr(bench, "slot_cores", lambda slots: 16)
    monkeypatch.setattr(bench, "physical_cores", lambda: list(range(128)))
    a = argparse.Namespace(slot_cores=0, cores=0, smt="pair", server_threads=0, gpu_slots=1)
    for budget, fits, sib, want in ((16, False, lambda c: c + 128, 8),   # the box's quota
                                    (256, True, lambda c: c + 128, 16),  # an 8-GPU node
                                    (16, False, lambda c: None, 16)):    # no SMT at all
        monkeypatch.setattr(bench, "cpu_budget", lambda b=budget: b)
        monkeypatch.setattr(bench, "smt_fits", lambda slots, per, f=fits: f)
        monkeypatch.setattr(bench, "sibling_of", sib)
        p = bench._plan(a, 1, avoid_busy=False)
        assert seen == {"n": 1, "per_rank": want, "smt": "pair"} and p["cores_per_slot"] == want, (budget, seen)


def test_latency_curve_runs_open_loop_with_the_server_busy_poll_it_names(tmp_path):
    """`bench/latency_curve.py` (the open-loop curve of `box_session.sh latency`): one short
    rate on the CPU, every body checked, and `server_busy_poll` "0" means the server really ran
    with `--busy-poll-us 0` (hola's own default is auto, so the flag must be passed)."""
    out = tmp_path / "curve.json"
    r = subprocess.run([sys.executable, str(ROOT / "bench" / "latency_curve.py"), "--rates", "20000",
                        "--duration", "1", "--out", str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(out.read_text())
    assert d["server_busy_poll"] == "0"
    (row,) = d["rows"]
    assert row["errors"] == 0 and row["achieved_rps"] > 0.9 * row["target_rps"], row
    assert d["server_args"] == ["--busy-poll-us", "0"]
    # the tail attribution of the point: the scheduler's run_delay of both sides and the load
    # generator's own lateness (bench/tail_report.py names causes from these)
    assert d["spin_us"] == 1000
    assert {"run_delay_ms", "run_delay_max_thread_ms", "invol"} <= set(row["server_threads"]["workers"])
    assert {"run_delay_ns", "run_delay_max_thread_ns", "send_late_max_ns", "behind_max_ns"} <= set(row["loadgen"])
    # service time from the kernel's receive timestamps: never longer than the open-loop latency
    # measured from the intended send time (which adds the generator's own delays)
    svc = row["service_us"]
    assert svc and 0 < svc["p50"] <= svc["p999"] <= svc["max"], svc
    assert svc["p50"] <= row["p50_us"] * 1.05 + 5, (svc, row["p50_us"])
    rep = subprocess.run([sys.executable, str(ROOT / "bench" / "tail_report.py"), str(out), "--threshold-us", "0"],
                         capture_output=True, text=True, timeout=60)
    assert rep.returncode == 0 and "with nothing recorded" in rep.stdout, rep.stdout + rep.stderr
