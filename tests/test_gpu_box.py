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
                        "--reqs-per-conn", "200"], capture_output=True, text=True, timeout=600,
                       env={**os.environ, "HOLA_BENCH_PORT": "18700"})
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


@pytest.mark.gpu
def test_bench_two_ranks_on_host():
    """The multi-replica path (torchrun, gloo barriers, client-side round-robin across
    replicas, cross-rank L3-aware load-generator placement) on the real host."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29517", str(ROOT / "bench.py"),
                        "--gpus", "2", "--steps", "3", "--warmup", "1", "--reqs-per-conn", "500"],
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


@pytest.mark.gpu
def test_tracing_as_deployed_on_host():
    """`bench.py --zipkin-sink`: a native collector attached, as ZIPKIN_SERVER_URL is in the
    reference image. Spans beyond the Brave-parity budget are dropped and counted, the rest
    reach the collector, and the request path does not slow down."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "4", "--warmup", "1",
                        "--reqs-per-conn", "20000", "--c1-seconds", "0", "--zipkin-sink"],
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
                        "--reqs-per-conn", "16000"], capture_output=True, text=True, timeout=300,
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
