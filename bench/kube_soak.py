#!/usr/bin/env python3
"""BASELINE config 5 soak: back-to-back rolling updates of the 8-pod deployment under one
continuous load, at the manifests' real timings.

The manifests are applied by the local executor (hola_amd/kube), with `hola-dc.yaml`, the
translation ConfigMap and `translation-patch.yaml`, as `bench/kube_rollout.py` applies them.
One `hola_loadgen` then keeps 512 kept-alive connections on the Service for the whole run,
through connect-time DNAT (`--service dnat`, the default) or through the userspace proxy. Each
response body is checked against its own pod's greeting. Meanwhile `oc set env` rolls the
template again as soon as the previous rollout has completed and its old pods are gone.

Every rollout replaces all 8 pods, with the manifests' `--shutdown-delay-ms 5000`. The claim
under test: the load generator sees 0 errors and 0 non-2xx over all of them, no pod outlives
its grace period, and the executor's own file descriptors and threads stay flat. Progress
goes to stderr, one line per rollout. One JSON line goes to stdout and to OUT/result.json.

  python bench/kube_soak.py [--minutes 6] [--service dnat|proxy] [--out DIR] [--time-scale 1]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from hola_amd import native  # noqa: E402
from hola_amd.kube import Cluster  # noqa: E402

OS = ROOT / "deploy" / "openshift"


def log(msg: str) -> None:
    print(f"[kube_soak {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def own_fds_threads() -> tuple[int, int]:
    return len(os.listdir("/proc/self/fd")), threading.active_count()


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--minutes", type=float, default=6.0)
    ap.add_argument("--service", choices=["dnat", "proxy"], default="dnat")
    ap.add_argument("--out", default="gpurun_out/kube_soak")
    ap.add_argument("--replicas", type=int, default=8)
    ap.add_argument("--policy", choices=["none", "static"], default="static")
    ap.add_argument("--node-cpus", type=float, default=None)
    ap.add_argument("--time-scale", type=float, default=1.0)
    ap.add_argument("--connections", type=int, default=512)
    ap.add_argument("--loadgen-threads", type=int, default=4)
    ap.add_argument("--shutdown-delay-ms", type=int, default=None,
                    help="patch the pods' --shutdown-delay-ms before the soak (0 = the pre-round-3 "
                         "termination: drain at once; the rollouts then drop connections, and the run "
                         "hunts for drains that do not finish instead)")
    ap.add_argument("--busy-poll-us", default="auto",
                    help="the pods' --busy-poll-us with --shutdown-delay-ms (0 = sleeping event loops, the "
                         "server's default before round 3's session 2)")
    a = ap.parse_args()
    out = Path(a.out)
    if out.exists():
        shutil.rmtree(out)
    out.mkdir(parents=True)
    native.ensure_built("release")
    c = Cluster([OS / "hola-dc.yaml", OS / "translation-configmap.yaml"], patches=[OS / "translation-patch.yaml"],
                state_dir=out / "state", replicas=a.replicas, cpu_manager_policy=a.policy, node_cpus=a.node_cpus,
                time_scale=a.time_scale, service_port=0).start()
    res: dict = {"config": f"BASELINE config 5 soak: {a.replicas} pods of hola-dc.yaml, back-to-back `oc set env` "
                           f"rollouts under {a.connections} connections ({a.service})",
                 "service": a.service, "time_scale": a.time_scale, "cpu_manager_policy": a.policy}
    lg = None
    try:
        c.wait_ready(a.replicas, timeout=300)
        if a.shutdown_delay_ms is not None:
            rev = c.rollout_status()["revision"]
            c.patch({"spec": {"template": {"spec": {"containers": [{"name": "hola", "args": [
                "--shutdown-delay-ms", str(a.shutdown_delay_ms), "--busy-poll-us", a.busy_poll_us]}]}}}})
            c.wait(lambda: c.rollout_status()["revision"] > rev and c.rollout_status()["complete"], 600, "patch")
            c.wait(lambda: all(p["status"] != "Terminating" for p in c.get_pods()), 120, "old pods gone")
            res["shutdown_delay_ms"] = a.shutdown_delay_ms
        extra = ["--verify-body", "--endpoints-file", str(c.endpoints_file())] if a.service == "dnat" else []
        lg = subprocess.Popen([str(native.binary("hola_loadgen")), "-t", str(a.loadgen_threads), "-c",
                               str(a.connections), "-d", "86400s", "--json", *extra, c.service_url() + "/api/hola"],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        time.sleep(2.0)
        fds0, th0 = own_fds_threads()
        t0 = time.monotonic()
        rollouts = []
        k = 0
        while time.monotonic() - t0 < a.minutes * 60:
            k += 1
            rev0 = c.rollout_status()["revision"]
            ts = time.monotonic()
            c.set_env({"JAVA_OPTIONS": f"-Xmx512m -Dconf=/etc/config/translation.properties -Dsoak={k}"})
            c.wait(lambda: c.rollout_status()["revision"] > rev0 and c.rollout_status()["complete"], 600, "rollout")
            c.wait(lambda: all(p["status"] != "Terminating" for p in c.get_pods()), 120, "old pods gone")
            dt = time.monotonic() - ts
            fds, th = own_fds_threads()
            rollouts.append({"revision": c.rollout_status()["revision"], "s": round(dt, 2), "executor_fds": fds,
                             "executor_threads": th})
            log(f"rollout {k} to revision {rollouts[-1]['revision']} in {dt:.1f} s (executor fds {fds}, threads {th})")
            if lg.poll() is not None:
                raise RuntimeError(f"load generator exited early: {lg.stderr.read()[-2000:]}")
        time.sleep(2.0)
        lg.send_signal(2)
        stdout, stderr = lg.communicate(timeout=60)
        lines = [ln for ln in stdout.strip().splitlines() if ln.startswith("{")]
        r = json.loads(lines[-1]) if lines else {"error": stderr[-2000:]}
        lat = r.get("latency", {})
        killed = [e for e in c.events if e[2] == "Killed"]
        res.update({
            "minutes": round((time.monotonic() - t0) / 60, 2), "rollouts": len(rollouts),
            "pods_replaced": len(rollouts) * a.replicas, "rollout_s": [x["s"] for x in rollouts],
            "requests": lat.get("count"), "rps": r.get("rps"), "errors": lat.get("errors"),
            "non2xx": lat.get("non2xx"), "reconnects": lat.get("reconnects"), "pods_reached": r.get("targets"),
            "body_checked": lat.get("body_checked"), "body_mismatch": lat.get("body_mismatch"),
            "p50_ms": round(lat.get("p50_ns", 0) / 1e6, 3), "p99_ms": round(lat.get("p99_ns", 0) / 1e6, 3),
            "grace_kills": len(killed), "grace_kill_events": [e[3] for e in killed][:5],
            "executor_fds": [fds0] + [x["executor_fds"] for x in rollouts],
            "executor_threads": [th0] + [x["executor_threads"] for x in rollouts],
            "restarts_total": sum(p["restarts"] for p in c.get_pods()),
            # terminations that did not finish on their own: the drain's stall reports and the
            # exit watchdog's (status 3), each with the worker's activity record and stack
            **_stalls(c, out),
        })
        lg = None
    finally:
        if lg is not None and lg.poll() is None:
            lg.kill()
            lg.wait()
        c.close(grace_s=10)
        shutil.copy(c.state / "events.log", out / "events.log")
    print(json.dumps(res), flush=True)
    (out / "result.json").write_text(json.dumps(res, indent=1) + "\n")
    return 0


def _stalls(c: Cluster, out: Path) -> dict:
    stalled = []
    for log_path in sorted((c.state / "pods").glob("*/container.log")):
        text = log_path.read_text(errors="replace")
        if "did not answer" in text or "termination did not complete" in text:
            stalled.append(log_path.parent.name)
            dst = out / "stalls"
            dst.mkdir(exist_ok=True)
            shutil.copy(log_path, dst / f"{log_path.parent.name}.log")
    watchdog = [e for e in c.events if e[2] == "Deleted" and "exit 3 " in e[3]]
    return {"stalled_pods": stalled, "watchdog_exits": len(watchdog)}


if __name__ == "__main__":
    sys.exit(main())
