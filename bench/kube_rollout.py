#!/usr/bin/env python3
"""BASELINE config 5 on the real node: the manifests applied to the local cluster executor
(hola_amd/kube) at their real timings, with the evidence in one JSON line.

  1. apply hola-dc.yaml + the translation ConfigMap + translation-patch.yaml, 8 replicas:
     time until 8 pods pass their readiness probe (initialDelaySeconds 5, periodSeconds 10)
     and are endpoints of the Service, and the 8 pod-name greetings seen through it;
  2. `oc set env dc/hola ...` under 512 kept-alive connections through the Service, with the
     manifests' --shutdown-delay-ms 5000: rollout time, load-generator errors / non-2xx;
  3. the same rollout with the delay patched to 0 (the pre-round-3 shutdown);
     2 and 3 run once per Service data path (--service): "proxy" through hola_rrproxy
     (kube-proxy's userspace mode: one proxy hop per request) and "dnat", where each new
     connection is DNATed at connect time to a published endpoint (the iptables/IPVS modes:
     no hop, an established connection keeps its pod);
  4. a SIGKILLed pod: when it leaves the Service endpoints and when it rejoins;
  5. a ConfigMap edit: when all 8 pods serve the new greeting.

  python bench/kube_rollout.py [--out DIR] [--policy static] [--time-scale 1]
"""
from __future__ import annotations

import argparse
import json
import shutil
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from hola_amd import native  # noqa: E402
from hola_amd.kube import Cluster  # noqa: E402
from hola_amd.utils.net import http_get  # noqa: E402

OS = ROOT / "deploy" / "openshift"


def log(msg: str) -> None:
    print(f"[kube_rollout {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def greetings(c: Cluster, n: int = 64) -> list[str]:
    """n GETs through the Service; a failed one is recorded as an "ERROR ..." entry."""
    host, port = c.service_ports["hola"]
    out = []
    for _ in range(n):
        try:
            out.append(http_get(host, port, "/api/hola", timeout=5)[2].decode())
        except OSError as e:
            out.append(f"ERROR {type(e).__name__}: {e}")
    return out


def rollout_under_load(c: Cluster, env: dict, conns: int, threads: int, settle_s: float,
                       service: str = "proxy") -> dict:
    """Starts the load, rolls the template, waits for the rollout and for the old pods to
    exit, lets the load run `settle_s` more, and returns the load generator's counters."""
    extra = ["--verify-body", "--endpoints-file", str(c.endpoints_file())] if service == "dnat" else []
    lg = subprocess.Popen([str(native.binary("hola_loadgen")), "-t", str(threads), "-c", str(conns), "-d", "600s",
                           "--json", *extra, c.service_url() + "/api/hola"], stdout=subprocess.PIPE,
                          stderr=subprocess.PIPE, text=True)
    time.sleep(3.0)
    rev0 = c.rollout_status()["revision"]
    t0 = time.monotonic()
    c.set_env(env)
    c.wait(lambda: c.rollout_status()["revision"] > rev0 and c.rollout_status()["complete"], 600, "rollout")
    t_roll = time.monotonic() - t0
    c.wait(lambda: all(p["status"] != "Terminating" for p in c.get_pods()), 120, "old pods gone")
    t_gone = time.monotonic() - t0
    time.sleep(settle_s)
    lg.send_signal(2)  # SIGINT: the load generator prints its summary and exits
    out, err = lg.communicate(timeout=60)
    lines = [ln for ln in out.strip().splitlines() if ln.startswith("{")]
    r = json.loads(lines[-1]) if lines else {"error": err[-2000:]}
    lat = r.get("latency", {})
    return {"service": service, "rollout_s": round(t_roll, 2), "old_pods_gone_s": round(t_gone, 2),
            "revision": c.rollout_status()["revision"],
            "requests": lat.get("count"), "rps": r.get("rps"), "errors": lat.get("errors"),
            "non2xx": lat.get("non2xx"), "reconnects": lat.get("reconnects"), "pods_reached": r.get("targets"),
            "body_checked": lat.get("body_checked"), "body_mismatch": lat.get("body_mismatch"),
            "p50_ms": round(lat.get("p50_ns", 0) / 1e6, 3), "p99_ms": round(lat.get("p99_ns", 0) / 1e6, 3)}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--out", default="gpurun_out/kube_rollout")
    ap.add_argument("--replicas", type=int, default=8)
    ap.add_argument("--policy", choices=["none", "static"], default="static")
    ap.add_argument("--reserved-cpus", type=int, default=0)
    ap.add_argument("--node-cpus", type=float, default=None, help="node capacity (default: this host's CPUs)")
    ap.add_argument("--time-scale", type=float, default=1.0)
    ap.add_argument("--endpoint-sync-s", type=float, default=1.0)
    ap.add_argument("--configmap-sync-s", type=float, default=10.0)
    ap.add_argument("--connections", type=int, default=512)
    ap.add_argument("--loadgen-threads", type=int, default=4)
    ap.add_argument("--settle-s", type=float, default=2.0)
    ap.add_argument("--service", choices=["proxy", "dnat", "both"], default="both",
                    help="Service data path under the rollouts (default: both, one after the other)")
    a = ap.parse_args()
    out = Path(a.out)
    if out.exists():
        shutil.rmtree(out)
    out.mkdir(parents=True)
    native.ensure_built("release")
    res: dict = {"config": "BASELINE config 5: deploy/openshift/hola-dc.yaml + translation ConfigMap + patch, "
                           f"{a.replicas} pods, readiness-gated Service (local executor hola_amd/kube)",
                 "time_scale": a.time_scale, "cpu_manager_policy": a.policy, "endpoint_sync_s": a.endpoint_sync_s,
                 "configmap_sync_s": a.configmap_sync_s, "connections": a.connections}
    t0 = time.monotonic()
    c = Cluster([OS / "hola-dc.yaml", OS / "translation-configmap.yaml"], patches=[OS / "translation-patch.yaml"],
                state_dir=out / "state", replicas=a.replicas, cpu_manager_policy=a.policy, node_cpus=a.node_cpus,
                reserved_cpus=a.reserved_cpus, time_scale=a.time_scale, endpoint_sync_s=a.endpoint_sync_s,
                configmap_sync_s=a.configmap_sync_s, service_port=0).start()
    try:
        c.wait_ready(a.replicas, timeout=300)
        res["ready_s"] = round(time.monotonic() - t0, 2)
        pods = c.get_pods()
        res["pods"] = [{k: p[k] for k in ("name", "ip", "cpus")} for p in pods]
        seen = sorted(set(greetings(c, 16 * a.replicas)))
        res["greetings_seen"] = len(seen)
        res["greetings_match_pods"] = seen == sorted(f"Hola de {p['name']} mediante el archivo de configuraciones\n"
                                                     for p in pods)
        log(f"{a.replicas} pods ready after {res['ready_s']} s; {len(seen)} distinct greetings")

        services = ["proxy", "dnat"] if a.service == "both" else [a.service]
        k = 0
        for svc in services:
            k += 1
            key = "rollout_with_delay" + ("" if svc == "proxy" else "_dnat")
            res[key] = rollout_under_load(c, {"JAVA_OPTIONS": "-Xmx512m -Dconf=/etc/config/translation.properties "
                                                              f"-Drollout={k}"},
                                          a.connections, a.loadgen_threads, a.settle_s, svc)
            log(f"rollout with --shutdown-delay-ms 5000 ({svc}): {res[key]}")
        # the pre-round-3 behaviour: no delay (a rollout of its own, without load)
        rev = c.rollout_status()["revision"]
        c.patch({"spec": {"template": {"spec": {"containers": [{"name": "hola", "args": ["--shutdown-delay-ms", "0"]}]}}}})
        c.wait(lambda: c.rollout_status()["revision"] > rev and c.rollout_status()["complete"], 600, "patch rollout")
        c.wait(lambda: all(p["status"] != "Terminating" for p in c.get_pods()), 120, "old pods gone")
        for svc in services:
            k += 1
            key = "rollout_without_delay" + ("" if svc == "proxy" else "_dnat")
            res[key] = rollout_under_load(c, {"JAVA_OPTIONS": "-Xmx512m -Dconf=/etc/config/translation.properties "
                                                              f"-Drollout={k}"},
                                          a.connections, a.loadgen_threads, a.settle_s, svc)
            log(f"rollout with --shutdown-delay-ms 0 ({svc}): {res[key]}")

        victim = c.get_pods()[0]
        ip = victim["ip"]
        t_kill = time.monotonic()
        c.kill_container(victim["name"])
        c.wait(lambda: all(not e.startswith(ip + ":") for e in c.endpoints()), 60, "endpoint removal")
        t_left = time.monotonic() - t_kill
        c.wait(lambda: any(e.startswith(ip + ":") for e in c.endpoints()), 300, "rejoin")
        res["sigkill"] = {"pod": victim["name"], "left_endpoints_s": round(t_left, 2),
                          "rejoined_s": round(time.monotonic() - t_kill, 2),
                          "restarts": next(p["restarts"] for p in c.get_pods() if p["name"] == victim["name"])}
        log(f"SIGKILL: {res['sigkill']}")

        t_cm = time.monotonic()
        c.apply_configmap("translation", {"translation.properties": "hello=Aloha de %s desde el ConfigMap\n"})
        want = sorted(f"Aloha de {p['name']} desde el ConfigMap" for p in c.get_pods())
        c.wait(lambda: sorted(set(greetings(c, 16 * a.replicas))) == want, 600, "ConfigMap edit on every pod")
        res["configmap_edit_all_pods_s"] = round(time.monotonic() - t_cm, 2)
        res["restarts_total"] = sum(p["restarts"] for p in c.get_pods())
        res["grace_kills"] = sum(1 for e in c.events if e[2] == "Killed")  # pods SIGKILLed at the grace period
        log(f"ConfigMap edit on all pods after {res['configmap_edit_all_pods_s']} s")
    finally:
        c.close(grace_s=10)
        shutil.copy(c.state / "events.log", out / "events.log")
    res["wall_s"] = round(time.monotonic() - t0, 1)
    print(json.dumps(res), flush=True)
    (out / "result.json").write_text(json.dumps(res, indent=1) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
