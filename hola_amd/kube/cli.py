"""`python -m hola_amd apply` and `python -m hola_amd oc`: the reference's deploy flow
(`/root/reference/Readme.md:18-24`: `mvn fabric8:json fabric8:apply`, then `oc scale`,
`oc env`) against the local executor.

    python -m hola_amd apply -f deploy/openshift/hola-dc.yaml \\
        -f deploy/openshift/translation-configmap.yaml \\
        --patch deploy/openshift/translation-patch.yaml --replicas 8      # runs in the foreground
    python -m hola_amd oc get pods
    python -m hola_amd oc scale dc/hola --replicas=8
    python -m hola_amd oc set env dc/hola JAVA_OPTIONS="-Xmx512m -Dconf=/etc/config/translation.properties"
    python -m hola_amd oc rollout status dc/hola
    python -m hola_amd oc apply -f translation-configmap.yaml            # ConfigMap edit
    python -m hola_amd oc delete pod hola-1-abcde
    python -m hola_amd oc logs hola-1-abcde; python -m hola_amd oc describe pod hola-1-abcde
    python -m hola_amd oc top pods

`apply` serves a control socket in its state directory (`--state-dir`, default
`$HOLA_CLUSTER_DIR` or /tmp/hola-cluster); `oc` talks to it.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import sys
import threading
import time
from pathlib import Path

import yaml

DEFAULT_STATE = os.environ.get("HOLA_CLUSTER_DIR", "/tmp/hola-cluster")


def _state_args(ap: argparse.ArgumentParser) -> None:
    ap.add_argument("--state-dir", default=DEFAULT_STATE, help="executor state (pods, logs, control socket)")


def apply_main(argv: list[str]) -> int:
    from hola_amd.kube import Cluster

    ap = argparse.ArgumentParser(prog="python -m hola_amd apply", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-f", "--filename", action="append", required=True, help="manifest file (repeatable)")
    ap.add_argument("--patch", action="append", default=[], help="strategic-merge patch of the workload")
    ap.add_argument("--replicas", type=int, default=None, help="scale the workload at creation (oc scale)")
    _state_args(ap)
    ap.add_argument("--node-cpus", type=float, default=None, help="node CPU capacity (default: this host's)")
    ap.add_argument("--reserved-cpus", type=int, default=1, help="CPUs the kubelet keeps for itself")
    ap.add_argument("--cpu-manager-policy", choices=["none", "static"], default="none")
    ap.add_argument("--time-scale", type=float, default=1.0,
                    help="multiplies probe delays/periods, restart back-off and sync delays (tests)")
    ap.add_argument("--endpoint-sync-s", type=float, default=1.0, help="kube-proxy's delay applying endpoints")
    ap.add_argument("--configmap-sync-s", type=float, default=60.0, help="kubelet's ConfigMap volume sync period")
    ap.add_argument("--service-host", default="127.0.0.1", help="address of the LoadBalancer Service")
    ap.add_argument("--service-port", type=int, default=None, help="default: the Service's port (8080)")
    ap.add_argument("--proxy-threads", type=int, default=0,
                    help="threads of the userspace Service proxy (0 = a quarter of the node's CPUs, 2..16); "
                         "for load tests read the endpoints file and DNAT at connect time instead "
                         "(hola_loadgen --endpoints-file: no proxy hop, docs/OPERATIONS.md)")
    ap.add_argument("--no-zipkin", action="store_true", help="no stand-in collector for zipkin-query:9411")
    a = ap.parse_args(argv)
    state = Path(a.state_dir)
    state.mkdir(parents=True, exist_ok=True)
    sock_path = state / "control.sock"
    if sock_path.exists():
        try:
            _request(state, {"op": "ping"})
            print(f"apply: a cluster already runs in {state}", file=sys.stderr)
            return 1
        except OSError:
            sock_path.unlink()
    c = Cluster(a.filename, patches=a.patch, state_dir=state, replicas=a.replicas, node_cpus=a.node_cpus,
                reserved_cpus=a.reserved_cpus, cpu_manager_policy=a.cpu_manager_policy, time_scale=a.time_scale,
                endpoint_sync_s=a.endpoint_sync_s, configmap_sync_s=a.configmap_sync_s,
                service_host=a.service_host, service_port=a.service_port, proxy_threads=a.proxy_threads,
                zipkin=not a.no_zipkin)
    c.start()
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
    srv.bind(str(sock_path))
    srv.listen(16)
    stop = threading.Event()

    def on_signal(*_):
        stop.set()

    for s in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        signal.signal(s, on_signal)
    threading.Thread(target=_serve, args=(srv, c, stop), daemon=True).start()
    print(f"apply: {c.kind.lower()}/{c.name} x{c.desired}, service {c.service_url()} (state {state}; "
          f"`python -m hola_amd oc --state-dir {state} get pods`; connect-time DNAT to the endpoints: "
          f"`hola_loadgen --endpoints-file {c.endpoints_file()} {c.service_url()}/api/hola`)", flush=True)
    try:
        while not stop.is_set():
            stop.wait(0.5)
    finally:
        srv.close()
        sock_path.unlink(missing_ok=True)
        c.close()
    return 0


def _serve(srv: socket.socket, c, stop: threading.Event) -> None:
    while not stop.is_set():
        try:
            conn, _ = srv.accept()
        except OSError:
            return
        threading.Thread(target=_handle, args=(conn, c, stop), daemon=True).start()


def _handle(conn: socket.socket, c, stop: threading.Event) -> None:
    with conn:
        f = conn.makefile("rwb")
        line = f.readline()
        try:
            req = json.loads(line)
            out = {"ok": True, "result": _dispatch(c, req, stop)}
        except Exception as e:  # noqa: BLE001 - reported to the client
            out = {"ok": False, "error": f"{type(e).__name__}: {e}"}
        f.write((json.dumps(out) + "\n").encode())
        f.flush()


def _dispatch(c, req: dict, stop: threading.Event):
    op = req["op"]
    if op == "ping":
        return "pong"
    if op == "get-pods":
        return c.get_pods()
    if op == "get-endpoints":
        return {"published": c.endpoints(req.get("service")), "desired": c.endpoints(req.get("service"), False)}
    if op == "get-events":
        return [list(e) for e in list(c.events)[-int(req.get("n", 200)):]]
    if op == "scale":
        return c.scale(int(req["replicas"]))
    if op == "set-env":
        return c.set_env(req["env"], req.get("container"))
    if op == "patch":
        return c.patch(req["patch"])
    if op == "apply":
        for o in req["objects"]:
            if o.get("kind") == "ConfigMap":
                c.apply_configmap(o["metadata"]["name"], o.get("data") or {})
            elif o.get("kind") in ("DeploymentConfig", "Deployment"):
                c.patch({"spec": {"replicas": o["spec"].get("replicas", c.desired), "template": o["spec"]["template"]}})
        return None
    if op == "delete-pod":
        return c.delete_pod(req["name"])
    if op == "kill":
        return c.kill_container(req["name"], getattr(signal, "SIG" + req.get("signal", "KILL").upper()))
    if op == "rollout-status":
        return c.rollout_status()
    if op == "logs":
        path = c.state / "pods" / req["name"] / "container.log"
        if not path.exists():
            raise KeyError(f"no pod {req['name']!r}")
        lines = path.read_text(errors="replace").splitlines()
        return lines[-int(req["tail"]):] if req.get("tail") else lines
    if op == "describe":
        pod = next((p for p in c.get_pods() if p["name"] == req["name"]), None)
        if pod is None:
            raise KeyError(f"no pod {req['name']!r}")
        return {"pod": pod, "events": [list(e) for e in c.events if e[1] == req["name"]]}
    if op == "top":
        return c.top(float(req.get("sample_s", 0.5)))
    if op == "service-url":
        return c.service_url(req.get("service"))
    if op == "shutdown":
        stop.set()
        return None
    raise ValueError(f"unknown op {op!r}")


def _request(state: Path, req: dict, timeout: float = 30.0):
    with socket.socket(socket.AF_UNIX, socket.SOCK_STREAM) as s:
        s.settimeout(timeout)
        s.connect(str(state / "control.sock"))
        s.sendall((json.dumps(req) + "\n").encode())
        data = b""
        while not data.endswith(b"\n"):
            chunk = s.recv(65536)
            if not chunk:
                break
            data += chunk
    out = json.loads(data)
    if not out["ok"]:
        raise RuntimeError(out["error"])
    return out["result"]


def _env_pairs(items: list[str]) -> dict[str, str | None]:
    env: dict[str, str | None] = {}
    for it in items:
        if it.endswith("-") and "=" not in it:
            env[it[:-1]] = None  # `oc set env dc/hola KEY-` removes KEY
        else:
            k, _, v = it.partition("=")
            env[k] = v
    return env


def oc_main(argv: list[str]) -> int:
    ap = argparse.ArgumentParser(prog="python -m hola_amd oc")
    _state_args(ap)
    sub = ap.add_subparsers(dest="verb", required=True)
    g = sub.add_parser("get")
    g.add_argument("what", choices=["pods", "pod", "po", "endpoints", "ep", "events"])
    g.add_argument("name", nargs="?")
    g.add_argument("-o", "--output", choices=["wide", "json"], default="wide")
    s = sub.add_parser("scale")
    s.add_argument("target")
    s.add_argument("--replicas", type=int, required=True)
    e = sub.add_parser("set")
    e.add_argument("what", choices=["env"])
    e.add_argument("target")
    e.add_argument("pairs", nargs="+")
    e.add_argument("-c", "--containers", default=None)
    e2 = sub.add_parser("env")  # the demo era's `oc env dc/hola K=V`
    e2.add_argument("target")
    e2.add_argument("pairs", nargs="+")
    p = sub.add_parser("patch")
    p.add_argument("target")
    p.add_argument("-p", "--patch", default=None)
    p.add_argument("--patch-file", default=None)
    ap_ = sub.add_parser("apply")
    ap_.add_argument("-f", "--filename", action="append", required=True)
    d = sub.add_parser("delete")
    d.add_argument("what", choices=["pod", "pods", "po"])
    d.add_argument("name")
    k = sub.add_parser("kill", help="crash a pod's container (sends the signal to its process)")
    k.add_argument("name")
    k.add_argument("--signal", default="KILL")
    r = sub.add_parser("rollout")
    r.add_argument("what", choices=["status"])
    r.add_argument("target")
    r.add_argument("--timeout", type=float, default=600.0)
    lg = sub.add_parser("logs", help="a pod's container log")
    lg.add_argument("name")
    lg.add_argument("--tail", type=int, default=0)
    de = sub.add_parser("describe", help="a pod's state and its events")
    de.add_argument("what", choices=["pod", "po"])
    de.add_argument("name")
    t = sub.add_parser("top", help="CPU and memory of each pod (kubectl top pod)")
    t.add_argument("what", choices=["pods", "pod", "po"])
    sub.add_parser("url")
    sub.add_parser("stop")
    a = ap.parse_args(argv)
    state = Path(a.state_dir)
    try:
        if a.verb == "get":
            if a.what in ("pods", "pod", "po"):
                pods = _request(state, {"op": "get-pods"})
                if a.output == "json":
                    print(json.dumps(pods, indent=1))
                else:
                    print(f"{'NAME':<22} {'READY':<6} {'STATUS':<18} {'RESTARTS':<9} {'IP':<16} CPUS")
                    for x in pods:
                        print(f"{x['name']:<22} {('1/1' if x['ready'] else '0/1'):<6} {x['status']:<18} "
                              f"{x['restarts']:<9} {x['ip']:<16} {x['cpus'] or 'shared'}")
            elif a.what in ("endpoints", "ep"):
                ep = _request(state, {"op": "get-endpoints", "service": a.name})
                print(json.dumps(ep) if a.output == "json" else ",".join(ep["published"]) or "<none>")
            else:
                for t, obj, reason, msg in _request(state, {"op": "get-events"}):
                    print(f"{t:9.3f} {obj:<28} {reason:<14} {msg}")
        elif a.verb == "scale":
            _request(state, {"op": "scale", "replicas": a.replicas})
            print(f"{a.target} scaled")
        elif a.verb in ("set", "env"):
            _request(state, {"op": "set-env", "env": _env_pairs(a.pairs), "container": getattr(a, "containers", None)})
            print(f"{a.target} updated")
        elif a.verb == "patch":
            text = Path(a.patch_file).read_text() if a.patch_file else a.patch
            _request(state, {"op": "patch", "patch": yaml.safe_load(text)})
            print(f"{a.target} patched")
        elif a.verb == "apply":
            from hola_amd.kube.manifests import load_objects
            _request(state, {"op": "apply", "objects": load_objects(a.filename)})
            print("applied")
        elif a.verb == "delete":
            _request(state, {"op": "delete-pod", "name": a.name})
            print(f'pod "{a.name}" deleted')
        elif a.verb == "kill":
            _request(state, {"op": "kill", "name": a.name, "signal": a.signal})
        elif a.verb == "rollout":
            deadline = time.monotonic() + a.timeout
            while True:
                st = _request(state, {"op": "rollout-status"})
                if st["complete"]:
                    print(f"replication controller \"{st['rc']}\" successfully rolled out")
                    break
                if time.monotonic() > deadline:
                    print(f"timed out: {st}", file=sys.stderr)
                    return 1
                time.sleep(0.5)
        elif a.verb == "logs":
            print("\n".join(_request(state, {"op": "logs", "name": a.name, "tail": a.tail})))
        elif a.verb == "describe":
            d = _request(state, {"op": "describe", "name": a.name})
            for k, v in d["pod"].items():
                print(f"{k + ':':<16}{v}")
            print("Events:")
            for t, _obj, reason, msg in d["events"]:
                print(f"  {t:9.3f}  {reason:<16} {msg}")
        elif a.verb == "top":
            print(f"{'NAME':<24}{'CPU(cores)':>12}{'MEMORY(bytes)':>15}  THROTTLED(periods)")
            for p in _request(state, {"op": "top"}):
                th = p["cpu_throttle"]
                thr = f"{th['nr_throttled']}/{th['nr_periods']}" if th else "-"
                print(f"{p['name']:<24}{round(p['cpu_cores'] * 1000):>11}m{p['memory_bytes'] >> 20:>13}Mi  {thr}")
        elif a.verb == "url":
            print(_request(state, {"op": "service-url"}))
        elif a.verb == "stop":
            _request(state, {"op": "shutdown"})
    except (OSError, RuntimeError) as e:
        print(f"oc: {e}", file=sys.stderr)
        return 1
    return 0
