#!/usr/bin/env python3
"""Why one pod of the shipped shape costs more server CPU per request.

BENCH_r05: the replica as the manifests start it, in the pod's 2-CPU limit
(deploy/openshift/hola-dc.yaml `limits.cpu: 2`; bench.py `deployed_pod_*`), served 582 k req/s
at 3.405 us of server CPU per request; the same binary and arguments on 8 CPUs (`deployed_*`)
took 1.802 us. This runs the pod shape with one thing varied at a time, interleaved, rounds
in swapped order, each variant with subruns.attributed_closed_loop()'s accounting (busy CPU
per request, serving threads vs. the rest, voluntary / involuntary switches, the loop's
waits, the load generator's poll outcomes, TCP segments, host load incl. IRQ time):

  ref8        the deployed replica on 8 CPUs (the deployed_* sub-run)
  pod         the deployed replica on 2 CPUs (the deployed_pod_* sub-run: 8 load-generator
              threads, 64 connections, load-generator busy-poll 20 us)
  lgbp0/200   pod with the load generator's busy-poll window at 0 / 200 us
  w1 / w4     pod with 1 / 4 server workers inside the 2-CPU cpuset
  c16 / c256  pod with 16 / 256 connections
  lgt2        pod with 2 load-generator threads (as many as the pod has CPUs)
  lgsame      pod with the load-generator threads in the pod's own L3 only
  lgcross     pod with the load-generator threads in the other L3 only
  lgt2x       pod with 2 load-generator threads, in the other L3

and finally one `pod` run with --cpu-profile (cpuprof_pod.txt via bench/cpuprof_report.py).

    python bench/pod_shape.py --reps 2 --seconds 8 --out DIR
"""
from __future__ import annotations

import argparse
import json
import statistics
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from hola_amd.native import ensure_built  # noqa: E402
from hola_amd.parallel import subruns  # noqa: E402
from hola_amd.utils.cpu import parse_cpu_list  # noqa: E402

VARIANTS = {
    "ref8": {},
    "pod": {},
    "lgbp0": {"loadgen_busy_poll": 0},
    "lgbp200": {"loadgen_busy_poll": 200},
    "w1": {"threads": 1},
    "w4": {"threads": 4},
    "c16": {"connections": 16},
    "c256": {"connections": 256},
    "lgt2": {},
    "lgsame": {},
    "lgcross": {},
    "lgt2x": {},
}


def run_variant(a, v: str, sv, ld, job, seconds: float, cpu_profile: str | None = None) -> dict:
    pod_cpus = sorted(sv)[:subruns.manifest_pod_cpus()]
    server = sv if v == "ref8" else pod_cpus
    same = subruns.pod_loadgen_cpus(pod_cpus, ld)
    cross = [c for c in ld if c not in same] or ld
    load = {"lgt2": ld[:len(pod_cpus)], "lgsame": same, "lgcross": cross, "lgt2x": cross[:len(pod_cpus)]}.get(v, ld)
    return subruns.deployed(a, server, load, job, seconds=seconds, cpu_profile=cpu_profile, **VARIANTS[v])


def summary_row(v: str, rows: list[dict]) -> dict:
    def med(f):
        xs = [f(r) for r in rows]
        xs = [x for x in xs if x is not None]
        return round(statistics.median(xs), 3) if xs else None

    return {"variant": v, "n": len(rows),
            "rps": med(lambda r: r["rps"]),
            "p99_us": med(lambda r: r["p99_ns"] / 1e3),
            "server_cpu_us_per_req": med(lambda r: r["cpu_us_per_req"]),
            "server_busy_cpu_us_per_req": med(lambda r: r["server_busy_cpu_us_per_req"]),
            "server_cpus_us_per_req": med(lambda r: r["server_cpus_us_per_req"]),
            "loadgen_threads": med(lambda r: len(parse_cpu_list(r["loadgen_cpus"]))),
            "same_l3_or_core": med(lambda r: r["locality"].get("same_l3", 0) + r["locality"].get("same_core", 0)),
            "workers_cpu_share": med(lambda r: r["server_threads"].get("workers", {}).get("cpu_s", 0) /
                                     max(1e-9, sum(g["cpu_s"] for g in r["server_threads"].values()))),
            "server_vol_per_req": med(lambda r: r["server_threads"].get("workers", {}).get("vol_per_req")),
            "server_invol_per_req": med(lambda r: r["server_threads"].get("workers", {}).get("invol_per_req")),
            "server_sleeps_per_req": med(lambda r: r["server_loop"]["blocking_waits_per_req"]),
            "loadgen_sleeps_per_req": med(lambda r: r["loadgen"]["blocking_waits_per_req"]),
            "loadgen_busy_cpu_us_per_req": med(lambda r: r["loadgen"]["busy_cpu_us_per_req"]),
            "tcp_out_per_req": med(lambda r: r["tcp_per_req"].get("OutSegs")),
            "server_cpus_busy": med(lambda r: r["host_load_server"]["own"]),
            "server_cpus_irq": med(lambda r: r["host_load_server"]["irq_own"]),
            "loadgen_cpus_busy": med(lambda r: r["host_load_loadgen"]["own"])}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--seconds", type=float, default=8.0)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--no-profile", action="store_true")
    ap.add_argument("--out", required=True)
    o = ap.parse_args()
    sys.argv = [sys.argv[0]]
    a = bench.parse_args()
    if a.busy_poll_pause < 0:
        a.busy_poll_pause = 0
    ensure_built("release")
    p = bench._plan(a, 1)
    sv, ld = list(p["cores"][0]["server"]), list(p["cores"][0]["loadgen"])
    job = sv + ld
    out = Path(o.out)
    out.mkdir(parents=True, exist_ok=True)
    variants = o.variants.split(",")
    rows: list[dict] = []
    with open(out / "runs.jsonl", "w") as f:
        for rep in range(o.reps):
            for v in (variants if rep % 2 == 0 else variants[::-1]):
                try:
                    r = run_variant(a, v, sv, ld, job, o.seconds)
                except Exception as e:  # noqa: BLE001 - recorded, the study goes on
                    r = {"error": f"{type(e).__name__}: {e}"}
                row = {"rep": rep, "variant": v, **r}
                rows.append(row)
                f.write(json.dumps(row) + "\n")
                f.flush()
                if "error" in r:
                    print(f"{rep} {v} ERROR {r['error']}", flush=True)
                    continue
                print(f"{rep} {v:8s} rps={r['rps']:9.0f} cpu={r['cpu_us_per_req']:.3f} busy="
                      f"{r['server_busy_cpu_us_per_req']:.3f} us/req sleeps/req srv={r['server_loop']['blocking_waits_per_req']}"
                      f" lg={r['loadgen']['blocking_waits_per_req']} thr={r['server_threads']}", flush=True)
    summary = [summary_row(v, [r for r in rows if r["variant"] == v and "error" not in r]) for v in variants]
    prof = None
    if not o.no_profile:
        path = str((out / "server_cpu_pod.prof").resolve())
        r = run_variant(a, "pod", sv, ld, job, o.seconds, cpu_profile=path)
        prof = {"rps": r["rps"], "cpu_us_per_req": r["cpu_us_per_req"], "profile": path}
        rep = subprocess.run([sys.executable, str(ROOT / "bench/cpuprof_report.py"), path, "--top", "40", "--threads", ""],
                             capture_output=True, text=True, timeout=300)
        (out / "cpuprof_pod.txt").write_text(rep.stdout + rep.stderr)
    (out / "summary.json").write_text(json.dumps({"cpus": {"server8": sv, "loadgen": ld}, "summary": summary,
                                                  "profiled": prof}, indent=1))
    for s in summary:
        print(json.dumps(s), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
