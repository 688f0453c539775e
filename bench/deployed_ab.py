#!/usr/bin/env python3
"""Where the as-deployed replica's req/s goes against the headline replica:
interleaved rounds, order swapped each round, on the CPUs bench.py gives rank 0, each side a
~10 s closed-loop run with its own host load.

  headline  the bench.py replica: --threads/--cpu-list pinned, tracing on, no collector
            (ZIPKIN_SERVER_URL unset: spans dropped at the source)
  deployed  image ENTRYPOINT + manifests' args and env: ZIPKIN_SERVER_URL=http://zipkin-query:9411,
            which does not resolve on a bare host (spans recorded, then dropped when the post fails)
  unset     the deployed replica with ZIPKIN_SERVER_URL removed
  sink      the deployed replica posting to a native discard collector (--zipkin-sink)

    python bench/deployed_ab.py --reps 4 --seconds 10 --out DIR
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402
from hola_amd.native import ensure_built  # noqa: E402
from hola_amd.parallel import subruns  # noqa: E402
from hola_amd.parallel.loadgen import ControlledLoadgen  # noqa: E402
from hola_amd.server import HolaProcess  # noqa: E402
from hola_amd.utils.cpu import format_cpu_list  # noqa: E402


def headline(a, sv, ld, job, seconds):
    args = ["--busy-poll-us", a.server_busy_poll]
    with HolaProcess(args=args, env={"HOSTNAME": "replica-0"}, threads=len(sv), cpu_list=format_cpu_list(sv),
                     log_level="warn") as s:
        lg = ControlledLoadgen([("127.0.0.1", s.port)], a.connections, len(ld), cpu_list=",".join(map(str, ld)),
                               busy_poll_us=a.busy_poll_us, expect_bodies=["Hola de replica-0"])
        try:
            return subruns.timed_closed_loop(lg, a.connections, seconds, s.proc.pid, sv + ld, job)
        finally:
            lg.close()


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--variants", default="headline,deployed,unset,sink")
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
    rows = []
    with open(out / "runs.jsonl", "w") as f:
        for rep in range(o.reps):
            for v in (variants if rep % 2 == 0 else variants[::-1]):
                if v == "headline":
                    r = headline(a, sv, ld, job, o.seconds)
                else:
                    r = subruns.deployed(a, sv, ld, job, zipkin=v, seconds=o.seconds)
                row = {"rep": rep, "variant": v, **r}
                rows.append(row)
                f.write(json.dumps(row) + "\n")
                f.flush()
                print(f"{rep} {v} rps={r['rps']:.0f} p99={r['p99_ns'] / 1e3:.1f}us cpu={r['cpu_us_per_req']:.3f}us "
                      f"load={r['host_load']}", flush=True)
    summary = {}
    for v in variants:
        x = [r["rps"] for r in rows if r["variant"] == v]
        c = [r["cpu_us_per_req"] for r in rows if r["variant"] == v]
        summary[v] = {"n": len(x), "rps_mean": statistics.mean(x), "rps_min": min(x), "rps_max": max(x),
                      "cpu_us_per_req_mean": statistics.mean(c)}
    base = summary.get("headline", {}).get("rps_mean")
    if base:
        for v in summary:
            summary[v]["vs_headline_pct"] = round(100 * (summary[v]["rps_mean"] / base - 1), 2)
    (out / "summary.json").write_text(json.dumps(summary, indent=1))
    print(json.dumps(summary))
    return 0


if __name__ == "__main__":
    sys.exit(main())
