#!/usr/bin/env python3
"""Parameter sweep for the 1-replica headline config on the current host: server/loadgen
core split, busy-polling and tracing. Writes one JSON row per point (bench.py output plus
the knobs) to --out; used to pick bench.py's defaults from measurements, not guesses."""
import argparse
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent

ap = argparse.ArgumentParser()
ap.add_argument("--out", required=True)
ap.add_argument("--points", default="8:0:on,8:0:off,6:0:on,10:0:on,8:20:on,8:50:on,6:20:on,10:20:on",
                help="comma list of server_threads:busy_poll_us:tracing")
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--timeout", type=int, default=120)
a = ap.parse_args()
rows = []
for pt in a.points.split(","):
    st, bp, tr = pt.split(":")
    cmd = [sys.executable, str(ROOT / "bench.py"), "--steps", str(a.steps), "--warmup", "3",
           "--server-threads", st, "--busy-poll-us", bp]
    if tr == "off":
        cmd.append("--no-tracing")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=a.timeout)
    if r.returncode != 0:
        rows.append({"point": pt, "error": r.stderr[-2000:]})
        print(pt, "FAILED", flush=True)
        break
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    row = {"point": pt, "server_threads": int(st), "busy_poll_us": int(bp), "tracing": tr,
           "value": d["value"], "p50_ms": d["p50_ms"], "p99_ms": d["p99_ms"],
           "server_cpu_us_per_req": d["server_cpu_us_per_req"], "loadgen_cpu_us_per_req": d["loadgen_cpu_us_per_req"]}
    rows.append(row)
    print(json.dumps(row), flush=True)
    Path(a.out).write_text(json.dumps(rows, indent=1))
