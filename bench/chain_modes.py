#!/usr/bin/env python3
"""The chaining sub-run of bench.py (`chain_*` keys), repeated back to back, one JSON line per
run: what separates its fast runs from its slow ones.

Each run is exactly bench.py's chain sub-run on the CPUs bench.py gives rank 0 (load
generator -> hola A -> hola B, 64 connections), with the attribution it reports: host load,
accept locality of both hops, both replicas' busy-poll counters. `--variants` interleaves
settings of the load generator's busy-poll window and of the replicas' server flags, so a
variable that splits the runs shows up in the table.

    python bench/chain_modes.py --reps 10 --seconds 10 [--variants lg0,lg20] --out DIR
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402  (bench.py's planner and defaults)
from hola_amd.native import ensure_built  # noqa: E402
from hola_amd.parallel import subruns  # noqa: E402


def variant_args(v: str) -> dict:
    """lgN = load-generator busy-poll window N us; lgN/prev = the same with build/prev/hola as
    A and B (a server built from an earlier commit)."""
    lg, _, exe = v.partition("/")
    if not lg.startswith("lg"):
        raise ValueError(f"unknown variant {v}")
    out: dict = {"loadgen_busy_poll": int(lg[2:])}
    if exe:
        out["exe"] = ROOT / "build" / exe / "hola"
    return out


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--variants", default="lg0", help="comma-separated: lgN (load generator busy-poll N us), "
                                                        "lgN/prev (with build/prev/hola as A and B)")
    ap.add_argument("--shipped", action="store_true", help="the shipped configuration (pool 10, BASIC logging)")
    ap.add_argument("--out", required=True)
    o = ap.parse_args()
    sys.argv = [sys.argv[0]]
    a = bench.parse_args()
    ensure_built("release")
    p = bench._plan(a, 1)
    cpus = list(p["cores"][0]["server"]) + list(p["cores"][0]["loadgen"])
    job = cpus
    out_dir = Path(o.out)
    out_dir.mkdir(parents=True, exist_ok=True)
    rows = []
    variants = o.variants.split(",")
    with open(out_dir / "runs.jsonl", "w") as f:
        for rep in range(o.reps):
            order = variants if rep % 2 == 0 else variants[::-1]  # swap the order each round
            for v in order:
                t0 = time.time()
                r = subruns.chain(a, cpus, job, shipped=o.shipped, seconds=o.seconds, **variant_args(v))
                row = {"rep": rep, "variant": v, "wall_s": round(time.time() - t0, 2),
                       **{k: r[k] for k in r if k not in ("hystrix",)}}
                rows.append(row)
                f.write(json.dumps(row) + "\n")
                f.flush()
                sp = r.get("spins", {})
                print(f"{rep} {v} rps={r.get('rps', 0):.0f} A={r.get('a_cpu_us_per_req', 0):.2f}us "
                      f"p99={r.get('p99_ns', 0) / 1e3:.1f}us A.spins={sp.get('a')} B.spins={sp.get('b')} "
                      f"loc={r.get('locality')} load={r.get('host_load')} thr={r.get('cgroup_throttle')}", flush=True)
    summary = {}
    for v in variants:
        x = [r["rps"] for r in rows if r["variant"] == v and "rps" in r]
        if x:
            summary[v] = {"n": len(x), "mean": statistics.mean(x), "min": min(x), "max": max(x),
                          "spread_pct": 100 * (max(x) - min(x)) / statistics.mean(x)}
    # each variant against the first, paired by round (the order is swapped every round), with
    # a 95 % t-interval: req/s and A's CPU per chained request
    from ab_report import ci
    base = variants[0]
    for v in variants[1:]:
        pairs = [(b, c) for b in rows for c in rows
                 if b["variant"] == base and c["variant"] == v and b["rep"] == c["rep"] and "rps" in b and "rps" in c]
        if len(pairs) < 2:
            continue
        for key in ("rps", "a_cpu_us_per_req"):
            m, lo, hi = ci([100.0 * (c[key] - b[key]) / b[key] for b, c in pairs])
            summary[v][f"{key}_vs_{base}_pct"] = {"mean": round(m, 2), "ci95": [round(lo, 2), round(hi, 2)],
                                                  "pairs": len(pairs)}
    (out_dir / "summary.json").write_text(json.dumps(summary, indent=1))
    print(json.dumps(summary))
    return 0


if __name__ == "__main__":
    sys.exit(main())
