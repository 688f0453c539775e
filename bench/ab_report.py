#!/usr/bin/env python3
"""Gated A/B of interleaved bench.py runs (`bench/box_session.sh ab REPS "a|..." "b|..."`).

Pairs run i of the baseline with run i of the candidate. A pair is kept only when neither
side's `host_load.siblings` (busy share of the SMT siblings of the replica's cores: other
tenants on our physical cores) exceeds --max-sibling-load. For the kept pairs it reports the
paired difference, with a 95 % t-interval, of the server's own efficiency figures and of
req/s. The primary efficiency figure is the server's user-space instructions per request
(`server_user_instr_per_req`, hardware counters of its workers: its own code's work, which
neither a saturated peer nor sibling load moves), then its user cycles and its busy CPU per
request (CPU minus empty polls). Raw CPU µs per request is shown last: at saturation a server
and its load generator both run flat out, so that figure is their CPUs' wall time over the
request count for both, the same number by construction.
Because the sibling load moves every run's cost, it also fits one line through all runs of
both variants, server µs/request = a + d * [candidate] + b * sibling load, and reports d (the
candidate's cost at equal sibling load) with its 95 % interval: a gate that keeps every run.

  python bench/ab_report.py DIR --baseline r1 --candidate final [--max-sibling-load 0.02]
"""
from __future__ import annotations

import argparse
import json
import math
import statistics
import sys
from pathlib import Path

# two-sided 95 % t quantiles by degrees of freedom
_T95 = {1: 12.706, 2: 4.303, 3: 3.182, 4: 2.776, 5: 2.571, 6: 2.447, 7: 2.365, 8: 2.306, 9: 2.262, 10: 2.228,
        12: 2.179, 15: 2.131, 20: 2.086, 30: 2.042}


def t95(df: int) -> float:
    if df in _T95:
        return _T95[df]
    # between table rows take the smaller df's (larger, conservative) quantile
    return next(v for k, v in sorted(_T95.items(), reverse=True) if k <= df)


def ci(diffs: list[float]) -> tuple[float, float, float]:
    m = statistics.fmean(diffs)
    if len(diffs) < 2:
        return m, float("nan"), float("nan")
    h = t95(len(diffs) - 1) * statistics.stdev(diffs) / math.sqrt(len(diffs))
    return m, m - h, m + h


# Efficiency figures, primary first (see the module docstring); a figure is reported when both
# runs of a pair carry it.
EFFICIENCY = (("server_user_instr_per_req", "server user instr/req"),
              ("server_user_cycles_per_req", "server user cycles/req"),
              ("server_busy_cpu_us_per_req", "server busy CPU us/req"),
              ("server_cpu_us_per_req", "server CPU us/req (raw)"))


def load(d: Path, label: str) -> dict[int, dict]:
    out = {}
    for p in d.glob(f"{label}_*.json"):
        try:
            out[int(p.stem.rsplit("_", 1)[1])] = json.loads(p.read_text().strip().splitlines()[-1])
        except (ValueError, IndexError, json.JSONDecodeError):
            pass
    return out


def sib(r: dict) -> float:
    # None in SMT-pair layouts: both threads of each core are ours, so no other tenant shares them
    return max((h.get("siblings") or 0.0) for h in r.get("host_load", [{}]))


def adjusted(rows: list[dict]) -> dict | None:
    """Least squares us = a + d*cand + b*sib over both variants' runs; d with a 95 % interval."""
    import numpy as np

    ys, xs = [], []
    for r in rows:
        ys += [r["us_base"], r["us_cand"]]
        xs += [[1.0, 0.0, r["sib_base"]], [1.0, 1.0, r["sib_cand"]]]
    if len(ys) < 5:
        return None
    X, y = np.array(xs), np.array(ys)
    if np.ptp(X[:, 2]) == 0.0:  # no sibling load varies (e.g. SMT-pair layouts): plain two-group fit
        X = X[:, :2]
    coef, *_ = np.linalg.lstsq(X, y, rcond=None)
    resid = y - X @ coef
    dof = len(y) - X.shape[1]
    s2 = float(resid @ resid) / dof
    cov = s2 * np.linalg.inv(X.T @ X)
    se = math.sqrt(cov[1, 1])
    slope = float(coef[2]) if X.shape[1] == 3 else 0.0
    base = coef[0] + slope * statistics.fmean([r["sib_base"] for r in rows])
    h = t95(dof) * se
    return {"delta_us": round(float(coef[1]), 4), "delta_pct": round(100 * float(coef[1]) / base, 2),
            "ci95_pct": [round(100 * float(coef[1] - h) / base, 2), round(100 * float(coef[1] + h) / base, 2)],
            "us_per_sibling_pct": round(slope / 100, 4), "runs": len(y)}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("dir")
    ap.add_argument("--baseline", required=True)
    ap.add_argument("--candidate", required=True)
    ap.add_argument("--max-sibling-load", type=float, default=0.02)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    d = Path(a.dir)
    base, cand = load(d, a.baseline), load(d, a.candidate)
    rows, kept = [], []
    for i in sorted(set(base) & set(cand)):
        b, c = base[i], cand[i]
        ok = sib(b) <= a.max_sibling_load and sib(c) <= a.max_sibling_load
        rows.append({"pair": i, "kept": ok, "sib_base": round(sib(b), 4), "sib_cand": round(sib(c), 4),
                     "us_base": b["server_cpu_us_per_req"], "us_cand": c["server_cpu_us_per_req"],
                     "rps_base": b["value"], "rps_cand": c["value"]})
        if ok:
            kept.append(rows[-1])
    print(f"{'pair':>4} {'kept':>5} {'sib A':>7} {'sib B':>7} {'us/req A':>9} {'us/req B':>9} {'req/s A':>11} {'req/s B':>11}")
    for r in rows:
        print(f"{r['pair']:>4} {str(r['kept']):>5} {r['sib_base']:>7.3f} {r['sib_cand']:>7.3f} {r['us_base']:>9.3f} "
              f"{r['us_cand']:>9.3f} {r['rps_base']:>11.0f} {r['rps_cand']:>11.0f}")
    res = {"baseline": a.baseline, "candidate": a.candidate, "pairs": len(rows), "kept": len(kept),
           "max_sibling_load": a.max_sibling_load, "rows": rows}
    if kept:
        print(f"\n{a.candidate} vs {a.baseline}, {len(kept)} kept pairs (siblings <= {a.max_sibling_load:.0%}):")
        for key, label in EFFICIENCY:
            pairs = [(base[r["pair"]].get(key), cand[r["pair"]].get(key)) for r in kept]
            pairs = [(x, y) for x, y in pairs if x and y]
            if not pairs:
                continue
            m, lo, hi = ci([100.0 * (y - x) / x for x, y in pairs])
            res[f"{key}_delta_pct"] = {"mean": round(m, 2), "ci95": [round(lo, 2), round(hi, 2)], "pairs": len(pairs)}
            print(f"  {label:<26}: {m:+.2f} % (95 % CI {lo:+.2f} .. {hi:+.2f}), {len(pairs)} pairs")
        res["server_us_per_req_delta_pct"] = res.get("server_cpu_us_per_req_delta_pct")
        rps = [100.0 * (r["rps_cand"] - r["rps_base"]) / r["rps_base"] for r in kept]
        m2, lo2, hi2 = ci(rps)
        res["rps_delta_pct"] = {"mean": round(m2, 2), "ci95": [round(lo2, 2), round(hi2, 2)]}
        print(f"  {'req/s':<26}: {m2:+.2f} % (95 % CI {lo2:+.2f} .. {hi2:+.2f})")
    else:
        print("\nno pair passed the sibling-load gate")
    adj = adjusted(rows)
    if adj:
        res["server_us_per_req_adjusted"] = adj
        print(f"  adjusted for sibling load (all {len(rows)} pairs): candidate {adj['delta_pct']:+.2f} % server us/req "
              f"(95 % CI {adj['ci95_pct'][0]:+.2f} .. {adj['ci95_pct'][1]:+.2f}); "
              f"{adj['us_per_sibling_pct']:+.3f} us per sibling-load percent")
    if a.json:
        Path(a.json).write_text(json.dumps(res, indent=1) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
