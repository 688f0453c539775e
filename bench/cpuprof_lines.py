#!/usr/bin/env python3
"""Source lines of one function's own samples in a `hola --cpu-profile` file.

  python bench/cpuprof_lines.py PROFILE FUNCTION_SUBSTRING [--threads hola-w] [--top 25]

Takes the samples whose innermost frame resolves (as in bench/cpuprof_report.py) to a
function whose name contains FUNCTION_SUBSTRING and maps their addresses to file:line with
addr2line (inlined callers included, innermost first). Run it where the profiled binary is,
on the box for a box profile. With HOLA_CPUPROF_EVENT=user-cycles the counts are user-space
cycles, so this is where a function's own cost sits.
"""
from __future__ import annotations

import argparse
import collections
import subprocess
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))

import cpuprof_report as cr  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("profile")
    ap.add_argument("function")
    ap.add_argument("--threads", default="hola-w")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    prof = cr.parse(a.profile)
    r = cr.Resolver(prof["maps"])
    by_addr: dict[tuple[str, int], int] = collections.Counter()
    total = 0
    for count, tid, pcs in prof["stacks"]:
        if a.threads and not prof["threads"].get(tid, "?").startswith(a.threads):
            continue
        total += count
        obj, fn = r.resolve(pcs[0])
        if a.function not in fn:
            continue
        i = next(k for k, m in enumerate(prof["maps"]) if m[0] <= pcs[0] < m[1])
        lo, _hi, off, path = prof["maps"][i]
        by_addr[(path, pcs[0] - lo + off)] += count
    mine = sum(by_addr.values())
    print(f"{mine} of {total} samples ({100 * mine / max(1, total):.2f} %) in functions matching {a.function!r}")
    lines: dict[str, int] = collections.Counter()
    by_obj = collections.defaultdict(list)
    for (path, off), n in by_addr.items():
        by_obj[path].append((off, n))
    for path, items in by_obj.items():
        segs = cr.load_segments(path)
        vaddrs = []
        for off, _n in items:
            va = next((off - p + v for p, sz, v in segs if p <= off < p + sz), off)
            vaddrs.append(hex(va))
        # one (function, file:line) pair per address: the innermost inlined location
        out_q = subprocess.run(["addr2line", "-f", "-C", "-e", path, *vaddrs], capture_output=True, text=True,
                               timeout=300).stdout.splitlines()
        for k, (_off, n) in enumerate(items):
            where = out_q[2 * k + 1] if 2 * k + 1 < len(out_q) else "?"
            lines[where.split(" (")[0]] += n
    for where, n in lines.most_common(a.top):
        print(f"  {100 * n / max(1, mine):6.2f} %  {where}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
