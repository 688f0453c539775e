#!/usr/bin/env python3
"""Symbolise a `hola --cpu-profile FILE` profile and print where the CPU time went.

    python bench/cpuprof_report.py FILE [--top 25] [--threads hola-w] [--json OUT]

Each sample is one period of a thread's CPU time (user + kernel). Kernel time shows up at
the libc wrapper of the syscall it was spent in (send, recv, epoll_wait, ...), so `self`
splits both user code and syscalls. `total` counts a function once per sample whose stack
contains it (callers included). Symbols come from `nm` (the static table if present, else
the dynamic one), looked up by the ELF virtual address of each sampled instruction. A name
marked `~` comes from a dynamic table only (stripped libc): the sample is at or after that
symbol, possibly in a local function next to it; the syscall wrappers are exact.
"""
from __future__ import annotations

import argparse
import bisect
import collections
import json
import struct
import subprocess
import sys


def parse(path: str) -> dict:
    prof = {"threads": {}, "maps": [], "stacks": [], "period_ns": 0, "samples": 0, "dropped": 0,
            "event": "cpu-time", "period_cycles": 0}
    with open(path) as f:
        for line in f:
            parts = line.split()
            if not parts or parts[0].startswith("#"):
                continue
            if parts[0] in ("period_ns", "samples", "dropped", "period_cycles"):
                prof[parts[0]] = int(parts[1])
            elif parts[0] == "event":  # HOLA_CPUPROF_EVENT=user-cycles / user-instructions
                prof["event"] = parts[1]
            elif parts[0] == "thread":
                prof["threads"][int(parts[1])] = parts[2] if len(parts) > 2 else "?"
            elif parts[0] == "map":
                lo, hi = (int(x, 16) for x in parts[1].split("-"))
                obj = parts[6] if len(parts) > 6 else parts[1]
                prof["maps"].append((lo, hi, int(parts[3], 16), obj))
            elif parts[0] == "stack":
                prof["stacks"].append((int(parts[1]), int(parts[2]), [int(x, 16) for x in parts[3:]]))
    prof["maps"].sort()
    return prof


def load_segments(obj: str) -> list[tuple[int, int, int]]:
    """PT_LOAD (p_offset, p_filesz, p_vaddr) of an ELF64 file; [] if unreadable."""
    try:
        with open(obj, "rb") as f:
            hdr = f.read(64)
            if hdr[:4] != b"\x7fELF" or hdr[4] != 2:
                return []
            phoff, = struct.unpack_from("<Q", hdr, 0x20)
            phentsize, phnum = struct.unpack_from("<HH", hdr, 0x36)
            f.seek(phoff)
            out = []
            for _ in range(phnum):
                ph = f.read(phentsize)
                p_type, _flags, p_offset, p_vaddr, _paddr, p_filesz = struct.unpack_from("<IIQQQQ", ph)
                if p_type == 1:
                    out.append((p_offset, p_filesz, p_vaddr))
            return out
    except OSError:
        return []


class Symbols:
    def __init__(self, obj: str):
        self.addrs: list[int] = []
        self.names: list[str] = []
        self.approx = False  # only the dynamic table: a local function takes its neighbour's name
        for dyn in ([], ["-D"]):
            try:
                out = subprocess.run(["nm", "-C", "-n", "--defined-only", *dyn, obj], capture_output=True,
                                     text=True, timeout=120).stdout
            except (OSError, subprocess.TimeoutExpired):
                out = ""
            for line in out.splitlines():
                parts = line.split(" ", 2)
                if len(parts) == 3 and parts[1].lower() in ("t", "w", "i"):
                    self.addrs.append(int(parts[0], 16))
                    self.names.append(parts[2])
            if self.addrs:
                self.approx = bool(dyn)
                break

    def lookup(self, vaddr: int) -> str | None:
        i = bisect.bisect_right(self.addrs, vaddr) - 1
        if i < 0:
            return None
        return ("~" + self.names[i]) if self.approx else self.names[i]


class Resolver:
    def __init__(self, maps):
        self.maps = maps
        self.starts = [m[0] for m in maps]
        self.segs: dict[str, list] = {}
        self.syms: dict[str, Symbols] = {}
        self.cache: dict[int, tuple[str, str]] = {}

    def resolve(self, addr: int) -> tuple[str, str]:
        if addr in self.cache:
            return self.cache[addr]
        i = bisect.bisect_right(self.starts, addr) - 1
        res = ("?", f"0x{addr:x}")
        if i >= 0 and addr < self.maps[i][1]:
            lo, _hi, off, obj = self.maps[i]
            short = obj.rsplit("/", 1)[-1]
            file_off = addr - lo + off
            if obj.startswith("["):
                res = (short, obj)
            else:
                if obj not in self.segs:
                    self.segs[obj] = load_segments(obj)
                    self.syms[obj] = Symbols(obj)
                vaddr = None
                for p_off, p_sz, p_va in self.segs[obj]:
                    if p_off <= file_off < p_off + p_sz:
                        vaddr = file_off - p_off + p_va
                        break
                name = self.syms[obj].lookup(vaddr) if vaddr is not None else None
                res = (short, name or f"{short}+0x{file_off:x}")
        self.cache[addr] = res
        return res


def short_name(fn: str, width: int = 110) -> str:
    return fn if len(fn) <= width else fn[:width - 3] + "..."


def report(prof: dict, top: int, thread_prefix: str) -> dict:
    r = Resolver(prof["maps"])
    self_ = collections.Counter()
    total = collections.Counter()
    by_obj = collections.Counter()
    by_thread = collections.Counter()
    n = 0
    for count, tid, pcs in prof["stacks"]:
        tname = prof["threads"].get(tid, "?")
        by_thread[tname] += count
        if thread_prefix and not tname.startswith(thread_prefix):
            continue
        n += count
        frames = [r.resolve(pc if k == 0 else pc - 1) for k, pc in enumerate(pcs)]
        obj, fn = frames[0]
        self_[fn] += count
        by_obj[obj] += count
        for f in set(fn for _, fn in frames):
            total[f] += count
    return {"samples": n, "period_ns": prof["period_ns"], "dropped": prof["dropped"],
            "threads": dict(by_thread.most_common()),
            "by_object": {k: round(v / max(1, n), 4) for k, v in by_obj.most_common()},
            "self": [(round(v / max(1, n), 4), k) for k, v in self_.most_common(top)],
            "total": [(round(v / max(1, n), 4), k) for k, v in total.most_common(top)]}


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("profile")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--threads", default="hola-w", help="only threads whose name starts with this ('' = all)")
    ap.add_argument("--json", default="", help="also write the report here")
    a = ap.parse_args()
    rep = report(parse(a.profile), a.top, a.threads)
    prof = parse(a.profile)
    if prof["event"] in ("user-cycles", "user-instructions"):
        unit = prof["event"].split("-", 1)[1]
        print(f"{rep['samples']} samples of {prof['period_cycles']} user-space {unit} each "
              f"({rep['samples'] * prof['period_cycles'] / 1e9:.2f} G {unit}) of threads '{a.threads or '*'}'; "
              f"dropped {rep['dropped']}")
    else:
        cpu_s = rep["samples"] * rep["period_ns"] / 1e9
        print(f"{rep['samples']} samples ({cpu_s:.2f} CPU-s) of threads '{a.threads or '*'}'; dropped {rep['dropped']}")
    print("threads:", ", ".join(f"{k} {v}" for k, v in rep["threads"].items()))
    print("\nby object (self):")
    for k, v in rep["by_object"].items():
        print(f"  {100 * v:6.2f} %  {k}")
    for key in ("self", "total"):
        print(f"\n{key}:")
        for frac, fn in rep[key]:
            print(f"  {100 * frac:6.2f} %  {short_name(fn)}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rep, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
