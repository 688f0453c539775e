#!/usr/bin/env python3
"""User-space instructions per request of several server binaries, interleaved.

  python bench/instr_ab.py OUT_DIR head=build/release/hola r1=build/r1/hola [--rounds 3]
  python bench/instr_ab.py OUT_DIR 'traced=build/release/hola' 'untraced=build/release/hola|--no-tracing'

The CPU-time A/Bs (`bench/ab_report.py`) resolve about ±0.7 % per session on the shared box,
as large as what is left between trees. The server's own code, though, is deterministic work
per request: each side here runs under `bench/probes/instr_count.cc` (hardware counters of the
server and every thread it starts, user space only), serves a fixed closed-loop load of
/api/hola from `hola_loadgen` without busy-polling (a spin loop would count as work), and is
stopped with SIGTERM; its `shutdown complete (N requests served)` line gives N. The kernel's
share (the send/recv/epoll_wait sequence, the same for every tree) is not counted.

Prints one JSON line per run and a summary: instructions and cycles per request per side
(mean and spread over rounds). Sides run in the given order, reversed every other round.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import signal
import statistics
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from hola_amd import native  # noqa: E402
from hola_amd.utils.cpu import physical_cores  # noqa: E402


def build_counter(out: Path) -> Path:
    exe = out / "instr_count"
    subprocess.run(["g++", "-O2", "-std=c++20", "-o", str(exe), str(ROOT / "bench/probes/instr_count.cc")],
                   check=True)
    return exe


def run_side(counter: Path, label: str, exe: str, out: Path, rnd: int, cpus: list[int], lg_cpus: list[int],
             seconds: float, conns: int, count_loadgen: bool = False, aloha_port: int = 0) -> dict:
    exe, _, more = exe.partition("|")  # "path/to/hola|--no-tracing ...": extra server flags
    extra = more.split()
    path, expect = "/api/hola", ["--expect-body", "Hola de ab"]
    if aloha_port:  # --chain: this server is hola A, calling hola B as its aloha
        extra += ["--aloha-url", f"http://127.0.0.1:{aloha_port}/", "--aloha-path", "api/hola-chaining",
                  "--feign-log", "none", "--hystrix-pool-size", "128"]
        path, expect = "/api/hola-chaining", ["--verify-body"]
    # --count loadgen: the counters go on the load generator instead (its instructions per
    # completed request); the server runs plainly
    srv_wrap = [] if count_loadgen else [str(counter), str(out / f"{label}_{rnd}.counters.json"), "--"]
    lg_wrap = [str(counter), str(out / f"{label}_{rnd}.counters.json"), "--"] if count_loadgen else []
    tag = f"{label}_{rnd}"
    pf = out / f"{tag}.port"
    pf.unlink(missing_ok=True)
    log = open(out / f"{tag}.log", "w")
    threads = len(cpus)
    srv = subprocess.Popen([*srv_wrap, exe, "--host", "127.0.0.1",
                            "--port", "0", "--port-file", str(pf), "--threads", str(threads), "--cpu-list",
                            ",".join(map(str, cpus)), "--busy-poll-us", "0", "--hostname", "ab", *extra],
                           stdout=log, stderr=log)
    deadline = time.monotonic() + 20
    while not (pf.exists() and pf.read_text().strip()):
        if srv.poll() is not None or time.monotonic() > deadline:
            srv.kill()
            srv.wait()
            raise RuntimeError(f"{label}: server did not start (see {tag}.log)")
        time.sleep(0.02)
    port = int(pf.read_text().strip())
    try:
        lg = subprocess.run([*lg_wrap, str(native.binary("hola_loadgen")), "--targets", f"127.0.0.1:{port}", "-c", str(conns),
                             "-t", str(len(lg_cpus)), "--cpu-list", ",".join(map(str, lg_cpus)), "--path", path,
                             *expect, "--duration", str(seconds)],
                            capture_output=True, text=True, timeout=seconds + 60)
    finally:
        srv.send_signal(signal.SIGTERM)
        srv.wait(timeout=30)
        log.close()
    text = (out / f"{tag}.log").read_text()
    m = re.search(r"shutdown complete \((\d+) requests served\)", text)
    if lg.returncode != 0 or not m:
        raise RuntimeError(f"{label}: run failed: loadgen rc {lg.returncode} {lg.stderr[-500:]!r}; {tag}.log")
    served = int(m.group(1))
    cnt = json.loads((out / f"{tag}.counters.json").read_text())
    lgj = json.loads(lg.stdout.strip().splitlines()[-1])
    r = {"side": label, "round": rnd, "served": served, "loadgen_rps": lgj.get("rps"),
         "errors": (lgj.get("latency") or {}).get("errors"), "instructions": cnt["instructions"], "cycles": cnt["cycles"],
         "counter_error": cnt.get("error", "")}
    if cnt["instructions"] is not None and served:
        r["instructions_per_req"] = cnt["instructions"] / served
        r["cycles_per_req"] = cnt["cycles"] / served if cnt["cycles"] is not None else None
    return r


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("sides", nargs="+", help="label=path/to/hola[|extra server flags]")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--threads", type=int, default=4, help="server workers (and load-generator threads)")
    ap.add_argument("--connections", type=int, default=64)
    ap.add_argument("--count", choices=["server", "loadgen"], default="server",
                    help="which side runs under the counters (per request served either way)")
    ap.add_argument("--chain", action="store_true",
                    help="/api/hola-chaining: each side is hola A, calling one uncounted hola B (as "
                         "bench/chain_bench.py: B answers with its own fallback) on cores of its own")
    a = ap.parse_args()
    out = Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    sides = [s.split("=", 1) for s in a.sides]
    counter = build_counter(out)
    cores = physical_cores(sorted(os.sched_getaffinity(0)))
    if len(cores) < 2 * a.threads:
        raise SystemExit(f"need {2 * a.threads} physical cores, have {len(cores)}")
    cpus, lg_cpus = cores[:a.threads], cores[a.threads:2 * a.threads]
    b_proc, aloha_port = None, 0
    if a.chain:
        b_cpus = cores[2 * a.threads:3 * a.threads]
        if len(b_cpus) < a.threads:
            raise SystemExit(f"--chain needs {3 * a.threads} physical cores, have {len(cores)}")
        pf = out / "b.port"
        pf.unlink(missing_ok=True)
        b_log = open(out / "b.log", "w")
        b_proc = subprocess.Popen([str(native.binary("hola")), "--host", "127.0.0.1", "--port", "0", "--port-file",
                                   str(pf), "--threads", str(len(b_cpus)), "--cpu-list", ",".join(map(str, b_cpus)),
                                   "--hostname", "B", "--aloha-url", "http://127.0.0.1:1/", "--feign-log", "none",
                                   "--no-tracing", "--feign-retry", "off", "--log-level", "warn"],
                                  stdout=b_log, stderr=b_log)
        deadline = time.monotonic() + 20
        while not (pf.exists() and pf.read_text().strip()):
            if b_proc.poll() is not None or time.monotonic() > deadline:
                raise SystemExit("hola B did not start (b.log)")
            time.sleep(0.02)
        aloha_port = int(pf.read_text().strip())
    results = []
    try:
        with open(out / "runs.jsonl", "w") as f:
            for rnd in range(1, a.rounds + 1):
                order = sides if rnd % 2 else sides[::-1]
                for label, exe in order:
                    r = run_side(counter, label, exe, out, rnd, cpus, lg_cpus, a.seconds, a.connections,
                                 a.count == "loadgen", aloha_port)
                    results.append(r)
                    f.write(json.dumps(r) + "\n")
                    f.flush()
                    print(json.dumps(r), flush=True)
    finally:
        if b_proc:
            b_proc.terminate()
            b_proc.wait(timeout=30)
    summary = {}
    for label, _ in sides:
        ipr = [r["instructions_per_req"] for r in results if r["side"] == label and "instructions_per_req" in r]
        cpr = [r["cycles_per_req"] for r in results if r["side"] == label and r.get("cycles_per_req")]
        if ipr:
            summary[label] = {"instructions_per_req": round(statistics.mean(ipr), 1),
                              "instructions_spread": round(max(ipr) - min(ipr), 1),
                              "cycles_per_req": round(statistics.mean(cpr), 1) if cpr else None, "runs": len(ipr)}
    (out / "summary.json").write_text(json.dumps(summary, indent=1) + "\n")
    print(json.dumps({"summary": summary}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
