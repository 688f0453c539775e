"""Driver for the native closed-loop load generator (bench/loadgen.cc)."""
from __future__ import annotations

import json
import subprocess

from hola_amd.native import binary

SUB = 64  # must match src/core/histogram.h


def bin_value(b: int) -> int:
    if b < SUB:
        return b
    octave, sub = divmod(b - SUB, SUB)
    msb = octave + 6
    lo = (1 << msb) + (sub << (msb - 6))
    return lo + ((1 << (msb - 6)) >> 1)


def decode_hist(s: str) -> dict[int, int]:
    out: dict[int, int] = {}
    if not s:
        return out
    for part in s.split(","):
        b, c = part.split(":")
        out[int(b)] = out.get(int(b), 0) + int(c)
    return out


def merge_hists(hists: list[dict[int, int]]) -> dict[int, int]:
    out: dict[int, int] = {}
    for h in hists:
        for b, c in h.items():
            out[b] = out.get(b, 0) + c
    return out


def escape_body(b: str) -> str:
    """--expect-body argument form of a body (the loadgen unescapes \\n \\r \\t \\\\)."""
    return b.replace("\\", "\\\\").replace("\n", "\\n").replace("\r", "\\r").replace("\t", "\\t")


def body_args(expect_bodies: list[str] | None, verify_body: bool, alt_bodies: list[str] | None = None) -> list[str]:
    out: list[str] = []
    for b in expect_bodies or []:
        out += ["--expect-body", escape_body(b)]
    for b in alt_bodies or []:  # accepted second answers, counted as body_alt
        out += ["--alt-body", escape_body(b)]
    if verify_body:
        out += ["--verify-body"]
    return out


def percentile(hist: dict[int, int], p: float) -> int:
    total = sum(hist.values())
    if not total:
        return 0
    need = max(1, min(total, int(p / 100.0 * total + 0.5)))
    acc = 0
    for b in sorted(hist):
        acc += hist[b]
        if acc >= need:
            return bin_value(b)
    return bin_value(max(hist))


class ControlledLoadgen:
    """`hola_loadgen --control`: each run(R) completes R x connections requests, drawn by the
    connections from one shared budget (or exactly R per connection with `per_conn_quota`).
    `expect_bodies` (one per target, or one for all) and `verify_body` (learn each target's
    first 2xx body) make every response body checked; mismatches count as errors."""

    def __init__(self, targets: list[tuple[str, int]], connections: int, threads: int,
                 cpu_list: str | None = None, path: str = "/api/hola", target_offset: int = 0,
                 headers: list[str] | None = None, busy_poll_us: int = 0, per_conn_quota: bool = False,
                 busy_poll_pause: int = 0, epoll_lt: bool = False, pipeline: int = 1,
                 expect_bodies: list[str] | None = None, verify_body: bool = False,
                 conn_targets: list[int] | None = None, cpu_profile: str | None = None,
                 alt_bodies: list[str] | None = None):
        cmd = [str(binary("hola_loadgen")), "--targets", ",".join(f"{h}:{p}" for h, p in targets),
               "-c", str(connections), "-t", str(threads), "--path", path, "--control",
               "--target-offset", str(target_offset)] + body_args(expect_bodies, verify_body, alt_bodies)
        if cpu_list:
            cmd += ["--cpu-list", cpu_list]
        for h in headers or []:
            cmd += ["-H", h]
        if busy_poll_us:
            cmd += ["--busy-poll-us", str(busy_poll_us)]
            if busy_poll_pause:
                cmd += ["--busy-poll-pause", str(busy_poll_pause)]
        if per_conn_quota:
            cmd += ["--per-conn-quota"]
        if epoll_lt:
            cmd += ["--epoll-lt"]
        if pipeline > 1:
            cmd += ["--pipeline", str(pipeline)]
        if conn_targets:
            cmd += ["--conn-targets", ",".join(map(str, conn_targets))]
        if cpu_profile:
            cmd += ["--cpu-profile", cpu_profile]  # written when the generator quits
        self.proc = subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, bufsize=1)
        ready = self._read()
        if not ready.get("ready"):
            raise RuntimeError(f"loadgen failed to start: {ready}")

    def _read(self) -> dict:
        line = self.proc.stdout.readline()
        if not line:
            raise RuntimeError(f"loadgen exited (rc={self.proc.poll()})")
        return json.loads(line)

    def _cmd(self, c: str) -> dict:
        self.proc.stdin.write(c + "\n")
        self.proc.stdin.flush()
        out = self._read()
        if "error" in out:
            raise RuntimeError(f"loadgen: {out['error']}")
        return out

    def run(self, reqs_per_conn: int) -> dict:
        return self._cmd(f"run {reqs_per_conn}")

    def run_for(self, seconds: float, warm_s: float = 0.0) -> dict:
        """One continuous closed-loop run: every connection sends back to back for `warm_s` +
        `seconds`, then finishes its request in flight; only what completes after the warm-up
        counts (requests, errors, latency, bodies; elapsed_ns is that part). No idle gap inside
        it, as a series of `run`s has between them."""
        return self._cmd(f"runfor {max(1, int(round(seconds * 1000)))} {max(0, int(round(warm_s * 1000)))}")

    def stats(self) -> dict:
        return self._cmd("stats")

    def reset(self) -> dict:
        return self._cmd("reset")

    def close(self) -> None:
        if self.proc.poll() is None:
            try:
                self.proc.stdin.write("quit\n")
                self.proc.stdin.flush()
                self.proc.wait(timeout=10)
            except Exception:
                self.proc.kill()
                self.proc.wait()


def run_duration(targets: list[tuple[str, int]], connections: int, threads: int, duration_s: float,
                 warmup_s: float = 1.0, cpu_list: str | None = None, path: str = "/api/hola",
                 timeout: float | None = None, rate: float = 0.0, busy_poll_us: int = 0,
                 spin_us: int = 0, pipeline: int = 1, expect_bodies: list[str] | None = None,
                 verify_body: bool = False, alt_bodies: list[str] | None = None, busy_poll_pause: int = 0,
                 sched_slice_us: int = 0) -> dict:
    """wrk-style timed run (closed loop), or wrk2-style open loop at `rate` req/s with latency
    measured from intended send times; returns the loadgen's JSON summary. `busy_poll_us`
    spins in epoll after activity; `spin_us` (open loop) spins instead of sleeping when the
    next scheduled send is that close; `pipeline` > 1 sends that many requests per write
    (closed loop only)."""
    cmd = [str(binary("hola_loadgen")), "--targets", ",".join(f"{h}:{p}" for h, p in targets),
           "-c", str(connections), "-t", str(threads), "--path", path, "--duration", str(duration_s),
           "--warmup", str(warmup_s)] + body_args(expect_bodies, verify_body, alt_bodies)
    if cpu_list:
        cmd += ["--cpu-list", cpu_list]
    if rate > 0:
        cmd += ["--rate", str(rate)]
    if busy_poll_us:
        cmd += ["--busy-poll-us", str(busy_poll_us)]
        if busy_poll_pause:
            cmd += ["--busy-poll-pause", str(busy_poll_pause)]
    if spin_us:
        cmd += ["--spin-us", str(spin_us)]
    if sched_slice_us:
        cmd += ["--sched-slice-us", str(sched_slice_us)]
    if pipeline > 1:
        cmd += ["--pipeline", str(pipeline)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout or duration_s + warmup_s + 60)
    if r.returncode != 0:
        raise RuntimeError(f"loadgen failed: {r.stderr}")
    return json.loads(r.stdout.strip().splitlines()[-1])
