#!/usr/bin/env python3
"""Soak test: one replica under mixed load for a long time, sampling its resident memory,
open file descriptors and error counts, to show the service is flat (no leaks) over time.

Load mix, all running concurrently:
  * closed-loop GET /api/hola from the native load generator (most of the traffic);
  * GET /api/hola-chaining against a fake aloha that cycles ok / slow / 500 / garbage /
    connection-drop, so the breaker opens and closes and timeouts fire;
  * two /hystrix.stream subscribers, plus one that never reads (its backlog must stay
    bounded and the server must close it after --hystrix-stream-stall-ms); /metrics scrapes;
  * a config hot reload every few seconds.

    python bench/soak.py --minutes 5 --out soak.json
"""
import argparse
import json
import os
import sys
import threading
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

from hola_amd.parallel.loadgen import run_duration  # noqa: E402
from hola_amd.server import HolaProcess  # noqa: E402
from hola_amd.testing.fakes import FakeAloha  # noqa: E402
from hola_amd.utils.cpu import format_cpu_list, plan_node, split_server_loadgen  # noqa: E402
from hola_amd.utils.net import http_get  # noqa: E402

ap = argparse.ArgumentParser(description=__doc__)
ap.add_argument("--minutes", type=float, default=5)
ap.add_argument("--sample-s", type=float, default=10)
ap.add_argument("--feign-log", default="basic", choices=("basic", "none"),
                help="the replica's Feign logging (basic = the default, two log-ring lines per aloha call)")
ap.add_argument("--aloha-pipeline", type=int, default=1, help="the replica's --aloha-pipeline")
ap.add_argument("--chain-clients", type=int, default=1,
                help="concurrent /api/hola-chaining clients (several keep pipelined connections busy)")
ap.add_argument("--out", default="")
a = ap.parse_args()

duration = a.minutes * 60
cores = plan_node(1)[0]
srv, lg = split_server_loadgen(cores, max(1, len(cores) // 2))
conf = Path("/tmp") / f"hola-soak-{os.getpid()}.properties"
conf.write_text("hello=Hola de %s (v0)\n")
stop = threading.Event()
samples, errors = [], []

with FakeAloha() as aloha, HolaProcess(
        args=["--aloha-url", aloha.url, "--feign-log", a.feign_log, f"-Dconf={conf}",
              "--aloha-pipeline", str(a.aloha_pipeline),
              "-Dhystrix.command.default.circuitBreaker.sleepWindowInMilliseconds=1000",
              "--hystrix-stream-stall-ms", "5000"],
        env={"HOSTNAME": "soak"}, threads=len(srv), cpu_list=format_cpu_list(srv), log_level="warn",
        # BASIC logging writes two lines per aloha call: kept off the disk
        stderr_path=os.devnull if a.feign_log == "basic" else None) as s:
    pid = s.proc.pid

    def chaining_client():
        while not stop.is_set():
            try:
                st, _, _ = http_get("127.0.0.1", s.port, "/api/hola-chaining", timeout=5)
                if st != 200:
                    errors.append(("chaining", st))
            except OSError as e:
                errors.append(("chaining", repr(e)))

    def chaining():
        modes = ["ok", "slow", "error", "ok", "garbage", "close", "unavailable", "ok"]
        extra = [threading.Thread(target=chaining_client, daemon=True) for _ in range(a.chain_clients - 1)]
        for t in extra:
            t.start()
        i = 0
        while not stop.is_set():
            aloha.set_mode(modes[i % len(modes)], delay_s=1.0)
            end = time.monotonic() + 3
            while time.monotonic() < end and not stop.is_set():
                try:
                    st, _, _ = http_get("127.0.0.1", s.port, "/api/hola-chaining", timeout=5)
                    if st != 200:
                        errors.append(("chaining", st))
                except OSError as e:
                    errors.append(("chaining", repr(e)))
            i += 1

    def stream():
        import socket
        while not stop.is_set():
            with socket.create_connection(("127.0.0.1", s.port), timeout=5) as c:
                c.sendall(b"GET /hystrix.stream?delay=100 HTTP/1.1\r\nHost: x\r\n\r\n")
                c.settimeout(0.5)
                end = time.monotonic() + 20
                while time.monotonic() < end and not stop.is_set():
                    try:
                        c.recv(65536)
                    except socket.timeout:
                        pass

    def stalled_stream():
        import socket
        while not stop.is_set():
            c = socket.socket()
            c.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4096)
            try:
                c.connect(("127.0.0.1", s.port))
                c.sendall(b"GET /hystrix.stream?delay=10 HTTP/1.1\r\nHost: x\r\n\r\n")
                stop.wait(8)  # never reads; the server gives up after 5 s without progress
            except OSError:
                pass
            finally:
                c.close()

    def reload():
        v = 0
        while not stop.wait(3):
            v += 1
            conf.write_text(f"hello=Hola de %s (v{v})\n")

    def sampler():
        t0 = time.monotonic()
        while not stop.is_set():
            try:
                rss = next(int(l.split()[1]) for l in open(f"/proc/{pid}/status") if l.startswith("VmRSS:"))
                fds = len(os.listdir(f"/proc/{pid}/fd"))
                _, _, m = http_get("127.0.0.1", s.port, "/metrics", timeout=5)
                metric = {l.split()[0]: int(float(l.split()[-1])) for l in m.decode().splitlines()
                          if l.startswith(("hola_http_requests_total ", "hola_event_loop_timers ",
                                           "hola_log_lines_dropped_total "))}
                samples.append({"t_s": round(time.monotonic() - t0, 1), "rss_kb": rss, "fds": fds,
                                "requests": metric["hola_http_requests_total"],
                                # pending loop timers follow the calls in flight (a leak grows them)
                                "timers": metric.get("hola_event_loop_timers", -1),
                                "log_dropped": metric.get("hola_log_lines_dropped_total", -1)})
                print(json.dumps(samples[-1]), flush=True)
            except (OSError, StopIteration, KeyError) as e:
                errors.append(("sampler", repr(e)))
            stop.wait(a.sample_s)

    threads = [threading.Thread(target=f, daemon=True)
               for f in (chaining, stream, stream, stalled_stream, reload, sampler)]
    for t in threads:
        t.start()
    res = run_duration([("127.0.0.1", s.port)], 64, len(lg), duration, 1.0, cpu_list=",".join(map(str, lg)))
    stop.set()
    for t in threads:
        t.join(timeout=30)
    alive = s.proc.poll() is None
    stream_stats = {}
    try:
        _, _, m = http_get("127.0.0.1", s.port, "/metrics", timeout=5)
        for l in m.decode().splitlines():
            if l.startswith(("hola_hystrix_stream_frames_skipped_total ", "hola_hystrix_stream_stalled_closed_total ")):
                stream_stats[l.split()[0]] = int(float(l.split()[1]))
    except OSError as e:
        errors.append(("metrics", repr(e)))
conf.unlink()

first, last = samples[1] if len(samples) > 1 else samples[0], samples[-1]
out = {
    "minutes": a.minutes, "hola_rps": res["rps"], "hola_p99_ms": res["latency"]["p99_ns"] / 1e6,
    "hola_errors": res["latency"]["errors"], "other_errors": errors[:20], "alive_at_end": alive,
    "rss_kb_first": first["rss_kb"], "rss_kb_last": last["rss_kb"], "rss_kb_max": max(x["rss_kb"] for x in samples),
    "fds_first": first["fds"], "fds_last": last["fds"], "stream": stream_stats,
    "timers_max": max(x.get("timers", -1) for x in samples), "timers_last": last.get("timers", -1),
    "log_dropped_last": last.get("log_dropped", -1), "feign_log": a.feign_log,
    "aloha_pipeline": a.aloha_pipeline, "chain_clients": a.chain_clients, "samples": samples,
}
print(json.dumps({k: v for k, v in out.items() if k != "samples"}))
if a.out:
    Path(a.out).write_text(json.dumps(out, indent=1))
