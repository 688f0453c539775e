"""Tail attribution of open-loop latency points: the per-thread scheduler
facts the curve records (hola_amd/parallel/hostmetrics.py) and the causes bench/tail_report.py
names from a point's record."""
import importlib.util
import os
import threading
import time
from pathlib import Path

from hola_amd.parallel.hostmetrics import task_stats, task_stats_delta

ROOT = Path(__file__).resolve().parent.parent


def _tail_report():
    spec = importlib.util.spec_from_file_location("tail_report", ROOT / "bench" / "tail_report.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_task_stats_carry_the_run_delay_of_every_thread():
    stop = threading.Event()

    def spin():
        while not stop.is_set():
            pass

    t = threading.Thread(target=spin, name="spinner")
    a = task_stats(os.getpid())
    t.start()
    time.sleep(0.3)
    b = task_stats(os.getpid())
    stop.set()
    t.join()
    assert all("run_delay_ms" in d and d["run_delay_ms"] >= 0 for d in b.values())
    delta = task_stats_delta(a, b, group=lambda comm: "all")
    g = delta["all"]
    assert g["run_delay_ms"] >= 0 and 0 <= g["run_delay_max_thread_ms"] <= max(g["run_delay_ms"], 0) + 1e-6
    assert g["cpu_s"] > 0


def test_causes_name_cpu_waits_lateness_and_gaps():
    tr = _tail_report()
    row = {"server_loop": {"gaps_over_1ms": 2, "gaps_over_10ms": 1},
           "server_threads": {"workers": {"invol": 7, "run_delay_ms": 12.5, "run_delay_max_thread_ms": 9.0}},
           "loadgen": {"send_late_max_ns": 3_000_000, "sends_late_1ms": 4, "behind_max_ns": 5_000_000,
                       "run_delay_ns": 2_500_000, "run_delay_max_thread_ns": 2_000_000},
           "host_load_server": {"irq_own": 0.2}}
    c = " ".join(tr.causes(row))
    for want in ("gaps(2 >1ms, 1 >10ms)", "preempted(7)", "cpu-wait(12.5 ms, max thread 9.0 ms)",
                 "late(3000 us, 4 sends >1ms)", "behind(5000 us)", "lg-cpu-wait(2.5 ms, max thread 2.0 ms)",
                 "irq(0.20)"):
        assert want in c, (want, c)
    quiet = {"server_threads": {"workers": {"invol": 0, "run_delay_ms": 0.2}}, "loadgen": {"run_delay_ns": 10_000}}
    assert tr.causes(quiet) == []
