"""`hola --cpu-profile`: per-thread CPU-time sampling of the server, symbolised by
bench/cpuprof_report.py (the host-side profile on boxes without perf)."""
import subprocess
import sys
from pathlib import Path

from hola_amd.parallel.loadgen import run_duration

ROOT = Path(__file__).resolve().parent.parent


def test_cpu_profile_samples_workers_under_load(hola, tmp_path):
    prof = tmp_path / "cpu.prof"
    s = hola(args=["--cpu-profile", str(prof), "--cpu-profile-hz", "2000"], threads=2)
    res = run_duration([("127.0.0.1", s.port)], 8, 2, 1.5, 0.2)
    assert res["latency"]["errors"] == 0
    assert s.stop() == 0
    text = prof.read_text()
    assert "period_ns 500000" in text
    assert " hola-w0\n" in text and " hola-log\n" in text and "map " in text
    out = subprocess.run([sys.executable, str(ROOT / "bench/cpuprof_report.py"), str(prof), "--top", "40",
                          "--json", str(tmp_path / "rep.json")], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    import json
    rep = json.loads((tmp_path / "rep.json").read_text())
    # the workers spent a good part of 1.5 s each on the CPU: 2 samples per CPU-ms
    assert rep["samples"] > 100, rep["samples"]
    assert set(rep["threads"]) >= {"hola-w0", "hola-w1"}
    names = [fn for _, fn in rep["total"]]
    # the stacks reach from the syscall wrappers up into the server's own code
    assert any("send" in fn for fn in names), names
    assert any("hola::EventLoop::run" in fn for fn in names), names
    assert any("hola::http::Connection::" in fn for fn in names), names


def test_user_cycle_profile_or_its_fallback(hola, tmp_path):
    """HOLA_CPUPROF_EVENT=user-cycles samples user-space cycles through the hardware counter
    where there is one (the box), and says so in the file; without a PMU (this container's VM)
    each thread falls back to the CPU-time timer, says so in its name, and the file is the
    plain CPU-time profile. Either way the report reads it."""
    prof = tmp_path / "cyc.prof"
    s = hola(args=["--cpu-profile", str(prof)], threads=2, env={"HOLA_CPUPROF_EVENT": "user-cycles",
                                                                "HOLA_CPUPROF_PERIOD": "100000"})
    res = run_duration([("127.0.0.1", s.port)], 8, 2, 1.0, 0.2)
    assert res["latency"]["errors"] == 0
    assert s.stop() == 0
    text = prof.read_text()
    if "event user-cycles" in text:
        assert "period_cycles 100000" in text and " hola-w0\n" in text
    else:
        assert " hola-w0 (CPU-time timer: no cycle counter)" in text
    out = subprocess.run([sys.executable, str(ROOT / "bench/cpuprof_report.py"), str(prof)],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and "samples" in out.stdout, out.stderr


def test_loadgen_cpu_profile(hola, tmp_path):
    from hola_amd.parallel.loadgen import ControlledLoadgen

    s = hola(threads=1)
    prof = tmp_path / "lg.prof"
    lg = ControlledLoadgen([("127.0.0.1", s.port)], 4, 2, cpu_profile=str(prof))
    try:
        r = lg.run(20000)
        assert r["errors"] == 0
    finally:
        lg.close()
    text = prof.read_text()
    assert " hola-lg0\n" in text and " hola-lg1\n" in text and "\nstack " in text


def test_fpstack_prints_every_thread_of_a_live_server(hola):
    """`hola_fpstack PID` (the executor runs it on a pod that outlives its grace period): one
    line per thread with its name and state, and return addresses inside the hola binary
    (the worker threads wait in EventLoop::run)."""
    from hola_amd import native

    s = hola(threads=2)
    out = subprocess.run([str(native.binary("hola_fpstack", build_if_missing=False)), str(s.proc.pid)],
                         capture_output=True, text=True, timeout=30).stdout
    lines = out.splitlines()
    names = {ln.split()[1] for ln in lines}
    assert {"hola", "hola-log", "hola-w0", "hola-w1"} <= names, out
    tasks = list(Path(f"/proc/{s.proc.pid}/task").iterdir())
    assert len(lines) == len(tasks), out
    w0 = next(ln for ln in lines if ln.split()[1] == "hola-w0")
    if "seize:" not in w0:  # ptrace may be restricted (yama ptrace_scope) where this runs
        assert "hola+0x" in w0, w0
    assert s.proc.poll() is None  # detached, still serving
    assert s.get("/api/health")[0] == 200
