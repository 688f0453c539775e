"""The driver entry points run on CPU too (the service never needs the GPU)."""
import importlib.util
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent


def load_entry():
    spec = importlib.util.spec_from_file_location("graft_entry", ROOT / "__graft_entry__.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_smoke_runs(hola_bin, capsys):
    load_entry().smoke()
    assert "smoke: ok" in capsys.readouterr().out


def test_cli_info_and_help(capsys):
    from hola_amd.__main__ import main

    assert main(["info"]) == 0
    out = capsys.readouterr().out
    assert "physical cores" in out and "plan x8" in out
    assert "build          : hola 0.0.1-SNAPSHOT (revision " in out  # what is installed, first
    assert main([]) == 0


def _gone(procs, timeout=10.0):
    import time

    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline:
        if not any(q.is_running() and q.status() != "zombie" for q in procs):
            return True
        time.sleep(0.05)
    return False


@pytest.mark.parametrize("lb,stop", [("proxy", "SIGINT"), ("reuseport", "SIGINT"), ("proxy", "SIGTERM"),
                                     ("reuseport", "SIGHUP")])
def test_cli_cluster_round_robin(hola_bin, lb, stop):
    """`python -m hola_amd cluster`: 2 supervised replicas behind the round-robin proxy or in
    one SO_REUSEPORT group. Ctrl-C (SIGINT), SIGTERM (systemd, a container stop) and SIGHUP
    all stop the proxy and every replica before the command exits 0: none is left behind."""
    import http.client
    import signal
    import subprocess
    import sys
    import time

    import psutil

    from hola_amd.utils.net import free_port

    port = free_port()
    p = subprocess.Popen([sys.executable, "-m", "hola_amd", "cluster", "--replicas", "2", "--port", str(port),
                          "--proxy-threads", "1", "--lb", lb], cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                         text=True)
    try:
        line = ""
        deadline = time.monotonic() + 60
        while "hola cluster:" not in line and time.monotonic() < deadline and p.poll() is None:
            line = p.stdout.readline()
        assert "hola cluster:" in line, line
        seen = set()
        for _ in range(8 if lb == "proxy" else 60):  # reuseport: kernel hash, not strict rotation
            c = http.client.HTTPConnection("127.0.0.1", port, timeout=5)
            c.request("GET", "/api/hola")
            r = c.getresponse()
            assert r.status == 200
            seen.add(r.read())
            c.close()
        assert seen == {b"Hola de replica-0", b"Hola de replica-1"}
        children = psutil.Process(p.pid).children(recursive=True)
        assert len(children) == (3 if lb == "proxy" else 2), children
    finally:
        p.send_signal(getattr(signal, stop))
        rc = p.wait(timeout=30)
    assert rc == 0
    assert _gone(children), [q for q in children if q.is_running()]


def test_cli_serve_forwards_termination(hola_bin, tmp_path):
    """`python -m hola_amd serve` runs the binary as a child: SIGTERM to the wrapper reaches
    the server, which drains and exits 0, and the wrapper exits with that status."""
    import signal
    import subprocess
    import sys
    import time

    import psutil

    pf = tmp_path / "port"
    p = subprocess.Popen([sys.executable, "-m", "hola_amd", "serve", "--host", "127.0.0.1", "--port", "0",
                          "--threads", "1", "--port-file", str(pf)], cwd=ROOT,
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    deadline = time.monotonic() + 60
    while not (pf.exists() and pf.read_text().strip()) and time.monotonic() < deadline and p.poll() is None:
        time.sleep(0.02)
    assert pf.exists(), p.stderr.read() if p.poll() is not None else "no port file"
    (child,) = psutil.Process(p.pid).children()
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=30) == 0
    assert _gone([child])
    assert "received SIGTERM: draining" in p.stderr.read()
