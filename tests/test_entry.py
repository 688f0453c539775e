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
    assert main([]) == 0


@pytest.mark.parametrize("lb", ["proxy", "reuseport"])
def test_cli_cluster_round_robin(hola_bin, lb):
    """`python -m hola_amd cluster`: 2 supervised replicas behind the round-robin proxy or in
    one SO_REUSEPORT group, stopped with SIGINT (what Ctrl-C does)."""
    import http.client
    import signal
    import subprocess
    import sys
    import time

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
    finally:
        p.send_signal(signal.SIGINT)
        rc = p.wait(timeout=30)
    assert rc == 0
