"""Configuration layering (DeltaSpike ordinals) and hot reload without
per-request I/O (inotify on the parent directory + polling fallback)."""
import os
import time
from pathlib import Path

import pytest


def wait_body(s, expected: bytes, timeout=3.0, path="/api/hola"):
    deadline = time.monotonic() + timeout
    body = None
    while time.monotonic() < deadline:
        _, _, body = s.get(path)
        if body == expected:
            return body
        time.sleep(0.02)
    return body


def test_resolver_ordinals(native):
    srcs = [("ConfigFile", 0, {"hello": "file %s"}), ("Env", 300, {"hello": "env %s"}),
            ("Sys", 400, {}), ("Props", 100, {"hello": "props %s"})]
    assert native.resolve(srcs, "hello", "Hola de %s")[:2] == ("env %s", "Env")
    srcs[2] = ("Sys", 400, {"hello": "sys %s"})
    assert native.resolve(srcs, "hello", "Hola de %s")[:2] == ("sys %s", "Sys")
    assert native.resolve([("ConfigFile", 0, {})], "hello", "Hola de %s") == ("Hola de %s", "default", "hello", False)


def test_resolver_project_stage_and_empty(native):
    srcs = [("F", 0, {"hello": "base %s", "hello.Production": "prod %s"})]
    assert native.resolve(srcs, "hello", "d")[0] == "prod %s"
    srcs = [("S", 400, {"org.apache.deltaspike.ProjectStage": "Development"}),
            ("F", 0, {"hello": "base %s", "hello.Production": "prod %s", "hello.Development": "dev %s"})]
    assert native.resolve(srcs, "hello", "d")[0] == "dev %s"
    # empty values fall back to the default
    assert native.resolve([("S", 400, {"hello": ""})], "hello", "Hola de %s")[0] == "Hola de %s"


def test_java_options_parsing(native):
    d = native.parse_java_options("-Xmx512m -Dconf=/etc/hola/translation.properties -Dflag '-Dq=a b' -Dx=1=2")
    assert d == {"conf": "/etc/hola/translation.properties", "flag": "", "q": "a b", "x": "1=2"}


def test_env_and_sysprop_override_file(hola, tmp_path):
    conf = tmp_path / "t.properties"
    conf.write_text("hello=file %s\n")
    s = hola(args=[f"-Dconf={conf}"], env={"HOSTNAME": "h", "hello": "env %s"})
    assert s.get("/api/hola")[2] == b"env h"
    s = hola(args=[f"-Dconf={conf}", "-Dhello=sys %s"], env={"HOSTNAME": "h", "hello": "env %s"})
    assert s.get("/api/hola")[2] == b"sys h"


def test_conf_from_java_options(hola, tmp_path):
    conf = tmp_path / "t.properties"
    conf.write_text("hello=Hi from %s\n")
    s = hola(env={"HOSTNAME": "h", "JAVA_OPTIONS": f"-Xmx512m -Dconf={conf}"})
    assert s.get("/api/hola")[2] == b"Hi from h"


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_until_port(hola_bin, tmp_path, args, env=None, timeout=10.0):
    """Starts the binary without --port/--host and returns (proc, bound port)."""
    import subprocess

    pf = tmp_path / "port"
    p = subprocess.Popen([str(hola_bin), "--threads", "1", "--port-file", str(pf), "--log-level", "warn", *args],
                         env={**os.environ, "HOSTNAME": "h", **(env or {})},
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline and p.poll() is None:
        if pf.exists() and pf.read_text().strip():
            return p, int(pf.read_text())
        time.sleep(0.02)
    p.kill()
    raise AssertionError(f"no port (rc {p.wait()}): {p.stderr.read().decode()}")


def _get(port, host="127.0.0.1"):
    import http.client

    c = http.client.HTTPConnection(host, port, timeout=5)
    c.request("GET", "/api/hola")
    r = c.getresponse()
    return r.status, r.read()


@pytest.mark.parametrize("via", ["argv", "java_options"])
def test_swarm_socket_binding_properties(hola_bin, tmp_path, via):
    """`java -Dswarm.http.port=P -Dswarm.port.offset=K -jar hola-swarm.jar` listens on P + K
    (WildFly Swarm 1.0 socket bindings), on swarm.bind.address; JAVA_OPTIONS works too."""
    port = _free_port()
    props = [f"-Dswarm.http.port={port - 1}", "-Dswarm.port.offset=1", "-Dswarm.bind.address=127.0.0.1"]
    args, env = (props, None) if via == "argv" else ([], {"JAVA_OPTIONS": "-Xmx512m " + " ".join(props)})
    p, bound = _run_until_port(hola_bin, tmp_path, args, env)
    try:
        assert bound == port
        assert _get(bound) == (200, b"Hola de h")
    finally:
        p.terminate()
        assert p.wait(timeout=10) == 0


def test_explicit_port_flag_wins_over_swarm_properties(hola_bin, tmp_path):
    p, bound = _run_until_port(hola_bin, tmp_path, ["--host", "127.0.0.1", "--port", "0",
                                                     "-Dswarm.http.port=1", "-Dswarm.port.offset=5"])
    try:
        assert bound not in (1, 6) and _get(bound)[0] == 200
    finally:
        p.terminate()
        p.wait(timeout=10)


@pytest.mark.parametrize("bad", [["-Dswarm.http.port=http"], ["-Dswarm.http.port=65535", "-Dswarm.port.offset=1"]])
def test_bad_swarm_port_is_a_usage_error(hola_bin, bad):
    import subprocess

    r = subprocess.run([str(hola_bin), "--threads", "1", *bad], capture_output=True, text=True, timeout=10)
    assert r.returncode == 2 and "swarm" in r.stderr


def test_missing_or_broken_conf_uses_default(hola, tmp_path):
    s = hola(args=[f"-Dconf={tmp_path / 'absent.properties'}"], env={"HOSTNAME": "h"})
    assert s.get("/api/hola")[2] == b"Hola de h"
    bad = tmp_path / "bad.properties"
    bad.write_text("hello=x %s\nk=\\uZZZZ\n")
    s = hola(args=[f"-Dconf={bad}"], env={"HOSTNAME": "h"})
    assert s.get("/api/hola")[2] == b"Hola de h"


def test_deltaspike_properties_file(hola, tmp_path):
    ds = tmp_path / "apache-deltaspike.properties"
    ds.write_text("hello=ds %s\n")
    conf = tmp_path / "t.properties"
    conf.write_text("hello=file %s\n")
    s = hola(args=["--deltaspike-properties", str(ds), f"-Dconf={conf}"], env={"HOSTNAME": "h"})
    assert s.get("/api/hola")[2] == b"ds h"  # ordinal 100 beats ConfigFile's 0


def test_hot_reload_in_place_edit(hola, tmp_path):
    conf = tmp_path / "t.properties"
    conf.write_text("hello=one %s\n")
    s = hola(args=[f"-Dconf={conf}"], env={"HOSTNAME": "h"})
    assert s.get("/api/hola")[2] == b"one h"
    conf.write_text("hello=two %s\n")
    assert wait_body(s, b"two h") == b"two h"
    deadline = time.monotonic() + 3  # the log writer thread may lag the response
    while "New value two %s for key hello" not in s.log() and time.monotonic() < deadline:
        time.sleep(0.05)
    assert "New value two %s for key hello" in s.log()


def test_hot_reload_rename_over(hola, tmp_path):
    conf = tmp_path / "t.properties"
    conf.write_text("hello=one %s\n")
    s = hola(args=[f"-Dconf={conf}"], env={"HOSTNAME": "h"})
    tmp = tmp_path / "t.tmp"
    tmp.write_text("hello=renamed %s\n")
    os.replace(tmp, conf)
    assert wait_body(s, b"renamed h") == b"renamed h"


def test_hot_reload_configmap_symlink_swap(hola, tmp_path):
    # Kubernetes ConfigMap volume layout: file -> ..data/file, ..data -> ..<timestamp>
    d1 = tmp_path / "..2026_01"
    d1.mkdir()
    (d1 / "translation.properties").write_text("hello=v1 %s\n")
    (tmp_path / "..data").symlink_to(d1.name)
    (tmp_path / "translation.properties").symlink_to("..data/translation.properties")
    s = hola(args=[f"-Dconf={tmp_path / 'translation.properties'}"], env={"HOSTNAME": "h"})
    assert s.get("/api/hola")[2] == b"v1 h"
    d2 = tmp_path / "..2026_02"
    d2.mkdir()
    (d2 / "translation.properties").write_text("hello=v2 %s\n")
    tmp_link = tmp_path / "..data_tmp"
    tmp_link.symlink_to(d2.name)
    os.replace(tmp_link, tmp_path / "..data")  # atomic swap, as kubelet does
    assert wait_body(s, b"v2 h") == b"v2 h"


def test_reload_file_created_later_and_deleted(hola, tmp_path):
    conf = tmp_path / "late.properties"
    s = hola(args=[f"-Dconf={conf}"], env={"HOSTNAME": "h"})
    assert s.get("/api/hola")[2] == b"Hola de h"
    conf.write_text("hello=late %s\n")
    assert wait_body(s, b"late h") == b"late h"
    conf.unlink()
    assert wait_body(s, b"Hola de h") == b"Hola de h"


def test_no_file_descriptor_leak(hola, tmp_path):
    # The reference leaks one FileReader per request (Configuration.java:29).
    conf = tmp_path / "t.properties"
    conf.write_text("hello=x %s\n")
    s = hola(args=[f"-Dconf={conf}"], threads=1)
    pid = s.proc.pid
    for _ in range(50):
        s.get("/api/hola")
    n0 = len(os.listdir(f"/proc/{pid}/fd"))
    import http.client
    c = http.client.HTTPConnection("127.0.0.1", s.port)
    for _ in range(3000):
        c.request("GET", "/api/hola")
        c.getresponse().read()
    c.close()
    time.sleep(0.1)
    n1 = len(os.listdir(f"/proc/{pid}/fd"))
    assert n1 <= n0 + 2, (n0, n1)


def test_hystrix_config_file_hot_reload(hola, tmp_path):
    """Archaius re-reads config.properties; here the watcher re-applies Hystrix settings."""
    from hola_amd.testing.fakes import FakeAloha

    hc = tmp_path / "config.properties"
    hc.write_text("hystrix.command.default.execution.isolation.thread.timeoutInMilliseconds=2000\n")
    with FakeAloha(mode="slow", delay_s=0.5) as aloha:
        s = hola(args=["--aloha-url", aloha.url, "--hystrix-config", str(hc), "--feign-log", "none"])
        t0 = time.monotonic()
        st, _, body = s.get("/api/hola-chaining")
        assert b"Aloha mai" in body and time.monotonic() - t0 >= 0.45  # 2000 ms budget: no timeout
        hc.write_text("hystrix.command.default.execution.isolation.thread.timeoutInMilliseconds=100\n")
        deadline = time.monotonic() + 3
        while time.monotonic() < deadline:
            _, _, body = s.get("/api/hola-chaining")
            if b"fallback" in body:
                break
        assert b"Aloha response (fallback)" in body
        metrics = s.get("/metrics")[2].decode()
        reloads = int(next(l for l in metrics.splitlines() if l.startswith("hola_config_reloads_total ")).split()[1])
        assert reloads >= 1


def test_deltaspike_ordinal_override(hola, tmp_path):
    ds = tmp_path / "apache-deltaspike.properties"
    ds.write_text("deltaspike_ordinal=500\nhello=ds %s\n")  # now above system properties (400)
    s = hola(args=["--deltaspike-properties", str(ds), "-Dhello=sys %s"], env={"HOSTNAME": "h"})
    assert s.get("/api/hola")[2] == b"ds h"


def test_non_regular_conf_sources_are_refused(hola, tmp_path):
    s = hola(args=["-Dconf=/dev/zero"], env={"HOSTNAME": "h"})
    assert s.get("/api/hola")[2] == b"Hola de h"
    fifo = tmp_path / "fifo"
    os.mkfifo(fifo)  # opening a FIFO with no writer must not hang startup or the watcher
    s = hola(args=[f"-Dconf={fifo}"], env={"HOSTNAME": "h"})
    assert s.get("/api/hola")[2] == b"Hola de h"
