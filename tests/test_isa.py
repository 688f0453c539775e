"""The build's x86-64 ISA level: a binary built for x86-64-v3 (AVX2, the
release default) on a CPU without it exits 1 with one clear line before any worker starts,
instead of dying with SIGILL; and the `portable` build (x86-64-v2, no AVX2: the parser's and
the line scan's byte loops) answers every request exactly as the release build does."""
import os
import random
import socket
import subprocess
import sys

import pytest

from hola_amd import native
from hola_amd.server import HolaProcess


@pytest.mark.parametrize("name", ["hola", "hola_loadgen", "hola_rrproxy", "hola_zipkin_sink"])
def test_missing_feature_is_one_clear_line_and_exit_1(name):
    exe = native.binary(name)
    r = subprocess.run([str(exe), "--port", "0"], capture_output=True, text=True, timeout=30,
                       env={**os.environ, "HOLA_ISA_PRETEND_MISSING": "avx2,bmi2"})
    assert r.returncode == 1, (r.returncode, r.stderr)
    lines = r.stderr.strip().splitlines()
    assert len(lines) == 1, r.stderr
    assert lines[0].startswith(f"{name}: this build needs an x86-64-v3 CPU and this one lacks avx2,bmi2")
    assert "portable" in lines[0] and r.stdout == ""


def test_module_import_fails_with_the_line_printed_first():
    """the Python module checks the CPU in its first static initialiser (baseline
    code, init priority 101, src/pybind/isa_flag.cc): the line reaches stderr before any
    initialiser built for the -march runs, and the import then fails with it."""
    code = ("import sys\n"
            "try:\n"
            "    import hola_amd._native\n"
            "except ImportError as e:\n"
            "    print('IMPORT ERROR:', e)\n"
            "    sys.exit(3)\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                       cwd=str(native.REPO), env={**os.environ, "HOLA_ISA_PRETEND_MISSING": "avx2"})
    assert r.returncode == 3, (r.returncode, r.stdout, r.stderr)
    line = "hola_amd._native: this build needs an x86-64-v3 CPU and this one lacks avx2"
    assert r.stderr.startswith(line), r.stderr
    assert "IMPORT ERROR: " + line in r.stdout


def test_features_above_the_build_level_are_not_required(native):
    assert native.isa_build_level() == "x86-64-v3" and native.isa_missing_features() == ""
    # AVX-512 is x86-64-v4: pretending it is absent must not stop a v3 build
    r = subprocess.run([str(native_binary()), "--help"], capture_output=True, text=True, timeout=30,
                       env={**os.environ, "HOLA_ISA_PRETEND_MISSING": "avx512f,avx512bw"})
    assert r.returncode == 0 and r.stderr.startswith("usage: hola")


def native_binary():
    return native.binary("hola")


def _raw(port: int, req: bytes) -> bytes:
    with socket.create_connection(("127.0.0.1", port), timeout=5) as s:
        s.sendall(req)
        s.shutdown(socket.SHUT_WR)
        out = b""
        while True:
            try:
                b = s.recv(65536)
            except (ConnectionResetError, socket.timeout):
                break
            if not b:
                break
            out += b
    # Date is the only header that may differ between two servers
    return b"\r\n".join(ln for ln in out.split(b"\r\n") if not ln.lower().startswith(b"date:"))


def _corpus(n: int, seed: int = 5) -> list[bytes]:
    rnd = random.Random(seed)
    alphabet = b"/apiholhealth?=&%2F.;x-_~AZ09 \x01\x7f\x80"
    fixed = [b"/api/hola", b"/api/hola?x=1", b"/api/./hola", b"/api/hola;jsessionid=1", b"/api/health",
             b"/api/hola-chaining-nope", b"/" + b"a" * 40, b"/api/hola?" + b"q" * 40, b"/api/ho\x01la" + b"p" * 40,
             b"/api/swagger.json", b"http://host:8080/api/hola", b"/%2e%2e/api/hola", b"/api/hola?x=" + b"\x7f" * 3]
    out = []
    for i in range(n):
        target = fixed[i] if i < len(fixed) else b"/" + bytes(rnd.choice(alphabet) for _ in range(rnd.randrange(0, 64)))
        method = rnd.choice([b"GET", b"GET", b"HEAD", b"POST", b"OPTIONS", b"G@T"])
        version = rnd.choice([b"HTTP/1.1", b"HTTP/1.1", b"HTTP/1.0", b"HTTP/2.0", b"HTTP/1.x"])
        pad = rnd.choice([b"", b"X-Pad: " + b"p" * rnd.randrange(0, 48) + b"\r\n"])  # vector vs byte paths
        accept = rnd.choice([b"", b"Accept: application/json\r\n", b"Accept: text/*\r\n"])
        body = b"Content-Length: 0\r\n" if method == b"POST" else b""
        out.append(method + b" " + target + b" " + version + b"\r\nHost: x\r\n" + pad + accept + body +
                   b"Connection: close\r\n\r\n")
    return out


def test_portable_build_answers_like_release():
    """The x86-64-v2 build (no AVX2 anywhere) against the release build, request by request:
    status line, headers and body must be byte-identical for valid and malformed heads,
    short and long targets (byte loop vs 32-byte vector scan in the release build)."""
    native.build("portable")
    exe = native.build_dir("portable") / "hola"  # (not binary(): HOLA_BIN_DIR may name a sanitizer build)
    dis = subprocess.run(["objdump", "-d", str(exe)], capture_output=True, text=True, timeout=120)
    if dis.returncode == 0:
        assert "%ymm" not in dis.stdout  # no 256-bit AVX instruction in the portable binary
    args = ["--no-tracing", "--log-level", "warn"]
    with HolaProcess(args=args, env={"HOSTNAME": "p"}, threads=1, exe=native.build_dir("release") / "hola") as rel, \
            HolaProcess(args=args, env={"HOSTNAME": "p"}, threads=1, exe=exe) as port:
        for req in _corpus(400):
            assert _raw(rel.port, req) == _raw(port.port, req), req
