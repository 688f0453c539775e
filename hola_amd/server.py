"""Run a ``hola`` server process (used by tests, smoke(), bench.py and the scaling harness)."""
from __future__ import annotations

import os
import signal
import subprocess
import tempfile
import time
from pathlib import Path

from hola_amd.native import binary
from hola_amd.utils.net import http_get


class HolaProcess:
    """A ``hola`` child process listening on an ephemeral (or given) port.

    Use as a context manager. ``env`` entries are added to a minimal environment (so the
    test controls HOSTNAME / ZIPKIN_SERVER_URL / JAVA_OPTIONS / hello explicitly); pass
    ``inherit_env=True`` to start from os.environ instead.
    """

    def __init__(self, args: list[str] | None = None, env: dict | None = None, port: int = 0,
                 threads: int = 2, cpu_list: str | None = None, preset: str = "release",
                 inherit_env: bool = False, log_level: str = "info", exe: Path | None = None,
                 stderr_path: str | None = None, wrapper: list[str] | None = None):
        self.args = list(args or [])
        # e.g. ["setarch", "x86_64", "-R"] for TSan builds; $HOLA_WRAPPER supplies a default
        self.wrapper = list(wrapper) if wrapper is not None else os.environ.get("HOLA_WRAPPER", "").split()
        self.port = port
        self.threads = threads
        self.cpu_list = cpu_list
        self.exe = exe or binary("hola", preset)
        keep = ("PATH", "LANG", "LC_ALL", "TMPDIR", "LD_LIBRARY_PATH", "TSAN_OPTIONS", "ASAN_OPTIONS",
                "UBSAN_OPTIONS", "LSAN_OPTIONS", "SSL_CERT_FILE", "SSL_CERT_DIR",
                "HOLA_CPUPROF_EVENT", "HOLA_CPUPROF_PERIOD")  # --cpu-profile's sampling event
        base = dict(os.environ) if inherit_env else {k: v for k, v in os.environ.items() if k in keep}
        if not inherit_env:
            base.pop("HOSTNAME", None)
        base.update(env or {})
        self.env = base
        self.log_level = log_level
        self.proc: subprocess.Popen | None = None
        self.startup_ms: float | None = None
        self._tmp = tempfile.TemporaryDirectory(prefix="hola-")
        self.stderr_path = stderr_path or os.path.join(self._tmp.name, "stderr.log")

    @property
    def host(self) -> str:
        return "127.0.0.1"

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self.port}"

    def start(self, timeout: float = 30.0) -> "HolaProcess":
        port_file = os.path.join(self._tmp.name, "port")
        cmd = [*self.wrapper, str(self.exe), "--host", "127.0.0.1", "--port", str(self.port), "--threads", str(self.threads),
               "--port-file", port_file, "--log-level", self.log_level, *self.args]
        if self.cpu_list:
            cmd += ["--cpu-list", self.cpu_list]
        self._stderr = open(self.stderr_path, "wb")
        t0 = time.monotonic()
        self.proc = subprocess.Popen(cmd, env=self.env, stdout=subprocess.DEVNULL, stderr=self._stderr)
        deadline = time.monotonic() + timeout
        while time.monotonic() < deadline:
            if self.proc.poll() is not None:
                raise RuntimeError(f"hola exited early ({self.proc.returncode}): {self.log()}")
            if os.path.exists(port_file):
                try:
                    self.port = int(Path(port_file).read_text().strip())
                    self.startup_ms = (time.monotonic() - t0) * 1000.0  # exec -> listening
                    break
                except ValueError:
                    pass
            time.sleep(0.01)
        else:
            self.stop()
            raise RuntimeError(f"hola did not start within {timeout}s: {self.log()}")
        return self

    def get(self, path: str, headers: dict | None = None, method: str = "GET", timeout: float = 5.0,
            body: bytes | None = None):
        return http_get("127.0.0.1", self.port, path, headers=headers, method=method, timeout=timeout, body=body)

    def memory_kb(self) -> dict:
        """VmRSS / VmHWM (peak) of the running server, in kB."""
        out = {}
        try:
            for line in Path(f"/proc/{self.proc.pid}/status").read_text().splitlines():
                if line.startswith(("VmRSS:", "VmHWM:")):
                    k, v = line.split(":", 1)
                    out[k] = int(v.split()[0])
        except (OSError, ValueError, AttributeError):
            pass
        return out

    def log(self) -> str:
        try:
            return Path(self.stderr_path).read_text(errors="replace")
        except OSError:
            return ""

    def stop(self, sig: int = signal.SIGTERM, timeout: float = 15.0) -> int | None:
        if self.proc is None:
            return None
        if self.proc.poll() is None:
            self.proc.send_signal(sig)
            try:
                self.proc.wait(timeout=timeout)
            except subprocess.TimeoutExpired:
                self.proc.kill()
                self.proc.wait()
        rc = self.proc.returncode
        try:
            self._stderr.close()
        except Exception:
            pass
        return rc

    def __enter__(self) -> "HolaProcess":
        return self.start()

    def __exit__(self, *exc) -> None:
        self.stop()
        self._tmp.cleanup()
