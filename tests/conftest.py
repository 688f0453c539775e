import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def pytest_sessionstart(session):
    # HOLA_SANITIZER=tsan|asan: build that preset and run every integration test against it
    # (SURVEY.md §5.2), e.g. `HOLA_SANITIZER=asan pytest tests/test_contract.py tests/test_chaining.py`.
    san = os.environ.get("HOLA_SANITIZER")
    if not san and "PYTEST_XDIST_WORKER" not in os.environ:
        # build stale binaries once, before any (xdist) worker runs them: a worker's own
        # rebuild would relink executables that other workers are starting
        from hola_amd.native import ensure_built

        ensure_built("release")
    if san:
        from hola_amd.native import build, build_dir

        build(san)
        os.environ["HOLA_BIN_DIR"] = str(build_dir(san))
        if san == "tsan":
            import platform
            import shutil

            os.environ.setdefault("TSAN_OPTIONS", "halt_on_error=1 exitcode=66")
            if shutil.which("setarch"):  # gcc 11 TSan vs high-entropy mmap ASLR (see test_sanitizers)
                os.environ.setdefault("HOLA_WRAPPER", f"setarch {platform.machine()} -R")
        else:
            os.environ.setdefault("ASAN_OPTIONS", "detect_leaks=1 halt_on_error=1 exitcode=66")
            os.environ.setdefault("UBSAN_OPTIONS", "halt_on_error=1 print_stacktrace=1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: runs on the MI355X box (host-side perf/bench checks)")
    config.addinivalue_line("markers", "slow: longer integration tests")
    config.addinivalue_line("markers", "sanitizer: runs the integration suite against tsan/asan builds")


@pytest.fixture(scope="session")
def native():
    from hola_amd.native import load_native

    return load_native()


@pytest.fixture(scope="session")
def hola_bin():
    from hola_amd.native import binary, ensure_built

    ensure_built("release")
    return binary("hola")


@pytest.fixture
def hola(hola_bin):
    """Factory: hola(args=[...], env={...}) -> started HolaProcess (stopped at teardown)."""
    from hola_amd.server import HolaProcess

    procs = []

    def start(args=None, env=None, threads=2, **kw):
        env = {"HOSTNAME": "testhost", **(env or {})}
        p = HolaProcess(args=args, env=env, threads=threads, **kw).start()
        procs.append(p)
        return p

    yield start
    reports = []
    for p in procs:
        rc = p.stop()
        if os.environ.get("HOLA_SANITIZER"):
            # Under a sanitizer build every server must exit cleanly and report nothing,
            # including leaks found at exit (after the test's own assertions ran).
            log = p.log()
            # (a test whose server exits with the exit watchdog's status 3 by design says so)
            if rc != getattr(p, "expected_rc", 0) or "Sanitizer" in log or "runtime error" in log:
                reports.append((rc, log[-4000:]))
                with open(os.path.join(os.environ.get("TMPDIR", "/tmp"), "hola_sanitizer_report.log"), "a") as f:
                    f.write(log)
    assert not reports, reports[0]
