import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


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
    for p in procs:
        p.stop()
