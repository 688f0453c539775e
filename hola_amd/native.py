"""Locating, building and loading the native (C++20) parts of hola.

The product is a set of native executables (``hola``, ``hola_loadgen``, ``hola_rrproxy``)
plus the ``hola_amd._native`` pybind11 module that exposes the server's own core code to
the Python tests. Everything is built in-tree with CMake + Ninja into ``build/<preset>/``
(the module lands next to this file), so a snapshot of the repository carries the build.

Nothing here falls back to a Python re-implementation: if the native code is missing and
cannot be built, :func:`load_native` and :func:`binary` raise.
"""
from __future__ import annotations

import fcntl
import os
import shutil
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
BUILD_ROOT = REPO / "build"
BINARIES = ("hola", "hola_loadgen", "hola_rrproxy", "hola_zipkin_sink")

# preset name -> extra CMake arguments
PRESETS = {
    "release": ["-DCMAKE_BUILD_TYPE=Release"],
    "debug": ["-DCMAKE_BUILD_TYPE=Debug"],
    "tsan": ["-DCMAKE_BUILD_TYPE=RelWithDebInfo", "-DHOLA_SANITIZE=thread", "-DHOLA_BUILD_PYTHON=OFF"],
    "asan": ["-DCMAKE_BUILD_TYPE=RelWithDebInfo", "-DHOLA_SANITIZE=address,undefined", "-DHOLA_BUILD_PYTHON=OFF"],
    # gcov line coverage of the native code under the test suite (HOLA_SANITIZER=coverage)
    "coverage": ["-DCMAKE_BUILD_TYPE=Debug", "-DHOLA_COVERAGE=ON", "-DHOLA_BUILD_PYTHON=OFF"],
    # clock reads counted and exported (tests/test_clock_reads.py)
    "clockcount": ["-DCMAKE_BUILD_TYPE=Release", "-DHOLA_COUNT_CLOCK_READS=ON", "-DHOLA_BUILD_PYTHON=OFF"],
    # pre-AVX2 nodes: x86-64-v2, the parser's and line scan's byte loops (src/core/isa.h)
    "portable": ["-DCMAKE_BUILD_TYPE=Release", "-DHOLA_MARCH=x86-64-v2", "-DHOLA_MTUNE=generic",
                 "-DHOLA_BUILD_PYTHON=OFF"],
    # compile-flag A/B variants of the release build (server binary via HOLA_SERVER_BIN)
    "release-v4": ["-DCMAKE_BUILD_TYPE=Release", "-DHOLA_MARCH=x86-64-v4", "-DHOLA_BUILD_PYTHON=OFF"],
    "release-o3lto": ["-DCMAKE_BUILD_TYPE=Release", "-DHOLA_OPT=-O3", "-DHOLA_LTO=ON", "-DHOLA_BUILD_PYTHON=OFF"],
    "release-nofp": ["-DCMAKE_BUILD_TYPE=Release", "-DHOLA_FRAME_POINTERS=OFF", "-DHOLA_BUILD_PYTHON=OFF"],
    "release-v4-o3lto": ["-DCMAKE_BUILD_TYPE=Release", "-DHOLA_MARCH=x86-64-v4", "-DHOLA_OPT=-O3", "-DHOLA_LTO=ON",
                         "-DHOLA_BUILD_PYTHON=OFF"],
}


class NativeBuildError(RuntimeError):
    pass


def build_dir(preset: str = "release") -> Path:
    return BUILD_ROOT / preset


# Inputs of the native build: C++ sources and headers, embedded assets, CMake files. Python
# and shell tooling under bench/ is not one (editing it must not trigger a rebuild).
_NATIVE_SUFFIXES = {".cc", ".h", ".cpp", ".hpp", ".cmake", ".html", ".json", ".yaml"}


def _sources_newer_than(target: Path) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    for sub in ("src", "bench", "assets", "cmake"):
        for p in (REPO / sub).rglob("*"):
            if p.suffix in _NATIVE_SUFFIXES and p.is_file() and p.stat().st_mtime > t:
                return True
    return (REPO / "CMakeLists.txt").stat().st_mtime > t


def _drop_stale_cache(bdir: Path) -> None:
    """A build tree copied to another path (e.g. a repo snapshot on a GPU box, where
    /root/repo is a symlink) keeps the old absolute paths in CMakeCache.txt and CMake
    refuses to reuse it. Reconfigure from scratch in that case (objects are rebuilt)."""
    cache = bdir / "CMakeCache.txt"
    if not cache.exists():
        return
    recorded = None
    for line in cache.read_text(errors="replace").splitlines():
        if line.startswith("CMAKE_CACHEFILE_DIR:"):
            recorded = line.split("=", 1)[1].strip()
            break
    if recorded is None or recorded != str(bdir):
        shutil.rmtree(bdir / "CMakeFiles", ignore_errors=True)
        cache.unlink(missing_ok=True)


def build(preset: str = "release", jobs: int | None = None, quiet: bool = True) -> Path:
    """Configures and builds `preset` in-tree; returns the build directory.

    Serialised with a file lock so concurrent ranks (torchrun) do not race.
    """
    if preset not in PRESETS:
        raise ValueError(f"unknown preset {preset!r}; choose from {sorted(PRESETS)}")
    if shutil.which("cmake") is None:
        raise NativeBuildError("cmake not found on PATH")
    bdir = build_dir(preset)
    bdir.mkdir(parents=True, exist_ok=True)
    lock_path = BUILD_ROOT / f".{preset}.lock"
    jobs = jobs or min(16, os.cpu_count() or 4)
    gen = ["-G", "Ninja"] if shutil.which("ninja") else []
    with open(lock_path, "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        try:
            out = subprocess.DEVNULL if quiet else None
            _drop_stale_cache(bdir)
            if not (bdir / "CMakeCache.txt").exists():
                cmd = ["cmake", "-S", str(REPO), "-B", str(bdir), *gen, *PRESETS[preset],
                       f"-DPython3_EXECUTABLE={sys.executable}"]
                r = subprocess.run(cmd, stdout=out, stderr=subprocess.PIPE, text=True)
                if r.returncode != 0:
                    raise NativeBuildError(f"cmake configure failed:\n{r.stderr[-4000:]}")
            r = subprocess.run(["cmake", "--build", str(bdir), "-j", str(jobs)], stdout=out,
                               stderr=subprocess.PIPE, text=True)
            if r.returncode != 0:
                raise NativeBuildError(f"native build failed:\n{r.stderr[-4000:]}")
        finally:
            fcntl.flock(lock, fcntl.LOCK_UN)
    return bdir


def ensure_built(preset: str = "release") -> Path:
    """Builds when an artefact is missing or older than the sources."""
    bdir = build_dir(preset)
    need = any(_sources_newer_than(bdir / b) for b in BINARIES)
    if preset == "release" and not list(Path(__file__).parent.glob("_native*.so")):
        need = True
    if need:
        build(preset)
    return bdir


def binary(name: str = "hola", preset: str = "release", build_if_missing: bool = True) -> Path:
    """Absolute path of a native executable (``HOLA_BIN_DIR`` overrides the build dir;
    ``HOLA_SERVER_BIN`` overrides the ``hola`` server alone, for compile-flag A/B runs)."""
    server = os.environ.get("HOLA_SERVER_BIN")
    if name == "hola" and server:
        p = Path(server)
        if not p.is_absolute():
            p = REPO / p
        if not p.exists():
            raise NativeBuildError(f"HOLA_SERVER_BIN {p} is missing")
        return p
    override = os.environ.get("HOLA_BIN_DIR")
    bdir = Path(override) if override else build_dir(preset)
    p = bdir / name
    if not p.exists():
        if build_if_missing and not override:
            ensure_built(preset)
        if not p.exists():
            raise NativeBuildError(f"native binary {p} is missing (build with `python -m hola_amd build`)")
    return p


def load_native():
    """Imports the pybind11 module (built in-tree); raises if it cannot be built."""
    try:
        from hola_amd import _native  # type: ignore[attr-defined]
        return _native
    except ImportError:
        ensure_built("release")
        from hola_amd import _native  # type: ignore[attr-defined]
        return _native
