"""Coverage-guided fuzzing of the native parsers (bench/fuzz/fuzz_parsers.cc): libFuzzer with
AddressSanitizer + UndefinedBehaviorSanitizer over the request parser, the chunked codecs, the
aloha client's response parser, the path decoders, the JSON list codec, the Properties and
Formatter emulations and the B3/Accept/URL/Retry-After readers, each with its invariants.

The reference's equivalents are JVM libraries, memory-safe by construction; this build's are
C++ and read the same untrusted bytes. Needs clang (`cmake --preset fuzz`); skipped without it.
A short run here keeps the target building and the seeds clean; longer campaigns:
`build/fuzz/hola_fuzz -max_total_time=600 -fork=4 CORPUS bench/fuzz/seeds`."""
import os
import shutil
import subprocess

import pytest

from hola_amd.native import REPO

FUZZ_DIR = REPO / "build" / "fuzz"
SEEDS = REPO / "bench" / "fuzz" / "seeds"
# Global-variable checks are compiled out in this build (CMakeLists.txt, HOLA_FUZZ: the
# toolchain misplaces instrumented string literals when ASan, UBSan and coverage combine);
# every fuzzed input sits in a heap block of exactly its size, where ASan's checks stay on.
FUZZ_ENV = {"ASAN_OPTIONS": "detect_leaks=1", "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}


def _build() -> str:
    if not shutil.which("clang++"):
        pytest.skip("clang++ not on PATH: the fuzz preset needs clang")
    if not (FUZZ_DIR / "build.ninja").exists():
        r = subprocess.run(["cmake", "--preset", "fuzz"], cwd=REPO, capture_output=True, text=True)
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    r = subprocess.run(["cmake", "--build", "--preset", "fuzz", "-j", str(min(8, os.cpu_count() or 1))], cwd=REPO,
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return str(FUZZ_DIR / "hola_fuzz")


def test_seeds_cover_every_target():
    selectors = {p.read_bytes()[0] % 9 for p in SEEDS.iterdir()}
    assert set(range(8)) <= selectors, selectors


def test_fuzz_parsers_short_campaign(tmp_path):
    exe = _build()
    corpus = tmp_path / "corpus"
    corpus.mkdir()
    r = subprocess.run([exe, "-max_total_time=25", "-print_final_stats=1", "-rss_limit_mb=2048", "-timeout=10",
                        f"-artifact_prefix={tmp_path}/", str(corpus), str(SEEDS)],
                       capture_output=True, text=True, env={**os.environ, **FUZZ_ENV}, timeout=120)
    out = r.stderr
    crashes = sorted(p.name for p in tmp_path.iterdir() if p.name.startswith(("crash-", "leak-", "oom-", "timeout-")))
    assert r.returncode == 0 and not crashes, (crashes, out[-6000:])
    runs = int(next(ln.rsplit(":", 1)[1] for ln in out.splitlines() if ln.startswith("stat::number_of_executed_units")))
    assert runs > 10000, out[-3000:]  # it really ran
