"""Docs that name code must stay true to it: every metric docs/OPERATIONS.md tells operators
to watch is exported by /metrics, and every flag it lists is accepted by `hola`."""
import re
from pathlib import Path

from hola_amd.testing.fakes import FakeAloha, FakeZipkin

ROOT = Path(__file__).resolve().parent.parent
OPS = (ROOT / "docs" / "OPERATIONS.md").read_text()


def test_operations_metrics_are_exported(hola):
    # (the package and the native binaries are not metrics)
    names = set(re.findall(r"`(hola_[a-z_]+)", OPS)) - {"hola_amd", "hola_loadgen", "hola_rrproxy", "hola_zipkin_sink", "hola_fpstack",
                                                      "hola_micro"}
    with FakeAloha() as aloha, FakeZipkin() as zipkin:
        s = hola(args=["--aloha-url", aloha.url, "--zipkin-url", zipkin.url, "--feign-log", "none",
                       "--busy-poll-us", "auto"])  # the spin counters exist only while spinning adapts
        s.get("/api/hola")
        s.get("/api/hola-chaining")
        _, _, body = s.get("/metrics")
    exported = set(re.findall(r"^(hola_[a-z_]+)", body.decode(), re.M))
    exported |= {n[:-len("_bucket")] for n in exported if n.endswith("_bucket")}
    # the workers' hardware counters exist only where perf_event_open is allowed (the GPU box
    # allows it; a container without a PMU does not)
    if "hola_worker_user_instructions_total" not in exported:
        names -= {"hola_worker_user_instructions_total", "hola_worker_user_cycles_total"}
    missing = sorted(n for n in names if n not in exported)
    assert not missing, missing


def test_operations_flags_are_accepted(hola_bin):
    import subprocess

    help_text = ""
    for exe in (hola_bin, hola_bin.parent / "hola_rrproxy"):  # the server's flags and the proxy's
        r = subprocess.run([str(exe), "--help"], capture_output=True, text=True)
        help_text += r.stdout + r.stderr
    flags = set(re.findall(r"`(--[a-z][a-z0-9-]+)", OPS)) - {"--replicas", "--out", "--lb", "--minutes", "--zipkin-sink",
                                                              "--profile-out", "--proxy-threads",
                                                              "--count", "--chain"}  # bench/instr_ab.py's
    missing = sorted(f for f in flags if f not in help_text)
    assert not missing, missing


def test_bench_describes_the_deployed_replica_as_it_runs():
    """bench.py's deployed_* sub-run starts the replica with the manifests' container args;
    its docstring must describe exactly those (it said "no busy-polling"
    while the manifests pass --busy-poll-us auto)."""
    import yaml

    dc = next(o for o in yaml.safe_load((ROOT / "deploy/openshift/hola-dc.yaml").read_text())["items"]
              if o["kind"] == "DeploymentConfig")
    args = dc["spec"]["template"]["spec"]["containers"][0]["args"]
    pairs = [f"{args[i]} {args[i + 1]}" for i in range(0, len(args), 2)]
    bench = (ROOT / "bench.py").read_text()
    doc = bench.split('"""')[1]
    flat = " ".join(doc.split())
    for p in pairs:
        assert f"`{p}" in flat or f"{p}`" in flat or p in flat, (p, flat)
    assert "no busy-polling" not in bench and "no busy polling" not in bench
    # the key comment next to deployed_* in the JSON
    assert all(p in " ".join(bench.split("**_deployed_keys(")[0].split()[-40:]) for p in pairs)


def _tracked(*paths):
    import subprocess

    r = subprocess.run(["git", "ls-files", *paths], cwd=ROOT, capture_output=True, text=True)
    if r.returncode != 0:
        import pytest
        pytest.skip("not a git checkout")
    return r.stdout.split()


def test_every_profile_path_the_docs_name_exists():
    """Numbers in the READMEs and docs point at profile sessions (`profiles/roundN/...`, or
    relative inside profiles/): each path named must still be in the tree after the per-run
    files were folded into tables (bench/fold_profiles.py)."""
    skip = {"SURVEY.md", "VERDICT.md", "ADVICE.md", "PAPERS.md", "SNIPPETS.md", "BASELINE.md"}
    missing = []
    for rel in _tracked("*.md"):
        md = ROOT / rel
        if md.name in skip:
            continue
        text = md.read_text(errors="replace")
        for m in re.finditer(r"`([^`\s]+)`|\(([^)\s]+)\)", text):
            tok = (m.group(1) or m.group(2)).strip("`").rstrip(".,:;").split("#")[0]
            if "://" in tok or "round" not in tok:
                continue
            if not re.match(r"^(\.\./)*(profiles/)?round\d|^(\.\./)*\d\d_|^(\.\./)*r\d+_", tok):
                continue
            if not any(p.exists() for p in (md.parent / tok, ROOT / tok, ROOT / "profiles" / tok)):
                missing.append((rel, tok))
    assert not missing, missing


def test_profiles_stay_folded():
    """raw per-run files are folded into tables; the tree keeps < 400 of them."""
    assert len(_tracked("profiles")) < 400
