"""bench/ab_report.py: the gated A/B and its sibling-load fit (CPU only, synthetic run files)."""
from __future__ import annotations

import json
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "bench"))
import ab_report  # noqa: E402


def _write(d: Path, label: str, i: int, us: float, rps: float, siblings):
    line = {"value": rps, "server_cpu_us_per_req": us, "host_load": [{"siblings": siblings}]}
    (d / f"{label}_{i}.json").write_text("noise on stdout\n" + json.dumps(line) + "\n")


def test_fit_recovers_the_candidate_cost_at_equal_sibling_load(tmp_path):
    # cost = 1.8 + 0.09 * cand + 2.0 * sib: loaded runs must not be mistaken for the candidate
    sibs = [(0.0, 0.10), (0.05, 0.0), (0.10, 0.02), (0.01, 0.08)]
    for i, (sb, sc) in enumerate(sibs, 1):
        _write(tmp_path, "a", i, 1.8 + 2.0 * sb, 4.4e6, sb)
        _write(tmp_path, "b", i, 1.8 + 0.09 + 2.0 * sc, 4.3e6, sc)
    rows = []
    base, cand = ab_report.load(tmp_path, "a"), ab_report.load(tmp_path, "b")
    for i in sorted(base):
        rows.append({"sib_base": ab_report.sib(base[i]), "sib_cand": ab_report.sib(cand[i]),
                     "us_base": base[i]["server_cpu_us_per_req"], "us_cand": cand[i]["server_cpu_us_per_req"]})
    adj = ab_report.adjusted(rows)
    assert adj["delta_us"] == pytest.approx(0.09, abs=1e-6)
    assert adj["us_per_sibling_pct"] == pytest.approx(0.02, abs=1e-6)


def test_pair_layout_without_sibling_load_uses_the_two_group_fit(tmp_path):
    # SMT-pair runs report siblings = None (both threads are ours): no singular fit, no crash
    for i, (ua, ub) in enumerate([(2.29, 2.30), (2.30, 2.43), (2.48, 2.37)], 1):
        _write(tmp_path, "fpair", i, ua, 3.5e6, None)
        _write(tmp_path, "apair", i, ub, 3.4e6, None)
    out = tmp_path / "r.json"
    subprocess.run([sys.executable, str(ROOT / "bench" / "ab_report.py"), str(tmp_path), "--baseline", "fpair",
                    "--candidate", "apair", "--json", str(out)], check=True, capture_output=True, timeout=60)
    r = json.loads(out.read_text())
    assert r["kept"] == 3
    adj = r["server_us_per_req_adjusted"]
    assert adj["us_per_sibling_pct"] == 0.0
    assert adj["delta_us"] == pytest.approx((2.30 + 2.43 + 2.37 - 2.29 - 2.30 - 2.48) / 3, abs=1e-4)
    assert adj["ci95_pct"][0] < adj["delta_pct"] < adj["ci95_pct"][1]


def test_t_quantile_is_conservative_between_table_rows():
    assert ab_report.t95(11) == ab_report.t95(10)
    assert ab_report.t95(100) == ab_report.t95(30)


def test_instruction_counts_lead_the_efficiency_report(tmp_path):
    """with the servers' hardware-counter figures present, the report
    gives their paired delta first (raw CPU us/request of two saturated peers is the same
    number on both sides by construction)."""
    for i in range(1, 5):
        for label, instr in (("a", 1400.0), ("b", 1330.0 + i)):
            line = {"value": 4.5e6, "server_cpu_us_per_req": 1.72, "server_busy_cpu_us_per_req": 1.71,
                    "server_user_instr_per_req": instr, "server_user_cycles_per_req": 900.0,
                    "host_load": [{"siblings": 0.0}]}
            (tmp_path / f"{label}_{i}.json").write_text(json.dumps(line) + "\n")
    out = tmp_path / "r.json"
    r = subprocess.run([sys.executable, str(ROOT / "bench/ab_report.py"), str(tmp_path), "--baseline", "a",
                        "--candidate", "b", "--json", str(out)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    res = json.loads(out.read_text())
    assert res["server_user_instr_per_req_delta_pct"]["mean"] == pytest.approx(100 * (1332.5 - 1400) / 1400, abs=0.01)
    lines = [ln for ln in r.stdout.splitlines() if "%" in ln and "CI" in ln]
    assert "instr/req" in lines[0]
