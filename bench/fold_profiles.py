#!/usr/bin/env python3
"""Folds the raw per-run JSON files of profile sessions into one table per directory.

A session directory under profiles/ (an A/B, a repeat series, a rehearsal) keeps one JSON file
per run: `<label>_<rep>.json` (bench.py / chain_bench.py outputs; any directory with three or
more run outputs) and, from --profile-dir runs, `server_profile_rank<k>.json` stage histograms. The numbers the READMEs quote are the
session's `report.txt` / `summary.txt`; the per-run files behind them are folded here into
`runs.tsv` (one row per file: every numeric field up to two levels deep, plus a few strings
that say which variant it was), and the raw files are removed, except those a Markdown file
of the repository names.

    python bench/fold_profiles.py [--dry-run] [--min-files 2]
"""
from __future__ import annotations

import argparse
import json
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
PROFILES = ROOT / "profiles"
PER_RUN = re.compile(r"^(?P<label>.+?)_(?P<rep>\d+)\.json$|^(pair_)?n\d+(_[a-z]+)?\.json$")
# --profile-dir stage histograms: one file per prof_* directory, folded into the session's
# stage_profiles.tsv (grouped by the directory above the prof_* ones)
STAGES = re.compile(r"^server_profile_rank\d+\.json$")
# session-level files kept as they are: summaries, the round-end bench, single results
KEEP_NAMES = {"summary.json", "bench_default.json", "result.json", "soak.json", "kube.json", "micro.json",
              "plan8.json", "n8_plan_run.json"}
SKIP = {"config", "cgroup_throttle", "hist", "cpu_map", "per_replica", "chain_hystrix_events", "siblings"}
KEEP_STR = ("metric", "lb", "smt", "mode", "variant", "feign_log")


def flatten(d, prefix: str = "", depth: int = 0) -> dict:
    out = {}
    if isinstance(d, dict):
        for k, v in d.items():
            if k in SKIP:
                continue
            key = f"{prefix}{k}"
            if isinstance(v, bool):
                out[key] = int(v)
            elif isinstance(v, (int, float)):
                out[key] = v
            elif isinstance(v, str) and k in KEEP_STR and len(v) < 80:
                out[key] = v
            elif isinstance(v, dict) and depth < 1:
                out.update(flatten(v, key + ".", depth + 1))
            elif isinstance(v, list) and v and isinstance(v[0], dict) and depth < 1 and k == "host_load":
                out.update(flatten(v[0], key + ".", depth + 1))
    return out


def referenced_paths() -> set[Path]:
    """Every existing path a tracked Markdown file names (relative to itself, the repo, or profiles/)."""
    mds = subprocess.run(["git", "ls-files", "*.md"], cwd=ROOT, capture_output=True, text=True).stdout.split()
    out: set[Path] = set()
    for rel in mds:
        md = ROOT / rel
        for tok in re.findall(r"[\w./-]+\.(?:json|jsonl|txt|log|tsv|prof)", md.read_text(errors="replace")):
            for base in (md.parent, ROOT, PROFILES):
                p = (base / tok).resolve()
                if p.exists():
                    out.add(p)
    return out


def tracked(d: Path) -> list[Path]:
    names = subprocess.run(["git", "ls-files", "--", str(d)], cwd=ROOT, capture_output=True, text=True).stdout.split()
    return [ROOT / n for n in names]


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--dry-run", action="store_true")
    ap.add_argument("--min-files", type=int, default=2)
    ap.add_argument("--merge-sessions", default="",
                    help="comma-separated round directories (e.g. round1,round2) whose session "
                         "directories are merged into one session.txt each (every unreferenced text "
                         "file under the session, with a header per file)")
    a = ap.parse_args()
    keep = referenced_paths()
    by_dir: dict[tuple[Path, str], list[Path]] = {}
    removed = 0
    files_all = tracked(PROFILES)
    json_count: dict[Path, int] = {}
    for f in files_all:
        if f.suffix == ".json" and f.name not in KEEP_NAMES:
            json_count[f.parent] = json_count.get(f.parent, 0) + 1
    for f in files_all:
        if PER_RUN.match(f.name) or (f.suffix == ".json" and f.name not in KEEP_NAMES and json_count[f.parent] >= 3):
            by_dir.setdefault((f.parent, "runs.tsv"), []).append(f)
        elif STAGES.match(f.name):
            by_dir.setdefault((f.parent.parent, "stage_profiles.tsv"), []).append(f)
        elif f.name == "err.log" and f.resolve() not in keep and not a.dry_run:
            f.unlink()  # a bench's stderr (gloo banners, build lines); nothing a report quotes
            removed += 1
    # plain-text run logs: two or more unreferenced ones in a directory become one file with a
    # header per log (same bytes, one tracked file)
    logs: dict[Path, list[Path]] = {}
    for f in files_all:
        if f.suffix == ".log" and f.exists() and f.resolve() not in keep:
            logs.setdefault(f.parent, []).append(f)
    for d, fs in sorted(logs.items()):
        if len(fs) < 2:
            continue
        print(f"{d.relative_to(ROOT)}: {len(fs)} logs -> logs.txt")
        if a.dry_run:
            continue
        out = d / ("logs.txt" if not (d / "logs.txt").exists() else "logs_folded.txt")
        with open(out, "a") as w:
            for f in sorted(fs):
                w.write(f"===== {f.name} =====\n")
                w.write(f.read_text(errors="replace"))
                w.write("\n")
                f.unlink()
                removed += 1
    for (d, table), files in sorted(by_dir.items()):
        if len(files) < a.min_files:
            continue
        rows, cols = [], []
        for f in sorted(files, key=lambda p: (p.name.rsplit("_", 1)[0], int(re.sub(r"\D", "", p.name) or 0))):
            try:
                data = json.loads(f.read_text())
            except (OSError, ValueError):
                continue
            row = {"file": str(f.relative_to(d)), **flatten(data)}
            rows.append(row)
            cols += [c for c in row if c not in cols]
        if not rows:
            continue
        out = d / table
        lines = ["\t".join(cols)] + ["\t".join(str(r.get(c, "")) for c in cols) for r in rows]
        gone = [f for f in files if f.resolve() not in keep]
        print(f"{d.relative_to(ROOT)}: {len(rows)} runs -> {table}, removing {len(gone)}")
        if a.dry_run:
            continue
        if out.exists():
            out = d / out.name.replace(".tsv", "_folded.tsv")
        out.write_text("\n".join(lines) + "\n")
        for f in gone:
            f.unlink()
            removed += 1
    for rnd in filter(None, a.merge_sessions.split(",")):
        for sess in sorted(p for p in (PROFILES / rnd).iterdir() if p.is_dir()):
            members = [f for f in tracked(sess) if f.exists() and f.resolve() not in keep and f.name != "README.md"
                       and f.suffix in (".txt", ".tsv", ".json", ".jsonl", ".log", ".md") and f.name != "session.txt"]
            if len(members) < 2:
                continue
            print(f"{sess.relative_to(ROOT)}: {len(members)} files -> session.txt")
            if a.dry_run:
                continue
            with open(sess / "session.txt", "a") as w:
                for f in sorted(members):
                    w.write(f"===== {f.relative_to(sess)} =====\n")
                    w.write(f.read_text(errors="replace"))
                    w.write("\n")
                    f.unlink()
                    removed += 1
    print(f"removed {removed} files")
    return 0


if __name__ == "__main__":
    sys.exit(main())
