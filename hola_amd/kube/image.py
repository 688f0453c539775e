"""The container image, without a container runtime: `deploy/Dockerfile` read as data.

The final stage's ENV, WORKDIR, EXPOSE and ENTRYPOINT become the pod's defaults, and each
COPY becomes a file of the image's root filesystem, materialised as a symlink to what the
build produced (`COPY --from=build /src/build/hola /app/hola` is this repo's
`build/release/hola`; plain COPYs are repo files). A container path then resolves through
the pod's volume mounts first and the image root second, the way the container would see
it (`/root/reference/Dockerfile:1-10` is the contract being replayed: env, port, jar path).
"""
from __future__ import annotations

import json
import os
import shlex
from dataclasses import dataclass, field
from pathlib import Path

from hola_amd import native

REPO = native.REPO


@dataclass
class Image:
    name: str = "redhatmsa/hola:0.0.1-SNAPSHOT"
    entrypoint: list[str] = field(default_factory=list)
    cmd: list[str] = field(default_factory=list)
    env: dict[str, str] = field(default_factory=dict)
    workdir: str = "/"
    exposed: list[int] = field(default_factory=list)
    files: dict[str, Path] = field(default_factory=dict)  # container path -> host path

    @classmethod
    def from_dockerfile(cls, path: str | Path = REPO / "deploy" / "Dockerfile", preset: str = "release") -> "Image":
        lines = _logical_lines(Path(path).read_text())
        stages: list[list[tuple[str, str]]] = []
        for ins, arg in lines:
            if ins == "FROM":
                stages.append([])
            if stages:
                stages[-1].append((ins, arg))
        img = cls()
        if not stages:
            return img
        build_dir = native.build_dir(preset)
        for ins, arg in stages[-1]:
            if ins == "ENV":
                img.env.update(_parse_env(arg))
            elif ins == "WORKDIR":
                img.workdir = arg.strip()
            elif ins == "EXPOSE":
                img.exposed += [int(p.split("/")[0]) for p in arg.split()]
            elif ins == "ENTRYPOINT":
                img.entrypoint = _exec_form(arg)
            elif ins == "CMD":
                img.cmd = _exec_form(arg)
            elif ins in ("COPY", "ADD"):
                toks = shlex.split(arg)
                frm = next((t.split("=", 1)[1] for t in toks if t.startswith("--from=")), None)
                toks = [t for t in toks if not t.startswith("--")]
                *srcs, dst = toks
                for src in srcs:
                    if frm:  # the build stage's WORKDIR /src; its cmake tree is build/<preset>
                        rel = os.path.relpath(src, "/src")
                        host = build_dir / rel[len("build/"):] if rel.startswith("build/") else REPO / rel
                    else:
                        host = REPO / src
                    target = dst if not dst.endswith("/") else dst + Path(src).name
                    if host == build_dir / "hola" and os.environ.get("HOLA_SERVER_BIN"):
                        host = native.binary("hola")  # another server build (A/B runs, old trees)
                    img.files[os.path.normpath(target)] = host
        return img

    def materialize(self, root: Path) -> Path:
        """Lays the image's files out under `root` (symlinks to the host files)."""
        for cpath, host in self.files.items():
            dst = root / cpath.lstrip("/")
            dst.parent.mkdir(parents=True, exist_ok=True)
            if dst.is_symlink() or dst.exists():
                dst.unlink()
            dst.symlink_to(host)
        return root


def _logical_lines(text: str) -> list[tuple[str, str]]:
    out, cur = [], ""
    for raw in text.splitlines():
        line = raw.rstrip()
        if not cur and (not line.strip() or line.lstrip().startswith("#")):
            continue
        if line.endswith("\\"):
            cur += line[:-1] + " "
            continue
        cur += line
        ins, _, arg = cur.strip().partition(" ")
        out.append((ins.upper(), arg.strip()))
        cur = ""
    return out


def _exec_form(arg: str) -> list[str]:
    arg = arg.strip()
    if arg.startswith("["):
        return list(json.loads(arg))
    return ["/bin/sh", "-c", arg]


def _parse_env(arg: str) -> dict[str, str]:
    toks = shlex.split(arg)
    if toks and "=" not in toks[0]:  # legacy `ENV key value`
        return {toks[0]: " ".join(toks[1:])}
    return dict(t.split("=", 1) for t in toks)
