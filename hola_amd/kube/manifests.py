"""Kubernetes/OpenShift object handling for the local manifest executor.

Reads the objects of `deploy/openshift/*.yaml` (a `kind: List`, several YAML documents, or
one object), applies `oc patch`-style strategic-merge patches, and parses the resource
quantities the scheduler and the CPU manager need. Only what the reference's deploy
contract uses is modelled (`/root/reference/pom.xml:65-94`: Service, the generated
DeploymentConfig/Deployment with its env, readiness probe and ports; the demo's ConfigMap).
"""
from __future__ import annotations

import copy
import hashlib
import json
import math
from pathlib import Path

import yaml

SUPPORTED_KINDS = ("Service", "DeploymentConfig", "Deployment", "ConfigMap")

# Keys of list items that `kubectl patch --type strategic` merges by, per list name.
_MERGE_KEYS = {"containers": "name", "initContainers": "name", "env": "name", "volumes": "name",
               "volumeMounts": "mountPath", "ports": "containerPort", "items": "key"}


def load_objects(paths: list[str | Path]) -> list[dict]:
    """Every object in the files, `kind: List` expanded, in file order."""
    out: list[dict] = []
    for p in paths:
        for doc in yaml.safe_load_all(Path(p).read_text()):
            if not doc:
                continue
            if doc.get("kind") == "List":
                out.extend(i for i in doc.get("items") or [] if i)
            else:
                out.append(doc)
    return out


def strategic_merge(base, patch):
    """`kubectl patch --type strategic` for the shapes used here: maps merge key by key (a
    null value deletes), lists of maps with a known merge key merge item by item, every other
    list is replaced."""
    if isinstance(base, dict) and isinstance(patch, dict):
        out = copy.deepcopy(base)
        for k, v in patch.items():
            if v is None:
                out.pop(k, None)
            elif k in out and isinstance(v, list) and isinstance(out[k], list) and k in _MERGE_KEYS:
                out[k] = _merge_list(out[k], v, _MERGE_KEYS[k])
            elif k in out:
                out[k] = strategic_merge(out[k], v)
            else:
                out[k] = copy.deepcopy(v)
        return out
    return copy.deepcopy(patch)


def _merge_list(base: list, patch: list, key: str) -> list:
    out = [copy.deepcopy(x) for x in base]
    for item in patch:
        if not isinstance(item, dict) or key not in item:
            return copy.deepcopy(patch)
        for i, cur in enumerate(out):
            if isinstance(cur, dict) and cur.get(key) == item[key]:
                out[i] = strategic_merge(cur, item)
                break
        else:
            out.append(copy.deepcopy(item))
    return out


def set_env(template: dict, container: str | None, env: dict[str, str | None]) -> dict:
    """`oc set env` / `oc env`: sets (or, with None, removes) variables of one container (the
    first when `container` is None) in a pod template; returns the new template."""
    t = copy.deepcopy(template)
    cs = t["spec"]["containers"]
    c = next((x for x in cs if container is None or x.get("name") == container), None)
    if c is None:
        raise KeyError(f"no container {container!r}")
    cur = c.setdefault("env", [])
    for k, v in env.items():
        idx = next((i for i, e in enumerate(cur) if e.get("name") == k), None)
        if v is None:
            if idx is not None:
                cur.pop(idx)
        elif idx is None:
            cur.append({"name": k, "value": v})
        else:
            cur[idx] = {"name": k, "value": v}
    return t


def parse_cpu(q) -> float:
    """CPU quantity ('2', '500m', 1.5) in cores."""
    if q is None:
        return 0.0
    s = str(q).strip()
    if s.endswith("m"):
        return float(s[:-1]) / 1000.0
    return float(s)


_MEM = {"Ki": 1 << 10, "Mi": 1 << 20, "Gi": 1 << 30, "Ti": 1 << 40, "K": 10**3, "M": 10**6, "G": 10**9, "T": 10**12}


def parse_memory(q) -> int:
    """Memory quantity ('64Mi', '1G', 1024) in bytes."""
    if q is None:
        return 0
    s = str(q).strip()
    for suf in sorted(_MEM, key=len, reverse=True):
        if s.endswith(suf):
            return int(float(s[: -len(suf)]) * _MEM[suf])
    return int(float(s))


def resolve_int_or_percent(v, total: int, round_up: bool) -> int:
    """maxSurge / maxUnavailable: an int, or a percentage of `total` (surge rounds up,
    unavailable rounds down, as the deployment controllers do)."""
    if isinstance(v, str) and v.endswith("%"):
        x = float(v[:-1]) * total / 100.0
        return int(math.ceil(x) if round_up else math.floor(x))
    return int(v)


def qos_class(container: dict) -> str:
    """Guaranteed when every resource's request equals its limit (requests default to the
    limits); BestEffort with none; else Burstable."""
    res = container.get("resources") or {}
    lim, req = res.get("limits") or {}, res.get("requests") or {}
    if not lim and not req:
        return "BestEffort"
    req = {**lim, **req}

    def same(k):  # quantities compare by value: cpu "2" == 2 == "2000m", memory "1Gi" == "1024Mi"
        parse = parse_cpu if k == "cpu" else parse_memory if k == "memory" else str
        try:
            return parse(req.get(k)) == parse(lim.get(k))
        except (TypeError, ValueError):
            return str(req.get(k)) == str(lim.get(k))

    if lim and all(k in lim for k in ("cpu", "memory")) and all(same(k) for k in lim):
        return "Guaranteed"
    return "Burstable"


def template_hash(template: dict) -> str:
    """A stable 10-character hash of a pod template (the pod-template-hash label role)."""
    h = hashlib.sha256(json.dumps(template, sort_keys=True).encode()).hexdigest()
    alphabet = "bcdfghjklmnpqrstvwxz2456789"  # k8s SafeEncodeString alphabet
    n = int(h[:16], 16)
    out = []
    for _ in range(10):
        n, r = divmod(n, len(alphabet))
        out.append(alphabet[r])
    return "".join(out)


def selector_matches(selector: dict, labels: dict) -> bool:
    sel = selector.get("matchLabels", selector) if isinstance(selector, dict) else {}
    return all(labels.get(k) == v for k, v in sel.items() if isinstance(v, str))
