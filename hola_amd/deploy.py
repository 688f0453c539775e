"""Bare-metal deployment on one MI355X node: systemd units for N pinned replicas behind the
round-robin proxy — the node-local equivalent of the OpenShift Service + Deployment in
deploy/openshift/hola.yaml (replicas, LoadBalancer on :8080, readiness on /api/health).

    python -m hola_amd units --replicas 8 --out /etc/systemd/system [--prefix /opt/hola]

Each replica gets whole L3 domains (CPUAffinity= and --cpu-list agree) and is restarted by
systemd on failure (the platform restart policy). Two fronts:
* ``lb="proxy"`` (default): replicas listen on 127.0.0.1:<base+i>; `hola-rrproxy.service`
  fronts them on :8080 and health-checks /api/health.
* ``lb="reuseport"``: every replica binds :8080 itself with ``--accept reuseport``; the kernel
  spreads connections over the SO_REUSEPORT group (no proxy hop, no proxy unit). A replica
  that is down has no sockets in the group, so it gets no connections.
"""
from __future__ import annotations

from pathlib import Path

from hola_amd.utils.cpu import format_cpu_list, plan_node


def render_units(replicas: int, prefix: str = "/opt/hola", base_port: int = 18080, public_port: int = 8080,
                 proxy_threads: int = 4, cores_per_replica: int | None = None,
                 env_file: str = "/etc/hola/hola.env", lb: str = "proxy") -> dict[str, str]:
    if lb not in ("proxy", "reuseport"):
        raise ValueError(f"lb must be 'proxy' or 'reuseport', not {lb!r}")
    shared = lb == "reuseport"
    plan = plan_node(replicas + (0 if shared else 1), cores_per_replica, avoid_busy=False)
    units: dict[str, str] = {}
    backends = []
    for i in range(replicas):
        cpus = format_cpu_list(plan[i])
        port = public_port if shared else base_port + i
        listen = f"--port {port} --accept reuseport" if shared else f"--host 127.0.0.1 --port {port}"
        caps = "CAP_NET_BIND_SERVICE" if shared and public_port < 1024 else ""
        backends.append(f"127.0.0.1:{port}")
        units[f"hola-replica{i}.service"] = f"""[Unit]
Description=hola replica {i} (pinned to CPUs {cpus})
After=network-online.target
PartOf=hola.target

[Service]
Type=simple
EnvironmentFile=-{env_file}
Environment=HOSTNAME=%H-replica{i}
ExecStart={prefix}/hola {listen} --threads {len(plan[i])} --cpu-list {cpus} \\
    --hystrix-config {prefix}/conf/config.properties
CPUAffinity={cpus.replace(',', ' ')}
AmbientCapabilities={caps}
Restart=always
RestartSec=1
KillSignal=SIGTERM
TimeoutStopSec=15
LimitNOFILE=1048576
User=hola
NoNewPrivileges=true

[Install]
WantedBy=hola.target
"""
    if shared:
        units["hola.target"] = f"""[Unit]
Description=hola service ({replicas} replicas sharing :{public_port} via SO_REUSEPORT)
Wants={" ".join(sorted(u for u in units if u.endswith(".service")))}

[Install]
WantedBy=multi-user.target
"""
        return units
    proxy_cpus = format_cpu_list(plan[replicas][:proxy_threads])
    units["hola-rrproxy.service"] = f"""[Unit]
Description=hola round-robin front on :{public_port} ({replicas} replicas)
After=network-online.target
PartOf=hola.target

[Service]
Type=simple
ExecStart={prefix}/hola_rrproxy --port {public_port} --threads {proxy_threads} --cpu-list {proxy_cpus} \\
    --backends {",".join(backends)} --health-ms 500
CPUAffinity={proxy_cpus.replace(',', ' ')}
Restart=always
RestartSec=1
LimitNOFILE=1048576
User=hola
AmbientCapabilities={"CAP_NET_BIND_SERVICE" if public_port < 1024 else ""}

[Install]
WantedBy=hola.target
"""
    units["hola.target"] = f"""[Unit]
Description=hola service ({replicas} replicas + round-robin proxy)
Wants={" ".join(sorted(u for u in units if u.endswith(".service")))}

[Install]
WantedBy=multi-user.target
"""
    return units


def write_units(out: str | Path, **kw) -> list[Path]:
    out = Path(out)
    out.mkdir(parents=True, exist_ok=True)
    paths = []
    for name, text in render_units(**kw).items():
        p = out / name
        p.write_text(text)
        paths.append(p)
    return paths
