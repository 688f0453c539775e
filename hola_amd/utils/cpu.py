"""Host CPU topology, cgroup quota and per-replica core planning.

On the MI355X node the service runs on the EPYC host cores (2 sockets x 64 cores, SMT2 on
the box probed for this build). A gpurun box is a CFS-quota slice of that host (cpu.max
"1600000 100000" = 16 CPUs) with the full 256-CPU affinity mask, so plans are sized from
the quota and laid out on distinct *physical* cores (one SMT sibling each), NUMA node by
NUMA node, so replica i and replica j never share a core or an L2.
"""
from __future__ import annotations

import os
from pathlib import Path


def parse_cpu_list(s: str) -> list[int]:
    out: list[int] = []
    for tok in s.split(","):
        tok = tok.strip()
        if not tok:
            continue
        if "-" in tok:
            a, b = tok.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(tok))
    return out


def format_cpu_list(cpus: list[int]) -> str:
    cpus = sorted(cpus)
    parts = []
    i = 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        parts.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(parts)


def allowed_cpus() -> list[int]:
    return sorted(os.sched_getaffinity(0))


def cgroup_cpu_quota() -> float:
    """CPUs granted by cgroup v2 cpu.max; 0.0 when unlimited or unknown."""
    try:
        q, p = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q == "max":
            return 0.0
        return float(q) / float(p)
    except (OSError, ValueError):
        return 0.0


def cpu_budget() -> int:
    """Number of CPUs this process tree may keep busy. HOLA_IGNORE_QUOTA=1 plans as if the
    cgroup quota were absent (layout rehearsals of an unconstrained node on a quota'd box)."""
    n = len(allowed_cpus())
    q = cgroup_cpu_quota()
    if q > 0 and os.environ.get("HOLA_IGNORE_QUOTA") != "1":
        n = min(n, int(q))
    return max(1, n)


def _read(path: str) -> str | None:
    try:
        return Path(path).read_text().strip()
    except OSError:
        return None


def physical_cores(cpus: list[int] | None = None) -> list[int]:
    """One CPU per physical core (the lowest SMT sibling), ordered by NUMA node then id."""
    cpus = allowed_cpus() if cpus is None else cpus
    allowed = set(cpus)
    seen: set[tuple[str, str]] = set()
    picked: list[tuple[int, int]] = []
    for c in cpus:
        base = f"/sys/devices/system/cpu/cpu{c}/topology"
        sib = _read(f"{base}/thread_siblings_list") or _read(f"{base}/core_cpus_list")
        pkg = _read(f"{base}/physical_package_id") or "0"
        if sib is None:
            picked.append((0, c))
            continue
        key = (pkg, sib)
        if key in seen:
            continue
        seen.add(key)
        first = min(x for x in parse_cpu_list(sib) if x in allowed) if any(
            x in allowed for x in parse_cpu_list(sib)) else c
        node = 0
        for n in range(0, 16):
            if Path(f"/sys/devices/system/cpu/cpu{first}/node{n}").exists():
                node = n
                break
        picked.append((node, first))
    picked.sort()
    return [c for _, c in picked]


def l3_domain(cpu: int) -> int:
    """Id of the L3 (CCD on EPYC) a CPU belongs to; 0 when unknown."""
    v = _read(f"/sys/devices/system/cpu/cpu{cpu}/cache/index3/id")
    try:
        return int(v) if v is not None else 0
    except ValueError:
        return 0


def package_of(cpu: int) -> int:
    """Physical package (socket) of a CPU; 0 when unknown."""
    v = _read(f"/sys/devices/system/cpu/cpu{cpu}/topology/physical_package_id")
    try:
        return int(v) if v is not None else 0
    except ValueError:
        return 0


def online_cpus() -> list[int]:
    """Every online CPU of the host (not only this process's affinity mask)."""
    v = _read("/sys/devices/system/cpu/online")
    return parse_cpu_list(v) if v else allowed_cpus()


def siblings(cpu: int) -> list[int]:
    v = _read(f"/sys/devices/system/cpu/cpu{cpu}/topology/thread_siblings_list")
    return parse_cpu_list(v) if v else [cpu]


def cpu_busy(interval: float = 0.3) -> dict[int, float]:
    """Host-wide per-CPU busy fraction over `interval` seconds (from /proc/stat)."""
    import time

    def snap():
        d = {}
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("cpu") and line[3].isdigit():
                    parts = line.split()
                    v = list(map(int, parts[1:]))
                    d[int(parts[0][3:])] = (sum(v), v[3] + v[4])
        return d

    a = snap()
    time.sleep(interval)
    b = snap()
    return {c: 1.0 - (b[c][1] - a[c][1]) / max(1, b[c][0] - a[c][0]) for c in a if c in b}


def plan_node(local_world: int, per_rank: int | None = None, avoid_busy: bool = True) -> list[list[int]]:
    """Disjoint core lists for every co-located rank, L3-domain (CCD) aware.

    Physical cores are grouped by L3 domain; with ``avoid_busy`` the quietest domains (by
    host-wide /proc/stat load, which on a shared box includes other tenants) are used first.
    Each rank gets whole domains where possible so its server and load generator share an L3.
    Compute once (rank 0) and broadcast: measurements differ between processes.
    """
    budget = cpu_budget()
    if per_rank is None:
        per_rank = max(1, budget // max(1, local_world))
    phys = physical_cores()
    if len(phys) < per_rank * local_world:
        phys = allowed_cpus()
        per_rank = max(1, min(per_rank, len(phys) // max(1, local_world)))
    # 1 s of /proc/stat: other tenants' load on a shared host comes in bursts, and a short
    # sample can rank a busy L3 domain as quiet
    busy = cpu_busy(1.0) if avoid_busy else {}
    load = {c: sum(busy.get(x, 0.0) for x in siblings(c)) for c in phys}
    domains: dict[int, list[int]] = {}
    for c in phys:
        domains.setdefault(l3_domain(c), []).append(c)
    # Ranks take consecutive slices of the pool, so the pool runs socket by socket: a rank's
    # L3 domains then share a socket whenever its slice fits in one (L3 ids alternate between
    # the sockets on the 2-socket EPYC node, so id order alone spread a 2-domain rank over
    # both). Quietest socket first; inside it quietest domains first; inside a domain quietest
    # cores first (each stable by id).
    def dom_load(d: int) -> float:
        return round(sum(load[c] for c in domains[d]) / len(domains[d]), 1)
    sockets: dict[int, list[int]] = {}
    for d in domains:
        sockets.setdefault(package_of(domains[d][0]), []).append(d)
    sock_order = sorted(sockets, key=lambda k: (round(sum(dom_load(d) for d in sockets[k]) / len(sockets[k]), 1), k))
    order = [d for k in sock_order for d in sorted(sockets[k], key=lambda d: (dom_load(d), d))]
    pool = []
    for d in order:
        pool.extend(sorted(domains[d], key=lambda c: (round(load[c], 1), c)))
    return [pool[r * per_rank:(r + 1) * per_rank] for r in range(local_world)]


def split_server_loadgen(cores: list[int], server_threads: int) -> tuple[list[int], list[int]]:
    """Splits a rank's cores so that server worker t and load-generator thread t sit in the
    same L3 domain (connections are dealt round-robin on both sides, so connection i joins
    loadgen thread i%L to server worker i%S: with S == L each pair talks through one L3)."""
    by_dom: dict[int, list[int]] = {}
    for c in cores:
        by_dom.setdefault(l3_domain(c), []).append(c)
    server, load = [], []
    for dom_cores in by_dom.values():
        for i, c in enumerate(dom_cores):
            (server if i % 2 == 0 else load).append(c)
    # honour the requested server share
    while len(server) > server_threads and len(server) > 1:
        load.append(server.pop())
    while len(server) < server_threads and len(load) > 1:
        server.append(load.pop())
    # interleave so index t of each list is in the same domain whenever possible
    server.sort(key=lambda c: (l3_domain(c), c))
    load.sort(key=lambda c: (l3_domain(c), c))
    return server, load


def slot_cores(gpu_slots: int) -> int:
    """Physical cores per GPU slot: the node's usable physical cores (CPU budget or physical
    core count, whichever is smaller) divided by its GPUs. 16 on the 16-CPU gpurun box and on
    a 2 x 64-core 8-GPU node; it grows with bigger hosts."""
    return max(1, min(cpu_budget(), len(physical_cores())) // max(1, gpu_slots))


def sibling_of(cpu: int) -> int | None:
    """The other SMT thread of `cpu`'s physical core, if it exists and is allowed."""
    allowed = set(allowed_cpus())
    for s in siblings(cpu):
        if s != cpu and s in allowed:
            return s
    return None


def smt_fits(local_world: int, per_rank: int) -> bool:
    """True when both SMT threads of every planned physical core can run without the CPU
    budget (cgroup quota) throttling them: the budget covers 2 x per_rank x local_world."""
    need = per_rank * local_world
    phys = physical_cores()
    return (cpu_budget() >= 2 * need and len(phys) >= need
            and all(sibling_of(c) is not None for c in phys[:need]))


def plan_replicas_with_loadgen(local_world: int, per_rank: int | None = None, server_threads: int = 0,
                               avoid_busy: bool = True, smt: str = "off") -> list[dict]:
    """Core plan for `local_world` co-located (replica + load generator) ranks with
    client-side round-robin over all replicas.

    Connection i of a rank's load generator runs on thread t = i % T. Each thread drives only
    the replicas in ``thread_targets[t]``, and its CPU is taken from *those* replicas' L3
    domains, so every connection's client and server ends share an L3 even though traffic
    crosses ranks:
      * T % N == 0: thread t of rank r drives replica (t + r) % N alone;
      * N % T == 0 (fewer threads than replicas, e.g. 2 threads and 4 replicas on a 16-CPU
        slice) and each group of N/T consecutive ranks sits in one L3: thread t of rank r
        drives group (t + r) % T;
      * otherwise each thread stays on its own rank's cores and drives the replicas whose
        servers share its L3 (topology-aware round-robin: every replica still gets the same
        number of connections in aggregate, but a rank no longer reaches every replica);
        ``thread_targets`` is None (plain (i + r) % N dealing) only when no such replica
        exists.
    In the first two cases every replica receives the same number of connections from every
    rank (client-side round-robin). Returns, per rank, {"server": [...], "loadgen": [... one CPU
    per thread, in thread order], "thread_targets": [[replica, ...] per thread] or None}.

    `smt` decides what happens to the SMT sibling of each planned physical core:
      * "off"   - left idle (one thread per physical core);
      * "split" - the sibling joins the same side, so server and load generator each get
                  twice the threads on the same physical cores;
      * "pair"  - every physical core runs one server worker and, on its sibling, the
                  load-generator thread that drives it (the server steers a connection to
                  the worker on the client's own core: both socket buffers share L1/L2).
    """
    nodes = plan_node(local_world, per_rank, avoid_busy=avoid_busy)
    splits = []
    for cores in nodes:
        if smt == "pair":
            sib = [sibling_of(c) for c in cores]
            if all(x is not None for x in sib):
                splits.append((list(cores), sib))
                continue
        if len(cores) > 1:
            st = server_threads or max(1, len(cores) // 2)
            st = min(st, len(cores) - 1)
            sv, ld = split_server_loadgen(cores, st)
        else:
            sv, ld = cores, cores
        if smt == "split":
            sv = sv + [x for x in map(sibling_of, sv) if x is not None]
            ld = ld + [x for x in map(sibling_of, ld) if x is not None]
        splits.append((sv, ld))
    n = local_world
    t_threads = len(splits[0][1])
    uniform = all(len(sp[1]) == t_threads for sp in splits)
    plans = []
    for r in range(n):
        targets = None
        dealing = "round-robin over all replicas, each thread on the L3 of the replica it drives"
        if n == 1:
            load = splits[0][1]
            targets = [[0] for _ in load]
        elif uniform and t_threads % n == 0:
            per = t_threads // n
            load = [splits[(t + r) % n][1][r * per + t // n] for t in range(t_threads)]
            targets = [[(t + r) % n] for t in range(t_threads)]
        elif uniform and n % t_threads == 0 and _groups_share_l3(splits, n // t_threads):
            per = n // t_threads  # replicas per group
            load, targets = [], []
            for t in range(t_threads):
                g = (t + r) % t_threads
                members = [g * per + j for j in range(per)]
                pool = [c for m in members for c in splits[m][1]]  # per * T CPUs, one per rank
                load.append(pool[r])
                targets.append([members[(j + r) % per] for j in range(per)])
            dealing = "round-robin over all replicas, each thread on the L3 of the replica group it drives"
        else:
            load = splits[r][1]
            dealing = "topology-aware round-robin over the replicas in each thread's L3"
            targets = []
            for c in load:
                local = [m for m in range(n) if l3_domain(c) in {l3_domain(x) for x in splits[m][0]}]
                targets.append([local[(j + r) % len(local)] for j in range(len(local))] if local else None)
            if any(x is None for x in targets):
                targets = None
                dealing = "round-robin over all replicas from the rank's own cores"
        plans.append({"server": splits[r][0], "loadgen": load, "thread_targets": targets, "dealing": dealing})
    return plans


def plan_slot_subset(n: int, slots: int, k: int, smt: str = "pair", extra_cores: int = 0) -> list[dict]:
    """A miniature of the node plan for weak-scaling curves inside a small CPU quota.

    The node is laid out as `slots` slots of (physical cores / slots) cores each, exactly as
    plan_node places them on the real topology (socket by socket, L3 domain by domain; the
    quota is ignored for the layout), and replica r takes only the first `k` physical cores of
    slot r: with smt=pair its server workers run on one SMT thread of each and the
    load-generator thread that drives it on the other (the node plan's per-connection
    placement), with smt=off the next `k` cores of the slot carry the load generator.
    `extra_cores` more physical cores of the same slot are returned as "extra" (e.g. proxy
    threads); smt=auto is pair when the cores have SMT siblings, else off. Per replica:
    {"server", "loadgen", "extra", "slot", "smt"}."""
    phys = physical_cores()
    per = max(1, len(phys) // max(1, slots))
    if smt == "auto":  # pair where every core has an SMT sibling (not in a container without SMT)
        smt = "pair" if all(sibling_of(c) is not None for c in phys) else "off"
    need = k * (1 if smt == "pair" else 2) + extra_cores
    if per < need:
        raise ValueError(f"a slot has {per} physical cores, {need} needed")
    node = plan_node(slots, per, avoid_busy=False)
    out = []
    for r in range(n):
        cores = node[r % slots]
        srv = cores[:k]
        if smt == "pair":
            ld = [sibling_of(c) for c in srv]
            if any(c is None for c in ld):
                raise ValueError("smt=pair needs both SMT threads of every server core")
            rest = cores[k:]
        else:
            ld, rest = cores[k:2 * k], cores[2 * k:]
        out.append({"server": list(srv), "loadgen": list(ld), "extra": list(rest[:extra_cores]), "slot": r % slots,
                    "smt": smt})
    return out


def _groups_share_l3(splits: list[tuple[list[int], list[int]]], per: int) -> bool:
    """True when every group of `per` consecutive replicas has its servers and load-generator
    CPUs in one L3 domain."""
    for g in range(0, len(splits), per):
        doms = {l3_domain(c) for sv, ld in splits[g:g + per] for c in sv + ld}
        if len(doms) != 1:
            return False
    return True


def connection_targets(thread_targets: list[list[int]], connections: int) -> list[int]:
    """Target replica of each connection (connection i runs on thread i % T)."""
    t_threads = len(thread_targets)
    return [thread_targets[i % t_threads][(i // t_threads) % len(thread_targets[i % t_threads])]
            for i in range(connections)]


def plan_mirrored(weights: dict[str, int], total: int | None = None, avoid_busy: bool = True) -> dict[str, list[int]]:
    """Splits `total` cores (quietest L3 domains first) between several processes so that
    EVERY L3 domain holds a share of each, in proportion to `weights`.

    For a chain of processes (load generator -> hola A -> hola B), accept steering
    (SO_INCOMING_CPU) then keeps each hop inside one L3: a connection lands on a worker in
    the domain of the thread that opened it. Returns {name: [cores...]}, each non-empty.
    """
    return split_mirrored(plan_node(1, total, avoid_busy=avoid_busy)[0], weights)


def split_mirrored(cores: list[int], weights: dict[str, int]) -> dict[str, list[int]]:
    """plan_mirrored's split of a given CPU set (e.g. the CPUs a bench rank already owns)."""
    names = list(weights)
    by_dom: dict[int, list[int]] = {}
    for c in cores:
        by_dom.setdefault(l3_domain(c), []).append(c)
    out: dict[str, list[int]] = {n: [] for n in names}
    wsum = sum(weights.values())
    for dom_cores in by_dom.values():
        m = len(dom_cores)
        if m < len(names):  # too small to mirror: give it to the heaviest process
            out[max(names, key=lambda n: weights[n])].extend(dom_cores)
            continue
        shares = {n: max(1, round(m * weights[n] / wsum)) for n in names}
        while sum(shares.values()) > m:  # rounding overflow: trim the largest share
            shares[max(names, key=lambda n: shares[n])] -= 1
        while sum(shares.values()) < m:
            shares[max(names, key=lambda n: weights[n])] += 1
        i = 0
        for n in names:
            out[n].extend(dom_cores[i:i + shares[n]])
            i += shares[n]
    for n in names:  # a domain-starved process still needs one core
        if not out[n]:
            donor = max(names, key=lambda k: len(out[k]))
            out[n].append(out[donor].pop())
    return out


def plan_cores(rank: int, local_world: int, per_rank: int | None = None) -> list[int]:
    """Disjoint CPU set for `rank` out of `local_world` co-located ranks.

    Defaults to an equal share of the CPU budget, on distinct physical cores when enough
    exist (falls back to SMT siblings / any allowed CPU otherwise).
    """
    budget = cpu_budget()
    if per_rank is None:
        per_rank = max(1, budget // max(1, local_world))
    phys = physical_cores()
    pool = phys if len(phys) >= per_rank * local_world else allowed_cpus()
    if len(pool) < per_rank * local_world:
        per_rank = max(1, len(pool) // max(1, local_world))
    start = rank * per_rank
    return pool[start:start + per_rank] or pool[:per_rank]
