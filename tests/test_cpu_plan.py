"""Core planning for replicas and load generators (hola_amd/utils/cpu.py) on a mocked
2-socket EPYC topology: 8-core L3 domains, SMT siblings at +128, 16-CPU cgroup quota."""
import pytest

from hola_amd.utils import cpu


@pytest.fixture
def epyc(monkeypatch):
    cpus = list(range(256))
    monkeypatch.setattr(cpu, "allowed_cpus", lambda: cpus)
    monkeypatch.setattr(cpu, "cgroup_cpu_quota", lambda: 16.0)
    monkeypatch.setattr(cpu, "physical_cores", lambda cpus=None: list(range(128)))
    monkeypatch.setattr(cpu, "l3_domain", lambda c: (c % 128) // 8)
    monkeypatch.setattr(cpu, "siblings", lambda c: [c % 128, c % 128 + 128])
    busy = {c: 0.0 for c in cpus}
    monkeypatch.setattr(cpu, "cpu_busy", lambda interval=0.3: busy)
    return busy


def test_parse_format_roundtrip():
    assert cpu.parse_cpu_list("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert cpu.format_cpu_list([11, 0, 1, 2, 3, 8, 10]) == "0-3,8,10-11"


def test_budget_from_quota(epyc):
    assert cpu.cpu_budget() == 16


def test_plan_node_disjoint_whole_domains(epyc):
    plans = cpu.plan_node(2)
    assert [len(p) for p in plans] == [8, 8]
    assert not set(plans[0]) & set(plans[1])
    for p in plans:
        assert len({cpu.l3_domain(c) for c in p}) == 1  # a rank fits one L3 domain


def test_plan_node_avoids_busy_domains(epyc):
    for c in range(0, 8):
        epyc[c] = 1.0  # another tenant saturates domain 0
    plans = cpu.plan_node(1)
    assert all(cpu.l3_domain(c) != 0 for c in plans[0])


def test_split_pairs_server_and_loadgen_per_domain(epyc):
    cores = list(range(0, 16))  # domains 0 and 1
    srv, lg = cpu.split_server_loadgen(cores, 8)
    assert len(srv) == len(lg) == 8 and not set(srv) & set(lg)
    assert [cpu.l3_domain(c) for c in srv] == [cpu.l3_domain(c) for c in lg]


def test_cross_rank_loadgen_sits_with_target_replica(epyc):
    plans = cpu.plan_replicas_with_loadgen(2, per_rank=16)  # pretend 32 CPUs
    n = 2
    for r, p in enumerate(plans):
        for t, c in enumerate(p["loadgen"]):
            target = (t + r) % n
            assert cpu.l3_domain(c) in {cpu.l3_domain(x) for x in plans[target]["server"]}
    used = [c for p in plans for c in p["server"] + p["loadgen"]]
    assert len(used) == len(set(used)) == 32


def test_scaling_plan_places_threads_with_replicas(epyc, monkeypatch):
    from hola_amd.parallel import scaling

    p = scaling.plan(4, 16, 0.5, 0)
    assert len(p["replicas"]) == 4
    for t, c in enumerate(p["loadgen"]):
        assert cpu.l3_domain(c) in {cpu.l3_domain(x) for x in p["replicas"][t % 4]}


def test_plan_mirrored_every_domain_holds_every_process(epyc):
    plan = cpu.plan_mirrored({"A": 2, "B": 1, "loadgen": 1})  # 16 cores = 2 domains
    assert sorted(len(v) for v in plan.values()) == [4, 4, 8]
    assert len(plan["A"]) == 8
    every = [c for v in plan.values() for c in v]
    assert len(every) == len(set(every)) == 16
    for name, cores in plan.items():
        assert {cpu.l3_domain(c) for c in cores} == {0, 1}, name  # a share in both L3s


def test_plan_mirrored_small_budget_still_gives_each_a_core(epyc):
    plan = cpu.plan_mirrored({"A": 2, "B": 1, "loadgen": 1}, total=3)
    assert all(len(v) >= 1 for v in plan.values())
    assert len({c for v in plan.values() for c in v}) == 3


def test_full_node_eight_ranks(epyc, monkeypatch):
    """The driver's N=8 run on a whole node (no quota: 256 CPUs, 128 physical cores in 16 L3
    domains): 16 cores per rank, disjoint, no SMT siblings, every load-generator thread in
    the L3 of the replica it drives. Planning only; nothing is launched."""
    monkeypatch.setattr(cpu, "cgroup_cpu_quota", lambda: 0.0)
    n = 8
    per_rank = min(16, cpu.cpu_budget() // n)
    assert per_rank == 16
    plans = cpu.plan_replicas_with_loadgen(n, per_rank)
    used = [c for p in plans for c in p["server"] + p["loadgen"]]
    assert len(used) == len(set(used)) == 128 and max(used) < 128  # physical cores only
    for r, p in enumerate(plans):
        assert len(p["server"]) == 8 and len(p["loadgen"]) == 8
        for t, c in enumerate(p["loadgen"]):
            target = (t + r) % n
            assert cpu.l3_domain(c) in {cpu.l3_domain(x) for x in plans[target]["server"]}


def test_smt_pair_puts_each_loadgen_thread_on_its_workers_sibling(epyc, monkeypatch):
    """--smt pair: rank r's load-generator thread t runs on the SMT sibling of one server
    core of the replica it drives, and every sibling is used once across the node."""
    monkeypatch.setattr(cpu, "cgroup_cpu_quota", lambda: 0.0)
    n = 8
    assert cpu.smt_fits(n, 16)
    plans = cpu.plan_replicas_with_loadgen(n, 16, smt="pair")
    used = [c for p in plans for c in p["server"] + p["loadgen"]]
    assert len(used) == len(set(used)) == 256
    for r, p in enumerate(plans):
        assert len(p["server"]) == 16 and len(p["loadgen"]) == 16
        assert max(p["server"]) < 128
        for t, c in enumerate(p["loadgen"]):
            target = (t + r) % n
            assert c % 128 in plans[target]["server"]  # sibling of one of the target's cores


def test_smt_split_doubles_threads_on_the_same_cores(epyc):
    plans = cpu.plan_replicas_with_loadgen(1, 8, smt="split")
    p = plans[0]
    assert len(p["server"]) == 8 and len(p["loadgen"]) == 8
    assert {c % 128 for c in p["server"]}.isdisjoint({c % 128 for c in p["loadgen"]})
    assert not cpu.smt_fits(1, 16)  # the 16-CPU quota cannot run 32 threads


def test_smt_pair_single_rank_under_quota(epyc):
    p = cpu.plan_replicas_with_loadgen(1, 8, smt="pair")[0]
    assert [c + 128 for c in p["server"]] == p["loadgen"]
    assert cpu.smt_fits(1, 8)


def test_smt_auto_is_decided_per_node(epyc, monkeypatch):
    """bench.py --smt auto asks whether one GPU slot's CPU share holds both SMT threads of
    its 16 cores: yes on an unconstrained 256-CPU 8-GPU node, no under a 128-CPU quota or
    the 1-GPU box's 16-CPU quota, whatever the number of ranks N in this run."""
    assert not cpu.smt_fits(1, 16)  # 1-GPU box: quota 16
    monkeypatch.setattr(cpu, "cgroup_cpu_quota", lambda: 128.0)
    assert not cpu.smt_fits(8, 16)
    monkeypatch.setattr(cpu, "cgroup_cpu_quota", lambda: 0.0)
    assert cpu.smt_fits(8, 16)
    monkeypatch.setattr(cpu, "physical_cores", lambda cpus=None: list(range(64)))
    assert not cpu.smt_fits(8, 16)  # not enough physical cores for 8 x 16


def test_slot_cores_per_node(epyc, monkeypatch):
    """bench.py's default cores per replica: one GPU slot's share of the node."""
    assert cpu.slot_cores(1) == 16  # 1-GPU box: 16-CPU quota
    monkeypatch.setattr(cpu, "cgroup_cpu_quota", lambda: 0.0)
    assert cpu.slot_cores(8) == 16  # 2 x 64 cores, 8 GPUs
    assert cpu.smt_fits(8, cpu.slot_cores(8))
    monkeypatch.setattr(cpu, "allowed_cpus", lambda: list(range(384)))
    monkeypatch.setattr(cpu, "physical_cores", lambda cpus=None: list(range(192)))
    assert cpu.slot_cores(8) == 24  # 2 x 96 cores


def test_fewer_loadgen_threads_than_replicas_stay_in_l3(epyc):
    """The 16-CPU rehearsal at N = 4: 4 cores per rank, 2 server workers + 2 load-generator
    threads, so T = 2 < N = 4. Each thread drives one L3 group of replicas from a CPU in
    that group's L3, and every replica still gets the same connections from every rank."""
    n = 4
    plans = cpu.plan_replicas_with_loadgen(n, 4)
    used = [c for p in plans for c in p["server"] + p["loadgen"]]
    assert len(used) == len(set(used)) == 16
    per_replica = [0] * n
    for r, p in enumerate(plans):
        assert p["thread_targets"] is not None and len(p["thread_targets"]) == len(p["loadgen"]) == 2
        for t, c in enumerate(p["loadgen"]):
            for target in p["thread_targets"][t]:
                assert cpu.l3_domain(c) in {cpu.l3_domain(x) for x in plans[target]["server"]}
        conns = cpu.connection_targets(p["thread_targets"], 64)
        for x in conns:
            per_replica[x] += 1
        assert sorted(set(conns)) == list(range(n)) and all(conns.count(x) == 16 for x in range(n))
    assert per_replica == [64] * n


def test_aligned_thread_targets_match_the_dealing(epyc):
    plans = cpu.plan_replicas_with_loadgen(2, per_rank=16)
    for r, p in enumerate(plans):
        assert p["thread_targets"] == [[(t + r) % 2] for t in range(len(p["loadgen"]))]


def test_one_thread_per_rank_drives_same_l3_replicas(epyc):
    """N = 8 in a 16-CPU slice: 1 server worker + 1 load-generator thread per rank, 4 ranks
    per L3. One thread cannot reach all 8 replicas inside its L3, so each drives the 4
    replicas of its own L3; every replica still gets 64 connections in total."""
    n = 8
    plans = cpu.plan_replicas_with_loadgen(n, 2)
    per_replica = [0] * n
    for r, p in enumerate(plans):
        (c,) = p["loadgen"]
        (targets,) = p["thread_targets"]
        assert len(targets) == 4
        for m in targets:
            assert cpu.l3_domain(c) == cpu.l3_domain(plans[m]["server"][0])
        for x in cpu.connection_targets(p["thread_targets"], 64):
            per_replica[x] += 1
    assert per_replica == [64] * n


def test_a_rank_stays_in_one_socket_when_l3_ids_alternate(epyc, monkeypatch):
    """The 2-socket box numbers its L3 domains alternately across the sockets, so taking
    domains in id order gave a 16-core rank one CCD on each socket (found by the box's
    8-slot plan test). The planner now fills socket by socket."""
    monkeypatch.setattr(cpu, "cgroup_cpu_quota", lambda: 0.0)
    monkeypatch.setattr(cpu, "package_of", lambda c: ((c % 128) // 8) % 2)
    plans = cpu.plan_replicas_with_loadgen(8, 16, smt="pair")
    for p in plans:
        assert len({cpu.package_of(c) for c in p["server"]}) == 1, p["server"]
    servers = [c for p in plans for c in p["server"]]
    assert len(servers) == len(set(servers)) == 128
    # quietest socket first: a busy socket 0 moves a single rank to socket 1
    for c in range(256):
        epyc[c] = 1.0 if cpu.package_of(c) == 0 else 0.0
    one = cpu.plan_node(1, 16)[0]
    assert {cpu.package_of(c) for c in one} == {1}


def test_slot_subset_mirrors_the_node_plan(epyc, monkeypatch):
    """--slot-cores K: replica r takes the first K physical cores of node slot r, so the
    miniature's slots sit where the 8-slot node plan puts them (both sockets), each server
    worker with its load-generator thread on the other SMT thread of its core."""
    monkeypatch.setattr(cpu, "package_of", lambda c: (c % 128) // 64)
    node = cpu.plan_node(8, 16, avoid_busy=False)
    for n in (1, 2, 4, 8):
        sub = cpu.plan_slot_subset(n, 8, 1, smt="pair")
        assert len(sub) == n
        for r, p in enumerate(sub):
            assert p["server"] == node[r][:1] and p["slot"] == r
            assert p["loadgen"] == [p["server"][0] + 128]  # the sibling of the server core
    sockets = {cpu.package_of(p["server"][0]) for p in cpu.plan_slot_subset(8, 8, 1)}
    assert sockets == {0, 1}
    off = cpu.plan_slot_subset(2, 8, 2, smt="off", extra_cores=1)
    for r, p in enumerate(off):
        assert p["server"] == node[r][:2] and p["loadgen"] == node[r][2:4] and p["extra"] == node[r][4:5]
    with pytest.raises(ValueError):
        cpu.plan_slot_subset(1, 8, 16, smt="off")  # 32 cores do not fit a 16-core slot


def test_host_load_siblings_exclude_the_job(epyc):
    """host_load.siblings counts only SMT siblings that no part of the job planned: in pair
    mode a rank's siblings are other ranks' load-generator threads, not another tenant."""
    from hola_amd.parallel import subruns

    own = [0, 1]
    assert subruns.other_siblings(own, []) == {128, 129}
    assert subruns.other_siblings(own, [128]) == {129}
    assert subruns.other_siblings(own, [128, 129, 5]) == set()
