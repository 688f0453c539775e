"""Accept steering's balance rule (src/http/server.h Server::steering_within_share), driven
the way Server::pick_worker drives it: a steered connection goes to the next worker of its
client's L3 while the rule allows, otherwise to the least loaded worker.

These run on the CPU: the rule is a pure function of the live connection counts, so the
topology (which this container does not have: one L3) is simulated here."""
from __future__ import annotations

import pytest

from hola_amd.native import load_native


def simulate(domains: list[list[int]], n_workers: int, client_domains: list[int]) -> list[int]:
    """Connections accepted in order from clients in `client_domains` (an L3 id each);
    `domains[d]` = the workers pinned in L3 d. Returns live connections per worker."""
    n = load_native()
    counts = [0] * n_workers
    rr = 0
    domain_rr = [0] * len(domains)
    for d in client_domains:
        rr += 1  # the round-robin index advances on every accept (used when the CPU is unknown)
        ws = domains[d]
        cand = ws[domain_rr[d] % len(ws)]
        domain_rr[d] += 1
        # steered, or (refused for balance) the least loaded worker, the first of equals
        k = cand if n.steering_within_share(counts, cand) else counts.index(min(counts))
        counts[k] += 1
    return counts


def test_two_workers_in_two_l3s_fed_from_one_l3_both_serve():
    """with two workers the old bound (2 x fair share + 8) never refused, so every
    connection from one L3's clients went to that L3's worker and the other idled."""
    counts = simulate([[0], [1]], 2, [0] * 256)
    assert min(counts) > 0
    assert max(counts) <= 0.75 * 256 + 9, counts


def test_two_workers_fed_from_both_l3s_stay_fully_steered():
    counts = simulate([[0], [1]], 2, [0, 1] * 64)
    assert counts == [64, 64]


def test_one_worker_takes_everything():
    assert simulate([[0]], 1, [0] * 50) == [50]


@pytest.mark.parametrize("first", [0, 1])
def test_four_workers_keep_late_l3_steered(first):
    """Round 5's case (profiles/round5/02_chain_modes): the clients of one L3 open all theirs
    before those of the other; with four workers the late ones must still be served in their
    own L3 (twice the fair share + 8 lets the early L3's two workers take all of theirs)."""
    order = [first] * 64 + [1 - first] * 64
    counts = simulate([[0, 1], [2, 3]], 4, order)
    assert counts == [32, 32, 32, 32], counts


def test_three_workers_bound_by_twice_the_fair_share():
    counts = simulate([[0], [1, 2]], 3, [0] * 300)
    assert counts[0] <= 2 * 300 // 3 + 9, counts
    assert min(counts) > 0


def test_rule_rejects_bad_index():
    n = load_native()
    with pytest.raises(IndexError):
        n.steering_within_share([1, 2], 2)
