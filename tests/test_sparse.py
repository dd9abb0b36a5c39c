"""Sparse engine layout: list-only inbox (no per-edge slots),
launches over compact lists of active nodes, hub-compact link state for Paxos on
the full mesh.  Every parity case must give the same bit-exact result as the
oracle in this layout too; BASELINE configs[2] (Paxos n=4096, multi-decree,
jittered links, batched replicas) runs in it at full size."""
import pytest

import oracle
from bcsim import _abi
from parity_cases import cases, compare, topology

pytestmark = pytest.mark.gpu
CASES = cases()


@pytest.mark.parametrize("name", sorted(CASES))
def test_sparse_layout_matches_oracle(name, engine_lib):
    import bcsim
    cfg = CASES[name]
    cfg.engine_mode = _abi.ENGINE_SPARSE
    topo = topology(name)
    ref = oracle.run(cfg, topology=topo)
    got = bcsim.run(cfg, topology=topo)
    d = compare(ref, got)
    assert d is None, f"{name} (sparse): {d}"


@pytest.mark.timeout(300)
def test_c3_paxos4096_multidecree_dense_equals_sparse(engine_lib):
    """BASELINE configs[2] at n=4096 (multi-decree, jittered U{0..49} ms links, counter-RNG
    replicas): the dense and the sparse layout give identical traces and counters over
    the first 2 s, and the prefix invariants hold -- no response without its request,
    broadcasts reach N-2 peers plus one dropped *end() send, at most one commit per
    (replica, proposer, decree)."""
    import bcsim
    from collections import Counter
    n = 4096
    res = {}
    for mode in (_abi.ENGINE_DENSE, _abi.ENGINE_SPARSE):
        c = bcsim.preset("c3_paxos")
        c.n_replicas = 8
        c.paxos_decrees = 2
        c.seed = 5
        c.t_end_ns = 2_000_000_000
        c.engine_mode = mode
        tr, cnt, st = bcsim.run(c)
        assert st["error"] == 0
        res[mode] = (tr, cnt)
    assert compare(res[_abi.ENGINE_DENSE], res[_abi.ENGINE_SPARSE]) is None
    tr, cnt = res[_abi.ENGINE_SPARSE]
    d = cnt["delivered"]
    assert 0 < d[3] <= d[0] and d[4] <= d[1] and d[5] <= d[2]
    tickets = sum(1 for r in tr if r[6] == _abi.TR["PAXOS_TICKET"])
    assert d[0] <= (n - 2) * tickets
    commits = Counter((r[0], r[5], r[8]) for r in tr if r[6] == _abi.TR["PAXOS_COMMIT"])
    assert max(commits.values(), default=1) == 1


@pytest.mark.timeout(900)
def test_c3_paxos4096_10k_replicas_fit(engine_lib):
    """The configs[2] batch size itself: 10,000 replicas of Paxos n=4096 (41M nodes, two
    decrees per proposer) in one sparse engine on one GPU over the first 16 s simulated -- the
    horizon where the dueling proposers start to win (the oracle's single n=4096 replicas commit
    first at 13-15 s for seeds 1-3) -- with the per-replica invariants of the reference's message
    flow that hold at every prefix, and commits that happened: at least one, and at most one per
    (replica, proposer, decree).  (The batch does not quiesce in a test's time; the quiescence
    equalities are checked at n=4096 on fewer replicas below.)"""
    import bcsim
    from collections import Counter, defaultdict
    n, reps = 4096, 10_000
    c = bcsim.preset("c3_paxos")
    c.n_replicas = reps
    c.paxos_decrees = 2
    c.t_end_ns = 0
    with bcsim.Simulator(c) as s:
        for k in range(1, 9):  # (in 2 s steps, each a bounded run)
            s.run(2_000_000_000 * k)
            print(f"[c3 10k] t={2 * k} s", flush=True)
        cnt, st, tr = s.counters(), s.status(), s.trace()
    assert st["error"] == 0
    d = cnt["delivered"]
    assert d[0] > reps * 3 * 4000
    # a response only for a delivered request (paxos-node.cc:177-247)
    assert d[3] <= d[0] and d[4] <= d[1] and d[5] <= d[2]
    # the three proposers of every replica request their first ticket at t = 0
    # (paxos-node.cc:136-138, :510-522), and every ticket broadcast is logged once (:518)
    t0 = defaultdict(set)
    tickets = 0
    for r in tr:
        if r[6] == _abi.TR["PAXOS_TICKET"]:
            tickets += 1
            if r[1] == 0:
                t0[r[0]].add(r[5])
    assert len(t0) == reps and all(v == {0, 1, 2} for v in t0.values())
    # a broadcast reaches N-2 peers plus one dropped *end() send (:481-496)
    assert d[0] <= (n - 2) * tickets
    assert d[0] + d[1] + d[2] <= (n - 2) * cnt["dropped"]
    # a proposer commits each of its decrees at most once
    commits = Counter((r[0], r[5], r[8]) for r in tr if r[6] == _abi.TR["PAXOS_COMMIT"])
    assert len(commits) > 0, "no replica committed by 16 s"
    assert max(commits.values()) == 1


@pytest.mark.timeout(600)
def test_c3_paxos4096_to_quiescence(engine_lib):
    """configs[2] at full n (Paxos n=4096, three proposers, two decrees each, jittered links)
    on 64 replicas, run to quiescence, with the equalities of the reference's message flow at
    the end: every request delivered was answered (paxos-node.cc:177-247), every broadcast
    reached its N-2 peers plus the one dropped *end() send (:481-496), and every proposer of
    every replica committed each of its decrees exactly once (:322-339)."""
    import bcsim
    from collections import Counter
    n, reps, K = 4096, 64, 2
    c = bcsim.preset("c3_paxos")
    c.n_replicas = reps
    c.paxos_decrees = K
    c.t_end_ns = 0
    with bcsim.Simulator(c) as s:
        t = 0
        while True:  # (in 5 s steps: a bound on a livelocked run)
            t += 5_000_000_000
            s.run(t)
            if s.status()["quiescent"] or t >= 120_000_000_000:
                break
        cnt, st, tr = s.counters(), s.status(), s.trace()
    assert st["error"] == 0 and st["quiescent"]
    d = cnt["delivered"]
    assert d[3] == d[0] and d[4] == d[1] and d[5] == d[2]
    assert d[0] + d[1] + d[2] == (n - 2) * cnt["dropped"]
    commits = Counter((r[0], r[5], r[8]) for r in tr if r[6] == _abi.TR["PAXOS_COMMIT"])
    assert len(commits) == reps * 3 * K and set(commits.values()) == {1}
