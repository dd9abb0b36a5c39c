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


@pytest.mark.timeout(600)
def test_c3_paxos4096_multidecree_sparse_replicas(engine_lib):
    """BASELINE configs[2] in the sparse layout: Paxos n=4096, 3 decrees, jittered
    U{0..49} ms app delays, 256 replicas in one launch -- per replica the
    request/response and broadcast KATs, and every proposer commits every decree."""
    import bcsim
    from collections import Counter
    n, reps, K = 4096, 256, 3
    c = bcsim.preset("c3_paxos")
    c.n_replicas = reps
    c.paxos_decrees = K
    c.seed = 5
    c.engine_mode = _abi.ENGINE_SPARSE
    tr, cnt, st = bcsim.run(c)
    assert st["error"] == 0 and st["quiescent"]
    d = cnt["delivered"]
    assert d[0] == d[3] and d[1] == d[4] and d[2] == d[5]
    tickets = sum(1 for r in tr if r[6] == _abi.TR["PAXOS_TICKET"])
    assert d[0] == (n - 2) * tickets
    assert cnt["dropped"] * (n - 2) == d[0] + d[1] + d[2]
    commits = Counter((r[0], r[5], r[8]) for r in tr if r[6] == _abi.TR["PAXOS_COMMIT"])
    # (replica, proposer, decree): each proposer commits each decree exactly once
    assert len(commits) == reps * c.paxos_proposers * K and max(commits.values()) == 1
