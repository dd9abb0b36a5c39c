"""Gossip (BCSIM_GOSSIP, BASELINE configs[4]) and the random-regular topology
builder on the CPU: generator invariants and analytic
known-answer tests of the oracle restatement.  Parity of the HIP engine with
these oracle runs is in tests/test_gpu_parity.py (cases gossip*, *_d6_ctr).

Gossip is a build extension (the reference has no gossip protocol), so its
parity is against the oracle's restatement only; the KATs below pin the
flooding semantics independently of both: every node relays each block once,
so deliveries = rounds * sum(degree), every non-origin node logs one first
receipt per block, and on an unloaded graph the hop count of a first receipt
is the BFS distance from the origin.
"""
from collections import deque

import numpy as np
import pytest

import oracle
from parity_cases import cases, topology


def _bfs(row, col, src=0):
    n = len(row) - 1
    dist = [-1] * n
    dist[src] = 0
    q = deque([src])
    while q:
        u = q.popleft()
        for v in col[row[u]:row[u + 1]]:
            if dist[v] < 0:
                dist[v] = dist[u] + 1
                q.append(v)
    return dist


@pytest.mark.parametrize("n,d,seed", [(64, 4, 1), (200, 8, 5), (65536, 8, 1), (11, 4, 3)])
def test_random_regular_is_simple_symmetric_regular(n, d, seed, engine_lib):
    import bcsim
    row, col = bcsim.random_regular(n, d, seed)
    assert row[0] == 0 and row[-1] == n * d
    assert np.all(np.diff(row.astype(np.int64)) == d)
    src = np.repeat(np.arange(n, dtype=np.int64), d)
    assert not np.any(src == col)  # no self-loops
    for i in range(min(n, 512)):  # rows ascending (reference peer order), no multi-edges
        r = col[row[i]:row[i + 1]]
        assert np.all(np.diff(r.astype(np.int64)) > 0)
    fwd = np.sort(src * n + col)
    bwd = np.sort(col.astype(np.int64) * n + src)
    assert np.array_equal(fwd, bwd)  # symmetric
    assert len(np.unique(fwd)) == len(fwd)
    row2, col2 = bcsim.random_regular(n, d, seed)  # deterministic in (n, d, seed)
    assert np.array_equal(col, col2)


def test_random_regular_rejects_bad_args(engine_lib):
    import bcsim
    with pytest.raises(bcsim.EngineError):
        bcsim.random_regular(9, 3, 1)  # n*d odd
    with pytest.raises(bcsim.EngineError):
        bcsim.random_regular(8, 8, 1)  # d >= n


@pytest.mark.parametrize("name", ["gossip64_d4_fixed", "gossip200_d8_jitter_ctr", "gossip512_d8_blocks",
                                  "gossip24_mesh"])
def test_oracle_gossip_kats(name, engine_lib):
    cfg = cases()[name]
    topo = topology(name)
    tr, cnt, st = oracle.run(cfg, topology=topo)
    assert st["error"] == 0
    n, rounds, reps = cfg.n_nodes, cfg.pbft_rounds, cfg.n_replicas
    deg_sum = len(topo[1]) if topo is not None else n * (n - 1)
    assert cnt["delivered_total"] == reps * rounds * deg_sum
    assert cnt["delivered"][1] == cnt["delivered_total"]
    assert cnt["echoes"] == cnt["delivered_total"] and cnt["wrong_msgs"] == 0
    blocks = [r for r in tr if r[6] == 30]
    firsts = [r for r in tr if r[6] == 31]
    assert len(blocks) == reps * rounds and all(r[5] == 0 for r in blocks)
    assert len(firsts) == reps * rounds * (n - 1)
    # one first receipt per (replica, node, seq), never at the origin
    keys = {(r[0], r[5], r[7]) for r in firsts}
    assert len(keys) == len(firsts) and all(r[5] != 0 for r in firsts)
    # blocks leave the origin every Seconds(0.05f) = 50,000,001 ns (round mode)
    assert sorted({r[1] for r in blocks}) == [50_000_001 * (k + 1) for k in range(rounds)]
    if name in ("gossip64_d4_fixed", "gossip24_mesh"):  # unloaded: first receipt on a shortest path
        row, col = topo[:2] if topo is not None else __import__("bcsim").full_mesh(n)
        dist = _bfs(row, col)
        assert all(r[8] == dist[r[5]] for r in firsts)
