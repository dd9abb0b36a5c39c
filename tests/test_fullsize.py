"""BASELINE configs at full size on the GPU, checked through size-independent
properties (the oracle is too slow at these sizes):

* C4  the bench configuration itself (bench.py: 50 KB blocks on saturated 3 Mbps links,
      fixed 3 ms app delay, the glibc rand()%100==5 lottery on, pbft-node.cc:371-411) run
      to quiescence over 66 blocks, so that the lottery hits at draws 60 and 65 (the glibc
      seed-1 stream, tests/golden/glibc_rand_seed1.json): deliveries per type, one commit
      per (node, block) in order with the leader's value, two VIEW records.
* C4  PBFT n=4096 full mesh, unsaturated blocks, view change off: every round
      delivers exactly 3(N-1)^2 + (N-1) messages (pbft-node.cc:193-265) and every
      node commits each sequence once, in order, with the leader's value.
* C5  gossip n=65536 on the random 8-regular graph (seed 1), echoes off so that
      every link carries one block per sequence: deliveries = rounds * sum(deg),
      one first receipt per (node, sequence) except the origin, and the hop count
      of the first receipt is the BFS distance from the origin.
* C3  Paxos n=4096, jittered U{0..49} ms app delays, counter-RNG replicas: every
      request gets exactly one response of its phase, each broadcast reaches N-2
      peers plus one dropped *end() send (paxos-node.cc:450-505), every ticket
      request is logged (:518), and every replica reaches a client commit (:339).
"""
from collections import Counter, deque

import numpy as np
import pytest

from bcsim import _abi

pytestmark = pytest.mark.gpu
TR = _abi.TR


@pytest.mark.timeout(300)
def test_c4_pbft4096_message_and_commit_kats(engine_lib):
    import bcsim
    n, rounds = 4096, 3
    c = _abi.default_config(_abi.PBFT, n)
    c.delay_mode = _abi.DELAY_FIXED
    c.app_delay_ns = 3_000_000
    c.pbft_rounds = rounds
    c.pbft_block_bytes = 1000       # unsaturated: 2.75 ms per block on a 3 Mbps link
    c.pbft_view_change = 0
    c.stop_ns = -1
    tr, cnt, st = bcsim.run(c)
    assert st["error"] == 0 and st["quiescent"]
    assert cnt["delivered_total"] == rounds * (3 * (n - 1) ** 2 + (n - 1))
    assert cnt["delivered"][1] == rounds * (n - 1)           # PRE_PREPARE
    for ty in (2, 3, 5):                                       # PREPARE, COMMIT, PREPARE_RES
        assert cnt["delivered"][ty] == rounds * (n - 1) ** 2
    commits = [r for r in tr if r[6] == TR["PBFT_COMMIT"]]
    assert len(commits) == rounds * n
    per_node = {}
    for r in sorted(commits):
        per_node.setdefault(r[5], []).append((r[8], r[9]))   # (block_num, value)
    assert len(per_node) == n
    # block k carries value n = k (:89-92) to every replica; the leader never receives its
    # own PRE_PREPARE, so its tx[k].val is the zero-initialised one
    assert all(v == [(k, k) for k in range(rounds)] for node, v in per_node.items() if node != 0)
    assert per_node[0] == [(k, 0) for k in range(rounds)]
    blocks = [r for r in tr if r[6] == TR["PBFT_BLOCK"]]
    assert [r[7] for r in sorted(blocks)] == list(range(rounds)) and {r[5] for r in blocks} == {0}


@pytest.mark.timeout(170)
def test_c4_bench_config_saturated_lottery_kats(engine_lib):
    import bcsim
    from fullsize_props import bench_config, check_bench_config
    c = bench_config(4096)
    tr, cnt, st = bcsim.run(c)
    check_bench_config(tr, cnt, st, c)


def bfs(row, col, src):
    d = np.full(len(row) - 1, -1, dtype=np.int64)
    d[src] = 0
    q = deque([src])
    while q:
        u = q.popleft()
        for v in col[row[u]:row[u + 1]]:
            if d[v] < 0:
                d[v] = d[u] + 1
                q.append(v)
    return d


@pytest.mark.timeout(300)
def test_c5_gossip65536_delivery_and_hop_kats(engine_lib):
    import bcsim
    n, rounds = 65536, 3
    c = bcsim.preset("c5_gossip65536")
    c.pbft_rounds = rounds
    c.echo = 0
    row, col = bcsim.random_regular(n, 8, 1)
    tr, cnt, st = bcsim.run(c, topology=(row, col, None))
    assert st["error"] == 0 and st["quiescent"]
    assert cnt["delivered_total"] == rounds * int(row[-1])
    first = [r for r in tr if r[6] == TR["GOSSIP_DELIVER"]]
    seen = Counter((r[5], r[7]) for r in first)
    assert len(seen) == rounds * (n - 1) and max(seen.values()) == 1
    assert all(r[5] != 0 for r in first)                       # the origin never "receives" its block
    dist = bfs(row, col, 0)
    hops = np.array([r[8] for r in first])
    nodes = np.array([r[5] for r in first])
    assert np.array_equal(hops, dist[nodes])


@pytest.mark.timeout(300)
def test_c3_paxos4096_replica_kats(engine_lib):
    import bcsim
    n, reps = 4096, 4
    c = bcsim.preset("c3_paxos")
    c.n_replicas = reps
    c.seed = 7
    tr, cnt, st = bcsim.run(c)
    assert st["error"] == 0
    d = cnt["delivered"]
    assert d[0] == d[3] and d[1] == d[4] and d[2] == d[5]      # one response per request
    tickets = Counter(r[0] for r in tr if r[6] == TR["PAXOS_TICKET"])
    commits = Counter(r[0] for r in tr if r[6] == TR["PAXOS_COMMIT"])
    assert d[0] == (n - 2) * sum(tickets.values())              # every requireTicket broadcast (:510-522)
    assert d[1] % (n - 2) == 0 and d[2] % (n - 2) == 0
    assert cnt["dropped"] * (n - 2) == d[0] + d[1] + d[2]      # one *end() send per broadcast
    assert set(commits) == set(range(reps))                     # every replica commits
