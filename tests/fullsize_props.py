"""Size-independent properties of the exact bench configuration (bench.py, BASELINE
configs[3]): PBFT on the full mesh with 50 KB blocks on saturated 3 Mbps links, fixed 3 ms
app delay and the glibc rand()%100==5 lottery on (pbft-node.cc:371-411), run to quiescence
over 66 blocks so that the lottery hits at draws 60 and 65 of the glibc seed-1 stream.

Shared by tests/test_fullsize.py (the engine at n = 4096, GPU) and
tests/test_fullsize_props.py (the oracle at small n, CPU: the properties themselves are
checked against the reference restatement before they judge the engine).
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "blockchain-simulator_amd"))
from bcsim import _abi  # noqa: E402

TR = _abi.TR
ROUNDS = 66


def lottery_hits(rounds=ROUNDS):
    """Blocks whose lottery draw hits: one draw per leader tick (pbft-node.cc:401)."""
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "glibc_rand_seed1.json")) as f:
        stream = json.load(f)["values"]
    return [k for k in range(rounds) if stream[k] % 100 == 5]


def bench_config(n, rounds=ROUNDS):
    import bcsim
    c = bcsim.preset("c4_pbft4096")          # exactly bench.py's configuration ...
    assert c.pbft_view_change == 1 and c.rng_mode == _abi.RNG_GLIBC and c.pbft_block_bytes in (0, 50000)
    c.n_nodes = n
    c.pbft_rounds = rounds                   # ... run to quiescence
    c.stop_ns = -1
    return c


def check_bench_config(tr, cnt, st, c):
    n, rounds = c.n_nodes, c.pbft_rounds
    hits = lottery_hits(rounds)
    assert hits == [60, 65]
    assert st["error"] == 0 and st["quiescent"]
    n1 = n - 1
    d = cnt["delivered"]
    assert d[1] == rounds * n1                                  # PRE_PREPARE (:193-211)
    assert d[2] == d[3] == d[5] == rounds * n1 * n1             # PREPARE, COMMIT, PREPARE_RES
    assert d[8] == len(hits) * n1 and d[4] == 0                 # VIEW_CHANGE (:293-303, pbft-node.h:90)
    assert cnt["delivered_total"] == rounds * (3 * n1 * n1 + n1) + len(hits) * n1
    assert cnt["wrong_msgs"] == len(hits) * n1                  # VIEW_CHANGE falls through (:271-286)
    blocks = sorted(r for r in tr if r[6] == TR["PBFT_BLOCK"])
    assert [r[7] for r in blocks] == list(range(rounds))
    # leaders: node 0 for blocks 0..60, node 1 after the first view change (the second one,
    # at block 65, hands over to node 2 after the last block)
    lead = {r[7]: r[5] for r in blocks}
    assert [lead[k] for k in range(rounds)] == [0] * 61 + [1] * 5
    views = sorted((r[5], r[7], r[8]) for r in tr if r[6] == TR["PBFT_VIEW"])
    assert views == [(1, 2, 1), (2, 3, 2)]                      # (new leader, global v, leader)
    per_node = {}
    for r in sorted(r for r in tr if r[6] == TR["PBFT_COMMIT"]):
        per_node.setdefault(r[5], []).append((r[8], r[9]))     # (block_num, value)
    assert len(per_node) == n
    for node, got in per_node.items():
        # one commit per block, in order (block_num = k)
        assert [b for b, _ in got] == list(range(rounds)), node
        # block k carries value k (:89-92); its own leader never receives its PRE_PREPARE
        # (tx[k].val stays zero), and node 0 -- whose in-links queue seconds
        # of echoed 50 KB blocks -- commits node 1's blocks 61..65 before their PRE_PREPARE
        # arrives (value 0 as well)
        want = [0] * rounds if node == 0 else [0 if lead[k] == node else k for k in range(rounds)]
        assert [v for _, v in got] == want, node
