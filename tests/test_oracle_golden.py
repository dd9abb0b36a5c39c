"""CPU oracle pinned against the golden fixtures (no GPU).

The oracle is test infrastructure; these tests pin it before it is trusted as
the parity checker of the HIP engine.
"""
import json
import os
import struct

import pytest

import oracle
from bcsim import _abi

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


def f32(x):
    return struct.unpack("f", struct.pack("f", x))[0]


def test_glibc_rand_restatement_matches_libc_fixture():
    gold = load("glibc_rand_seed1.json")["values"]
    assert oracle.glibc_rand(1, len(gold)) == gold


def test_glibc_rand_matches_live_libc_other_seeds():
    import ctypes
    libc = ctypes.CDLL("libc.so.6")
    for seed in (0, 2, 12345, 2**31 - 1):
        libc.srand(seed)
        live = [libc.rand() for _ in range(500)]
        assert oracle.glibc_rand(seed, 500) == live, seed


def test_time_tables():
    gold = load("time_tables.json")
    for name, mode in (("round", _abi.TIME_ROUND), ("trunc", _abi.TIME_TRUNC)):
        t = gold[name]
        assert [oracle.seconds_to_ns(f32((k + 3) / 1000), mode) for k in range(3)] == t["pbft_delay"]
        assert [oracle.seconds_to_ns(f32((k + 150) / 1000), mode) for k in range(150)] == t["raft_election"]
        assert [oracle.seconds_to_ns(f32(k / 1000), mode) for k in range(50)] == t["paxos_delay"]
        for b, v in t["msg_tx_3Mbps"].items():
            assert oracle.msg_tx(int(b), 1500, 3_000_000, mode) == v


def test_time_conversion_known_values():
    # 0.005f = 4,999,999.888 ns; 0.05f = 50,000,000.745 ns
    assert oracle.seconds_to_ns(f32(0.005), _abi.TIME_ROUND) == 5_000_000
    assert oracle.seconds_to_ns(f32(0.005), _abi.TIME_TRUNC) == 4_999_999
    assert oracle.seconds_to_ns(f32(0.05), _abi.TIME_ROUND) == 50_000_001
    assert oracle.seconds_to_ns(f32(0.05), _abi.TIME_TRUNC) == 50_000_000
    diffs = sum(oracle.seconds_to_ns(f32(k / 1000), 0) != oracle.seconds_to_ns(f32(k / 1000), 1)
                for k in range(300))
    assert diffs == 146


def test_wire_sizes():
    # PBFT 4-byte control: 34 B wire; 50,000 B block: 34 fragments, 50,756 B wire
    assert oracle.msg_tx(4)["wire"] == 34
    blk = oracle.msg_tx(50_000)
    assert blk["frames"] == 34 and blk["wire"] == 50_756
    rp = oracle.msg_tx(20_000)
    assert rp["frames"] == 14 and rp["wire"] == 20_316
    assert oracle.msg_tx(3)["tx_total"] == 88_000


def _fixed(proto, n, **kw):
    c = _abi.default_config(proto, n)
    c.delay_mode = _abi.DELAY_FIXED
    for k, v in kw.items():
        setattr(c, k, v)
    return c


@pytest.mark.parametrize("n", [4, 6, 8, 16])
def test_pbft_message_count_kat(n):
    # 3(N-1)^2 + (N-1) app messages per round; rounds = 10
    c = _fixed(_abi.PBFT, n, app_delay_ns=3_000_000, pbft_rounds=10, pbft_block_bytes=1000,
               pbft_view_change=0)
    tr, cnt, st = oracle.run(c)
    assert cnt["delivered_total"] == 10 * (3 * (n - 1) ** 2 + (n - 1))
    commits = [r for r in tr if r[6] == _abi.TR["PBFT_COMMIT"]]
    # non-leaders commit at the floor(N/2)+1-th COMMIT of N-2 received: N<=4 never
    per_node = {}
    for r in commits:
        per_node[r[5]] = per_node.get(r[5], 0) + 1
    if n <= 4:
        assert set(per_node) <= {0}
    else:
        assert all(per_node.get(i, 0) == 10 for i in range(n))


def test_pbft_odd_n_double_prepare_crossing():
    # N odd: N-1 = 2*floor(N/2) PREPARE_RES -> the >= N/2 threshold is crossed twice
    n = 5
    c = _fixed(_abi.PBFT, n, app_delay_ns=3_000_000, pbft_rounds=3, pbft_block_bytes=1000,
               pbft_view_change=0)
    tr, cnt, st = oracle.run(c)
    d = cnt["delivered"]
    assert d[3] == 3 * 2 * (n - 1) * (n - 1)  # two COMMIT broadcasts per non-leader


def test_raft_n8_first_election_kat():
    gold = load("kat.json")
    assert gold["raft_n8_initial_timeouts_ms"] == [283, 286, 177, 265, 293, 235, 286, 192]
    c = _fixed(_abi.RAFT, 8, app_delay_ns=1_000_000, t_end_ns=2_000_000_000)
    tr, cnt, st = oracle.run(c)
    first = [r for r in tr if r[6] == _abi.TR["RAFT_ELECTION"]][0]
    assert first[5] == 2 and first[1] == oracle.seconds_to_ns(f32(0.177))
    leader = [r for r in tr if r[6] == _abi.TR["RAFT_LEADER"]]
    assert leader and leader[0][5] == 2


def test_pbft_view_change_at_lottery_draw_60():
    # fixed delays: the only rand() draws are the per-block lottery; draw 60 hits
    c = _fixed(_abi.PBFT, 16, app_delay_ns=3_000_000, pbft_rounds=100)
    tr, cnt, st = oracle.run(c)
    blocks = [r for r in tr if r[6] == _abi.TR["PBFT_BLOCK"]]
    assert [b[7] for b in blocks[:61]] == list(range(61))
    assert all(b[5] == 0 for b in blocks[:61])            # node 0 leads blocks 0..60
    views = [r for r in tr if r[6] == _abi.TR["PBFT_VIEW"]]
    assert views and views[0][5] == 1 and views[0][7] == 2  # node 1 learns view 2


@pytest.mark.parametrize("name", ["pbft16_fixed_100", "pbft8_fixed_40", "raft8_fixed", "paxos8_fixed"])
def test_oracle_trace_fixture(name):
    gold = load(f"trace_{name}.json")
    c = _abi.Config()
    for k, v in gold["config"].items():
        if k == "reserved":
            continue
        setattr(c, k, v)
    tr, cnt, st = oracle.run(c)
    assert [list(r) for r in tr] == gold["trace"]
    # counters added after the fixture was made (link-queue drops) are zero there
    assert {k: cnt[k] for k in gold["counters"]} == gold["counters"]
    assert all(cnt[k] == 0 for k in cnt if k not in gold["counters"])


def test_paxos_offbyone_broadcast():
    # paxos-node.cc:481-496: N-2 real recipients + one dropped *end() send
    n = 8
    c = _fixed(_abi.PAXOS, n, app_delay_ns=2_000_000)
    tr, cnt, st = oracle.run(c)
    tickets = [r for r in tr if r[6] == _abi.TR["PAXOS_TICKET"]]
    assert cnt["dropped"] >= len(tickets)
    assert cnt["delivered"][0] == (n - 2) * len(tickets)  # REQUEST_TICKET deliveries


def test_oracle_partial_runs_equal_full_run():
    c = _fixed(_abi.PBFT, 8, app_delay_ns=3_000_000, pbft_rounds=12)
    full = oracle.run(c)
    o = oracle.OracleSim(c)
    t = 0
    while True:
        t += 37_000_001
        o.run(t)
        if o.status()["quiescent"]:
            break
    assert o.trace() == full[0]
    assert o.counters() == full[1]
    o.close()
