"""FQCODEL queue disc: ns-3 FqCoDelQueueDisc in front of the
PointToPointNetDevice queue, the version-dependent default root queue disc that
`address.Assign` installs (/root/reference/blockchain-simulator.cc:41-42).

CPU: the Murmur3 restatement against the published MurmurHash3_x86_32 vectors; the model is
FIFO-identical to the INFINITE queue on unsaturated links; message conservation.
GPU: the HIP engine equals the oracle bit for bit on every FQCODEL case.
ns-3 itself is absent, so the model beyond the hash is parity unpinned."""
import ctypes as C
import copy

import pytest

import oracle
from bcsim import _abi
from parity_cases import cases, compare, fq_cases, topology

FQ = fq_cases()


def test_murmur3_vectors():
    lib = oracle.lib()
    lib.oracle_murmur3_32.argtypes = [C.c_char_p, C.c_uint32, C.c_uint32]
    lib.oracle_murmur3_32.restype = C.c_uint32
    # MurmurHash3_x86_32 reference vectors (data, seed, hash)
    for data, seed, want in [(b"", 0, 0), (b"", 1, 0x514E28B7), (b"", 0xFFFFFFFF, 0x81F16F39),
                             (b"\0\0\0\0", 0, 0x2362F9DE), (b"aaaa", 0x9747B28C, 0x5A97808A),
                             (b"Hello, world!", 0x9747B28C, 0x24884CBA),
                             (b"The quick brown fox jumps over the lazy dog", 0x9747B28C, 0x2FA826CD)]:
        assert lib.oracle_murmur3_32(data, len(data), seed) == want


def test_flow_hash_spreads_classes():
    """The three packet classes of a link (app / echo first fragments, later fragments) hash to
    flow indices in [0, Flows); over the n=16 mesh most links keep them apart."""
    lib = oracle.lib()
    lib.oracle_fq_flow.argtypes = [C.c_uint32] * 6
    lib.oracle_fq_flow.restype = C.c_uint32
    n, k, apart = 16, 0, 0
    for i in range(1, n):
        for j in range(i):
            net = 0x01000000 + (k << 8)
            a, b = net + 1, net + 2
            h = {lib.oracle_fq_flow(a, b, 49153 + j, 7071, 0, 1024), lib.oracle_fq_flow(a, b, 7071, 49153 + i - 1, 0, 1024),
                 lib.oracle_fq_flow(a, b, 0, 0, 0, 1024)}
            assert all(x < 1024 for x in h)
            apart += len(h) == 3
            k += 1
    assert apart >= k - 3
    # Flows = 1: one queue per link
    assert lib.oracle_fq_flow(1, 2, 3, 4, 0, 1) == 0


@pytest.mark.parametrize("name", ["pbft16_small_blocks", "raft64_fixed", "paxos32_jitter_ctr", "gossip64_d4_fixed"])
def test_unsaturated_equals_fifo(name):
    """Without a standing device-queue backlog the disc never holds a packet across a wake:
    every message leaves in FIFO order, so the run equals the INFINITE queue."""
    cfg = cases()[name]
    fq = copy.copy(cfg)
    fq.queue_model = _abi.QUEUE_FQCODEL
    a = oracle.run(cfg, topology=topology(name))
    b = oracle.run(fq, topology=topology(name))
    assert b[1]["frames_dropped"] == 0
    assert compare(a, b) is None


@pytest.mark.parametrize("name", sorted(FQ))
def test_oracle_conservation(name):
    """Every application send is delivered, lost (a dropped fragment) or still in flight at the
    end; drops happen on the saturated cases and each lost message dropped >= 1 fragment."""
    tr, cnt, st = oracle.run(FQ[name], topology=topology(name))[:3]
    assert st["error"] == 0
    assert cnt["delivered_total"] + cnt["msgs_lost"] + cnt["dropped"] <= cnt["sends"]
    assert cnt["msgs_lost"] <= cnt["frames_dropped"]
    if name.startswith("pbft16") or name.startswith("gossip"):
        assert cnt["frames_dropped"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(FQ))
def test_engine_matches_oracle_fqcodel(name, engine_lib):
    import bcsim
    cfg = FQ[name]
    topo = topology(name)
    ref = oracle.run(cfg, topology=topo)
    got = bcsim.run(cfg, topology=topo)
    assert ref[2]["error"] == 0
    diff = compare(ref, got)
    assert diff is None, f"{name}: {diff}"


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_fqcodel_partitioned_p2_matches_oracle(engine_lib):
    """Node-partitioned at P=2 (host transport): the queue disc lives with the sender's edges, so
    records emitted at a device-queue wake for a receiver on the other rank are shipped like any
    other; the merged run equals the oracle."""
    import partition_run
    names = ["pbft16_fq_100", "pbft12_fq_jitter", "gossip64_d4_fq"]
    res = partition_run.run(2, names, transport="host", timeout=240)
    for name in names:
        merged, err = res[name]
        assert err is None, f"{name}: {err}"
        d = compare(oracle.run(FQ[name], topology=topology(name)), merged)
        assert d is None, f"{name} P=2: {d}"


def _ports(name):
    lib = oracle.lib()
    lib.oracle_fq_ports.argtypes = [C.c_void_p, C.POINTER(C.c_uint32), C.c_uint64]
    lib.oracle_fq_ports.restype = C.c_uint64
    cfg, topo = FQ[name], topology(name)
    with oracle.OracleSim(cfg) as o:
        if topo is not None:
            o.set_topology(*topo)
        o.run(_abi.INT64_MAX)
        n = cfg.n_nodes
        buf = (C.c_uint32 * (n * n))()
        E = lib.oracle_fq_ports(o.h, buf, n * n)
    return [list(buf[i * (n - 1):(i + 1) * (n - 1)]) for i in range(n)], E


def test_client_ports_bind_at_first_send():
    """ns-3's UdpSocketImpl::Connect only records the peer; the socket takes the node's next
    ephemeral port (49153, 49154, ...) at its first Send.  PBFT with fixed delays
    sends in peer order (the leader's block broadcast, then every node's PREPARE broadcast), so
    ports follow the peer order; a Raft follower's first send is its vote reply to the
    candidate (raft-node.cc:166), whose socket therefore holds 49153."""
    rows, E = _ports("pbft8_fq_40")
    assert E == 8 * 7
    for i, r in enumerate(rows):
        assert r == [49153 + k for k in range(7)], (i, r)
    rows, _ = _ports("raft16_fq")
    first = {i: r.index(49153) for i, r in enumerate(rows) if 49153 in r}
    peers = {i: (k if k < i else k + 1) for i, k in first.items()}
    cand = {p for p in peers.values()}
    assert len(cand) <= 2, peers          # one candidate (its own first send goes elsewhere)
    assert any(r != sorted(r) for r in rows if any(r)), "Raft ports should not follow peer order"
    for r in rows:                        # bound ports are dense from 49153
        b = sorted(x for x in r if x)
        assert b == [49153 + k for k in range(len(b))]


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_fqcodel_c4_fullsize_conservation(engine_lib):
    """The bench configuration (PBFT n=4096 full mesh, 50 KB blocks every 50 ms on 3 Mb/s links)
    under FQCODEL: the leader's saturated links drop (CoDel / overlimit), every application
    send is delivered, lost or still in flight, and each lost message dropped a fragment."""
    import bcsim
    from parity_cases import fullsize_cases
    c = fullsize_cases()["c4_fq_r6"]
    tr, cnt, st = bcsim.run(c)[:3]
    assert st["error"] == 0
    assert cnt["frames_dropped"] > 0
    assert cnt["delivered_total"] + cnt["msgs_lost"] + cnt["dropped"] <= cnt["sends"]
    assert 0 < cnt["msgs_lost"] <= cnt["frames_dropped"]
    assert cnt["delivered"][2] > 0  # PREPAREs got through


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_fqcodel_c4_n4096_matches_oracle_200ms(engine_lib):
    """The bench configuration under FQCODEL at BASELINE size (PBFT n=4096 full mesh, 16.8 M
    links each with its FqCoDel disc and device queue, blockchain-simulator.cc:41-42) against the
    oracle over the first 200 ms simulated: the leader's 50 KB PRE_PREPARE through 4095 discs
    (35 fragments each) and the PREPARE wave, 16.8 M deliveries -- traces and counters bit for
    bit.  (The oracle creates a link's FQ state at its first packet: ~60 s and ~13 GB here.)"""
    import bcsim
    c = bcsim.preset("c4_pbft4096")
    c.stop_ns = -1
    c.queue_model = _abi.QUEUE_FQCODEL
    c.t_end_ns = 200_000_000
    got = bcsim.run(c)
    assert got[2]["error"] == 0
    want = oracle.run(c)
    assert want[1]["delivered_total"] > 16_000_000
    d = compare(want, got)
    assert d is None, d
