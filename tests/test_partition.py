"""Node-partitioned multi-GPU PDES.

CPU (gloo, world 2): the host-callback transport (bcsim_transport) that the
engine calls once per lookahead cell, and the per-rank result merge.
GPU: the same parity cases run partitioned over 2 and 3 ranks sharing the
one GPU (gloo host transport) -- merged traces and summed counters must be
bit-identical to the oracle, i.e. to the single-process run -- and the RCCL
transport at world 1 (the device exchange path with no remote peers).
"""
import ctypes as C
import os
import socket

import pytest
import torch.multiprocessing as mp

import oracle
from parity_cases import cases, compare, topology


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _transport_worker(rank, world, port, q):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(repo, "blockchain-simulator_amd"))
    import torch.distributed as dist
    from bcsim.partition import TorchTransport
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tr = TorchTransport(dist)
    # all-reduce MIN / SUM, called the way the engine calls it (through the C thunk)
    v = (C.c_int64 * 3)(10 + rank, -rank, 1 << 40)
    assert tr.struct.allreduce_i64(None, v, 3, 0) == 0
    mn = list(v)
    v = (C.c_int64 * 3)(10 + rank, -rank, 1 << 40)
    assert tr.struct.allreduce_i64(None, v, 3, 1) == 0
    sm = list(v)
    # all-to-all-v: rank r sends (r+1)*(d+1) bytes of value 16*r+d to rank d
    segs = [bytes([16 * rank + d]) * ((rank + 1) * (d + 1)) for d in range(world)]
    send = b"".join(segs)
    sb = (C.c_uint64 * world)(*[len(x) for x in segs])
    rb = (C.c_uint64 * world)()
    cap = 64
    recv = (C.c_uint8 * cap)()
    sbuf = (C.c_uint8 * max(1, len(send))).from_buffer_copy(send or b"\0")
    assert tr.struct.alltoallv(None, C.cast(sbuf, C.c_void_p), sb, C.cast(recv, C.c_void_p), cap, rb) == 0
    got = bytes(recv[:sum(rb)])
    # a receive buffer that is too small is an error, not a truncation
    small = (C.c_uint8 * 1)()
    rc_small = tr.struct.alltoallv(None, C.cast(sbuf, C.c_void_p), sb, C.cast(small, C.c_void_p), 1, rb)
    # a failed rank (the last one) sends the PEER_ERR count and no payload: every rank's call
    # returns 0 with the counts only, so all of them leave the engine run together
    from bcsim.partition import PEER_ERR
    fail = rank == world - 1
    sb2 = (C.c_uint64 * world)(*([PEER_ERR] * world if fail else [len(x) for x in segs]))
    rb2 = (C.c_uint64 * world)()
    rc_peer = tr.struct.alltoallv(None, None if fail else C.cast(sbuf, C.c_void_p), sb2,
                                  C.cast(recv, C.c_void_p), cap, rb2)
    q.put((rank, mn, sm, list(rb), got, rc_small, rc_peer, list(rb2)))
    dist.destroy_process_group()


def test_torch_transport_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_transport_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, mn, sm, rb, got, rc_small, rc_peer, rb2 in res:
        assert mn == [10, -1, 1 << 40]
        assert sm == [21, -1, 2 << 40]
        want = [(r + 1) * (rank + 1) for r in range(world)]
        assert rb == want
        assert got == b"".join(bytes([16 * r + rank]) * want[r] for r in range(world))
        assert rc_small != 0
        assert rc_peer == 0 and rb2[world - 1] == 1 << 62


def test_merge_matches_single_process_shape():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "blockchain-simulator_amd"))
    from bcsim.partition import merge
    a = ([(0, 5, 1, 0, 0, 1, 2, 0, 0, 0)], dict(delivered=[1, 2], delivered_total=3, t_last_ns=7, events=4))
    b = ([(0, 3, 1, 0, 0, 0, 2, 0, 0, 0)], dict(delivered=[0, 5], delivered_total=5, t_last_ns=9, events=1))
    tr, cnt = merge([a, b])
    assert [t[1] for t in tr] == [3, 5]
    assert cnt == dict(delivered=[1, 7], delivered_total=8, t_last_ns=9, events=5)


# cases whose RNG is per node (counter) or absent: the glibc global stream of
# Raft is a single-GPU configuration (bcsim_run returns E_UNSUPPORTED)
PART_CASES = ["pbft12_jitter_b2", "pbft16_fixed_100", "pbft5_odd", "pbft12_jitter_ctr", "pbft8_rep3_ctr", "pbft8_compat",
              "raft16_jitter_ctr", "paxos8_fixed", "paxos32_jitter_ctr", "paxos16_jitter_rep4",
              "gossip64_d4_fixed", "gossip200_d8_jitter_ctr", "gossip24_mesh", "pbft32_d6_ctr",
              "pbft16_droptail_100", "gossip64_d4_droptail", "pbft12_hetero_prop", "paxos32_jitter_k4"]


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_matches_oracle(world, engine_lib):
    import partition_run
    res = partition_run.run(world, PART_CASES, transport="host", timeout=240)
    allc = cases()
    for name in PART_CASES:
        merged, err = res[name]
        assert err is None, f"{name} world={world}: {err}"
        ref = oracle.run(allc[name], topology=topology(name))
        d = compare(ref, merged)
        assert d is None, f"{name} world={world}: {d}"


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_partitioned_n512_matches_oracle(engine_lib):
    """SURVEY.md §8e at a size where each rank owns 256 nodes x 511 in-edges."""
    import partition_run
    name = "pbft512_small"
    merged, err = partition_run.run(2, [name], transport="host", timeout=240)[name]
    assert err is None, err
    d = compare(oracle.run(cases()[name]), merged)
    assert d is None, d


@pytest.mark.gpu
@pytest.mark.timeout(900)
@pytest.mark.parametrize("name,world", [("c4_bench_r4", 2), ("c5_gossip_r3", 2), ("c4_bench_r4", 4), ("c4_bench_r4", 8),
                                        ("c5_gossip_r3", 4), ("c5_gossip_r3", 8), ("c4_fq_r6", 2)])
def test_partitioned_fullsize_equals_single(name, world, engine_lib):
    """SURVEY.md §4 item 4 at BASELINE size: the bench configurations themselves --
    C4 PBFT n=4096 (50 KB blocks, glibc lottery on, 4 rounds; blockchain-simulator.cc:34-51
    mesh) and C5 gossip n=65536 on the random 8-regular graph (3 rounds, echoes on) --
    node-partitioned over 2, 4 and 8 ranks sharing the GPU (host transport; BASELINE configs[3]
    "1/2/4/8 MI355X node-partitioned PDES") give merged traces and counters identical to the
    single-process run, bit for bit."""
    import bcsim
    import partition_run
    from parity_cases import any_case
    topo = topology(name)
    single = bcsim.run(any_case(name), topology=topo)
    assert single[2]["error"] == 0 and single[2]["quiescent"]
    assert single[1]["delivered_total"] > 0
    merged, err = partition_run.run(world, [name], transport="host", timeout=840)[name]
    assert err is None, err
    d = compare(single, merged)
    assert d is None, f"{name} world={world}: {d}"
    if name == "c4_bench_r4" and world == 2:
        # broadcast de-dup (k_link_mesh xr_ship -> k_import): about half the 16.8 M records of
        # a heavy cell cross ranks, shipped as range records of up to 64 edges, so the volume
        # is far below one 32-byte record per cross-rank delivery
        cross = single[1]["delivered_total"] // 2
        assert merged[1]["xfer_bytes"] < cross * 32 // 16, (merged[1]["xfer_bytes"], cross)
    # one control exchange + one record exchange per window, plus the PBFT
    # tick's leader-flag all-reduce and the first / last agreement of a run() call
    assert merged[1]["collectives"] <= 2 * merged[1]["windows"] + 8 * 2 * 8, merged[1]


def _rccl1_worker(port, names, q, env=None):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [repo, os.path.join(repo, "tests"), os.path.join(repo, "blockchain-simulator_amd")]
    os.environ.update(env or {})
    import torch.distributed as dist
    import bcsim
    from parity_cases import any_case, topology
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    for name in names:
        with bcsim.Simulator(any_case(name)) as s:
            topo = topology(name)
            if topo is not None:
                s.set_topology(*topo)
            s.set_partition(dist, transport="rccl")
            s.run()
            q.put((name, s.trace(), s.counters()))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_transport_world1(engine_lib):
    names = ["pbft16_fixed_100", "raft16_jitter_ctr", "paxos16_jitter_rep4", "gossip200_d8_jitter_ctr"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl1_worker, args=(_free_port(), names, q))
    p.start()
    got = {}
    for _ in names:
        name, tr, cnt = q.get(timeout=180)
        got[name] = (tr, cnt)
    p.join(timeout=60)
    assert p.exitcode == 0
    allc = cases()
    for name in names:
        d = compare(oracle.run(allc[name], topology=topology(name)), got[name])
        assert d is None, f"{name}: {d}"


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", ["c4_bench_r4", "c5_gossip_r3"])
def test_rccl_world1_fullsize_partitioned_kernels(name, engine_lib):
    """BASELINE configs[3]/[4] at full size through the RCCL transport with the node-partitioned
    kernels forced at one rank (BCSIM_PDES_KERNELS=1): k_link_mesh<XR> / the partitioned generic
    kernels, the per-window RCCL control all-to-all and record sendrecv, k_import, the leader-flag
    all-reduce -- every device-side step of the P > 1 loop runs at n=4096 / n=65536 on the one GPU
    of the box (RCCL refuses two ranks on one device, so the cross-rank volume itself is covered by
    the host-transport P=2/4/8 tests above) and must equal the plain single-GPU run bit for bit."""
    import bcsim
    from parity_cases import any_case
    topo = topology(name)
    single = bcsim.run(any_case(name), topology=topo)
    assert single[2]["error"] == 0 and single[2]["quiescent"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    # (C5 with the control words computed on the device: k_ctl -> all-to-all on device buffers)
    env = {"BCSIM_PDES_KERNELS": "1", "BCSIM_CTL_DEV": "1" if name.startswith("c5") else "0"}
    p = ctx.Process(target=_rccl1_worker, args=(_free_port(), [name], q, env))
    p.start()
    got_name, tr, cnt = q.get(timeout=540)
    p.join(timeout=60)
    assert p.exitcode == 0 and got_name == name
    d = compare(single, (tr, cnt))
    assert d is None, f"{name}: {d}"


def _fail_worker(rank, world, port, fail_rank, q, fail_cell="3", t_until=None, hook="BCSIM_DBG_FAIL_CELL"):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [repo, os.path.join(repo, "tests"), os.path.join(repo, "blockchain-simulator_amd")]
    if rank == fail_rank:
        os.environ[hook] = fail_cell  # this rank alone fails at that cell
    import torch.distributed as dist
    import bcsim
    from parity_cases import cases
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    code = 0
    try:
        with bcsim.Simulator(cases()["pbft16_fixed_100"]) as s:
            s.set_partition(dist, transport="host")
            if t_until is None:
                s.run()
            else:
                s.run(t_until)
    except bcsim.EngineError as e:
        code = e.code
    q.put((rank, code))
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_one_rank_failure_stops_every_rank(engine_lib):
    """A rank-local failure (here injected) must end the run on every rank -- the failed
    one with its own error, the others with E_PEER -- instead of leaving them blocked in
    the next collective (include/bcsim.h bcsim_transport)."""
    world, fail_rank = 2, 1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_fail_worker, args=(r, world, port, fail_rank, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res[fail_rank] == -4  # BCSIM_E_OVERFLOW (injected)
    assert res[1 - fail_rank] == -11  # BCSIM_E_PEER


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_failure_in_last_partial_window_stops_every_rank(engine_lib):
    """A failure found after the exchange of the last window of a run() whose end is not a cell
    boundary (here: rank 1 fails after the exchange of the first window -- BCSIM_DBG_FAIL_IMPORT,
    as a k_import overflow found by the read-back would -- and the limit cuts that window at half
    a cell) is not lost: it is carried into the next iteration, which finds nothing left before
    the limit (bcsim_capi.hip run(), the lo >= hi exit), and every rank leaves with it."""
    world, fail_rank = 2, 1
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    t_half = 1_500_000  # half of the C1 lookahead cell (3 ms + one 34-byte frame)
    ps = [ctx.Process(target=_fail_worker, args=(r, world, port, fail_rank, q, "0", t_half, "BCSIM_DBG_FAIL_IMPORT")) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=180) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res[fail_rank] == -4  # BCSIM_E_OVERFLOW (injected)
    assert res[1 - fail_rank] == -11  # BCSIM_E_PEER
