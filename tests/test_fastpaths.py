"""Fast paths against the generic kernels at full size.

The dense-gossip kernels (k_gossip_scan / k_gossip_link) and the sparse-Paxos acceptor
kernels (k_paxos_scan / k_paxos_link) restate scan_node / link_node for the simple nodes of
a window.  The oracle parity cases cover them at the sizes the oracle runs; here the same
run with the fast paths switched off (BCSIM_NO_GFAST=1, BCSIM_NO_PXFAST=1: every node through
the generic kernels) must give identical traces and counters at BASELINE sizes.

k_scan_pbft (the PBFT heavy waves, one pass over each row in registers) is checked the same
way on the bench configuration (BCSIM_NO_SFAST=1: off), and against the oracle on every PBFT
parity case with BCSIM_FEW_SCAN=0, so that even the small cases' launches take it.
"""
import os

import pytest

from bcsim import _abi
from parity_cases import compare

pytestmark = pytest.mark.gpu


def _run(cfg, topo, env):
    import bcsim
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        tr, cnt, st = bcsim.run(cfg, topology=topo)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert st["error"] == 0
    return tr, cnt


@pytest.mark.timeout(300)
def test_c5_gossip65536_fast_equals_generic(engine_lib):
    import bcsim
    cfg = bcsim.preset("c5_gossip65536")
    cfg.pbft_rounds = 4
    cfg.t_end_ns = 260_000_000  # four blocks, each flooding the whole graph
    topo = bcsim.random_regular(65536, 8, 1)
    fast = _run(cfg, topo, {"BCSIM_NO_GFAST": "0"})
    gen = _run(cfg, topo, {"BCSIM_NO_GFAST": "1"})
    assert fast[1]["delivered_total"] > 1_000_000
    assert compare(gen, fast) is None


@pytest.mark.timeout(300)
def test_c3_paxos_sparse_fast_equals_generic(engine_lib):
    import bcsim
    cfg = bcsim.preset("c3_paxos")
    cfg.n_nodes = 1024
    cfg.n_replicas = 64
    cfg.paxos_decrees = 2
    cfg.seed = 9
    cfg.t_end_ns = 1_500_000_000
    cfg.engine_mode = _abi.ENGINE_SPARSE
    fast = _run(cfg, None, {"BCSIM_NO_PXFAST": "0"})
    gen = _run(cfg, None, {"BCSIM_NO_PXFAST": "1"})
    assert fast[1]["delivered_total"] > 1_000_000
    assert compare(gen, fast) is None


@pytest.mark.timeout(170)
def test_c4_bench_config_fast_scan_equals_generic(engine_lib):
    from fullsize_props import bench_config
    cfg = bench_config(4096, rounds=6)
    fast = _run(cfg, None, {"BCSIM_NO_SFAST": "0"})
    gen = _run(cfg, None, {"BCSIM_NO_SFAST": "1"})
    assert fast[1]["delivered_total"] == 6 * (3 * 4095 ** 2 + 4095)
    assert compare(gen, fast) is None
    # k_mesh_row with every row on one wave (no split of the leader's row over 16 waves)
    whole = _run(cfg, None, {"BCSIM_ROW_SPLIT": "0"})
    assert compare(whole, fast) is None


def _pbft_cases():
    from parity_cases import cases
    return sorted(n for n, c in cases().items() if c.protocol == _abi.PBFT)


@pytest.mark.parametrize("name", _pbft_cases())
def test_fast_scan_every_launch_matches_oracle(name, engine_lib):
    import oracle
    from parity_cases import cases, topology
    cfg = cases()[name]
    topo = topology(name)
    got = _run(cfg, topo, {"BCSIM_FEW_SCAN": "0", "BCSIM_NO_SFAST": "0"})
    d = compare(oracle.run(cfg, topology=topo), got)
    assert d is None, f"{name} (k_scan_pbft on every launch): {d}"
