"""KS acceptance for jittered links (north star: "on jittered links the
commit-latency distributions must match within a stated KS-test tolerance").

Reference order = the oracle with the glibc global stream (draws in global
event order, exactly the reference's rand() use), one run per seed.  The
engine = batched replicas with per-(replica, node, draw) counter streams.

Tolerance (stated here, applied to every comparison): the two-sample KS test
must not reject at the 1 % level (p >= 0.01) AND the statistic must satisfy
D <= KS_D_MAX (an effect-size bound that stays meaningful for large samples).
"""
import json
import os

import numpy as np
import pytest

import oracle
from bcsim import _abi
from bcsim.montecarlo import commit_latencies, ks_2samp

KS_P_MIN = 0.01
KS_D_MAX = 0.08


def _cfg(proto, n, rng, seed, reps):
    c = _abi.default_config(proto, n)
    c.delay_mode = _abi.DELAY_RANDOM  # getRandomDelay jitter
    c.rng_mode = rng
    c.seed = seed
    c.n_replicas = reps
    if proto == _abi.PBFT:
        c.pbft_rounds = 20
        c.pbft_block_bytes = 1000
        c.pbft_view_change = 0  # the lottery would change the leader differently per stream
        c.stop_ns = -1
    return c


CASES = {  # name: (protocol, n, glibc seeds, counter replicas)
    "pbft16": (_abi.PBFT, 16, 32, 64),
    "paxos16": (_abi.PAXOS, 16, 400, 400),
}


def _reference_order(proto, n, seeds):
    return np.concatenate([commit_latencies(oracle.run(_cfg(proto, n, _abi.RNG_GLIBC, s, 1))[0], proto)
                           for s in range(1, seeds + 1)])


def test_ks_matches_scipy():
    scipy_stats = pytest.importorskip("scipy.stats")
    rng = np.random.default_rng(0)
    for a, b in [(rng.normal(size=300), rng.normal(0.2, 1, size=500)),
                 (rng.integers(0, 5, 1000), rng.integers(0, 5, 700))]:
        d, p = ks_2samp(a, b)
        ref = scipy_stats.ks_2samp(a, b, method="asymp")
        assert abs(d - ref.statistic) < 1e-12
        assert abs(p - ref.pvalue) < 0.02


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_counter_stream_matches_glibc_order(name):
    """The counter RNG preserves the latency law of the reference's global stream."""
    proto, n, seeds, reps = CASES[name]
    ref = _reference_order(proto, n, seeds)
    ctr = commit_latencies(oracle.run(_cfg(proto, n, _abi.RNG_COUNTER, 7, reps))[0], proto)
    d, p = ks_2samp(ref, ctr)
    assert len(ref) > 1000 and len(ctr) > 1000
    assert p >= KS_P_MIN and d <= KS_D_MAX, (d, p)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_engine_replicas_match_glibc_order(name, engine_lib):
    from bcsim.montecarlo import run_replicas
    proto, n, seeds, reps = CASES[name]
    ref = _reference_order(proto, n, seeds)
    got = run_replicas(_cfg(proto, n, _abi.RNG_COUNTER, 0, 1), reps, seed=11)
    d, p = ks_2samp(ref, got)
    assert len(got) > 1000
    assert p >= KS_P_MIN and d <= KS_D_MAX, (d, p)


# ---- BASELINE sizes: C3 Paxos n=4096 and PBFT n=512 with the
# reference's getRandomDelay().  The glibc-order samples are too slow to make inside a test
# (~6 s of oracle per Paxos seed), so they are committed fixtures from
# tests/golden/make_ks_c3.py (200 / 48 seeds); the engine side is >= 1,000 counter-RNG replicas
# in one batched run.  Same tolerance as above.
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_c3_fixtures_reproduce_from_oracle():
    """The committed glibc-order samples are the oracle's: seed 1 of each, re-run here."""
    import sys
    sys.path.insert(0, GOLDEN)
    import make_ks_c3 as mk
    px = _golden("ks_c3_paxos4096.json")
    assert px["seeds"] >= 200 and len(px["latency_ns"]["1"]) >= 400 and len(px["latency_ns"]["2"]) >= 800
    assert mk._paxos((2, 1)) == px["per_seed"]["2"][0]
    pb = _golden("ks_pbft512.json")
    assert mk._pbft(1) == pb["per_seed"][0]


@pytest.mark.gpu
@pytest.mark.timeout(170)
@pytest.mark.parametrize("k", [1, 2])
def test_c3_paxos4096_replicas_match_glibc_order(k, engine_lib):
    """configs[2]: Paxos n=4096, U{0..49} ms app delays (paxos-node.cc:397-400), K decrees,
    1,000 counter-RNG replicas (sparse layout) vs 200 glibc-order oracle seeds."""
    from bcsim.montecarlo import run_replicas
    ref = np.array(_golden("ks_c3_paxos4096.json")["latency_ns"][str(k)])
    c = _abi.default_config(_abi.PAXOS, 4096)
    c.delay_mode = _abi.DELAY_RANDOM
    c.paxos_decrees = k
    got = run_replicas(c, 1000, seed=101 + k)
    d, p = ks_2samp(ref, got)
    assert len(got) >= 1000 * k
    assert p >= KS_P_MIN and d <= KS_D_MAX, (k, d, p, len(ref), len(got))


@pytest.mark.gpu
@pytest.mark.timeout(170)
def test_pbft512_getrandomdelay_replicas_match_glibc_order(engine_lib):
    """PBFT n=512 with the reference's 3-5 ms getRandomDelay() per send (pbft-node.cc:66-69):
    per (replica, block) the median commit latency over the nodes, 200 counter-RNG replicas
    vs 48 glibc-order oracle seeds."""
    import sys
    sys.path.insert(0, GOLDEN)
    import bcsim
    import make_ks_c3 as mk
    ref = np.array(_golden("ks_pbft512.json")["block_median_ns"])
    c = mk.pbft_cfg(0, _abi.RNG_COUNTER)
    c.n_replicas = 200
    c.seed = 77
    with bcsim.Simulator(c) as s:
        s.run()
        got = np.array(mk.pbft_block_medians(s.trace()))
    d, p = ks_2samp(ref, got)
    assert len(got) == 200 * 5
    assert p >= KS_P_MIN and d <= KS_D_MAX, (d, p)
