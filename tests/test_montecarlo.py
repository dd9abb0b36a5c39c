"""KS acceptance for jittered links (north star: "on jittered links the
commit-latency distributions must match within a stated KS-test tolerance").

Reference order = the oracle with the glibc global stream (draws in global
event order, exactly the reference's rand() use), one run per seed.  The
engine = batched replicas with per-(replica, node, draw) counter streams.

Tolerance (stated here, applied to every comparison): the two-sample KS test
must not reject at the 1 % level (p >= 0.01) AND the statistic must satisfy
D <= KS_D_MAX (an effect-size bound that stays meaningful for large samples).
"""
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
