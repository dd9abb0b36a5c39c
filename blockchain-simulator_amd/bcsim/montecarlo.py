"""Monte Carlo replicas and the KS acceptance test for jittered links
(BASELINE configs[2]).

With random app delays (getRandomDelay, pbft-node.cc:66-69, raft-node.cc:63-66,
paxos-node.cc:397-400) the reference draws from ONE global glibc stream in
event order, which is inherently serial.  The engine instead gives every
(replica, node, draw#) its own counter-based stream (BCSIM_RNG_COUNTER) and
runs many independent replicas in one launch.  Acceptance for such configs
is distributional: the commit-latency distribution of the batched replicas
must match the reference-order (glibc) distribution within a stated
two-sample Kolmogorov-Smirnov tolerance (tests/test_montecarlo.py).

Latency definitions (integer ns, from the trace records of include/bcsim.h):
  PBFT   commit line (pbft-node.cc:259) t  -  leader's block line (:387) t, same sequence
  Paxos  commit line (paxos-node.cc:339) t  (proposals start at t = 0, :136-138)
  Gossip first receipt t  -  origin block t, same sequence
"""
import math

import numpy as np

from . import _abi

_T = _abi.TR


def commit_latencies(trace, protocol):
    """Per-commit latencies (ns) from trace tuples
    (replica, t, key_ts, key_origin, key_sub, node, kind, a, b, c)."""
    if protocol == _abi.PAXOS:
        return np.array([r[1] for r in trace if r[6] == _T["PAXOS_COMMIT"]], dtype=np.int64)
    if protocol == _abi.PBFT:
        start_kind, end_kind, seq_start, seq_end = _T["PBFT_BLOCK"], _T["PBFT_COMMIT"], 7, 9
    elif protocol == _abi.GOSSIP:
        start_kind, end_kind, seq_start, seq_end = _T["GOSSIP_BLOCK"], _T["GOSSIP_DELIVER"], 7, 7
    else:
        raise ValueError("commit latency is defined for PBFT, Paxos and gossip")
    t0 = {(r[0], r[seq_start]): r[1] for r in trace if r[6] == start_kind}
    return np.array([r[1] - t0[(r[0], r[seq_end])] for r in trace
                     if r[6] == end_kind and (r[0], r[seq_end]) in t0], dtype=np.int64)


def run_replicas(cfg, n_replicas, seed=1, topology=None):
    """Batched counter-RNG replicas of `cfg` on the GPU engine -> latencies (ns)."""
    from . import Simulator
    c = _abi.Config.from_buffer_copy(cfg)
    c.rng_mode = _abi.RNG_COUNTER
    c.n_replicas = n_replicas
    c.seed = seed
    with Simulator(c) as s:
        if topology is not None:
            s.set_topology(*topology)
        s.run()
        return commit_latencies(s.trace(), c.protocol)


def _ks_pvalue(d, n, m):
    """Asymptotic two-sided p-value of the two-sample KS statistic
    (Kolmogorov distribution with the Stephens small-sample correction)."""
    en = math.sqrt(n * m / (n + m))
    lam = (en + 0.12 + 0.11 / en) * d
    if lam < 1e-3:
        return 1.0
    s = 0.0
    for k in range(1, 101):
        term = 2.0 * (-1) ** (k - 1) * math.exp(-2.0 * k * k * lam * lam)
        s += term
        if abs(term) < 1e-12:
            break
    return min(1.0, max(0.0, s))


def ks_2samp(a, b):
    """Two-sample KS test -> (D, p).  D = sup |F_a - F_b| over the pooled
    sample (ties handled by evaluating both CDFs after each distinct value)."""
    a = np.sort(np.asarray(a))
    b = np.sort(np.asarray(b))
    if len(a) == 0 or len(b) == 0:
        raise ValueError("empty sample")
    x = np.union1d(a, b)
    fa = np.searchsorted(a, x, side="right") / len(a)
    fb = np.searchsorted(b, x, side="right") / len(b)
    d = float(np.max(np.abs(fa - fb)))
    return d, _ks_pvalue(d, len(a), len(b))
