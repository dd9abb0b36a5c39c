"""Reference-order (glibc global stream) latency samples for the KS acceptance tests at
BASELINE sizes (tests/test_montecarlo.py): the oracle -- the reference's handlers with the
reference's single rand() stream consumed in event order (paxos-node.cc:397-400,
pbft-node.cc:66-69) -- run once per seed.  Too slow to regenerate inside a GPU test
(~6 s per Paxos n=4096 seed), so the samples are committed here:

    python tests/golden/make_ks_c3.py          (8 processes, ~6 min)

ks_c3_paxos4096.json  Paxos n=4096, jittered U{0..49} ms, K = 1 and K = 2 decrees, seeds 1..200:
                      every commit line's t (proposals start at t = 0, :136-138, :339)
ks_pbft512.json       PBFT n=512, getRandomDelay() 3-5 ms per send, 1000 B blocks, 5 blocks,
                      view change off, seeds 1..48: per (seed, block) the median over the
                      nodes of commit t - block t (pbft-node.cc:259, :387)
"""
import json
import multiprocessing as mp
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "blockchain-simulator_amd")]

PAXOS_SEEDS = 200
PBFT_SEEDS = 48


def paxos_cfg(k, seed, rng):
    from bcsim import _abi
    c = _abi.default_config(_abi.PAXOS, 4096)
    c.delay_mode = _abi.DELAY_RANDOM
    c.rng_mode = rng
    c.seed = seed
    c.paxos_decrees = k
    return c


def pbft_cfg(seed, rng):
    from bcsim import _abi
    c = _abi.default_config(_abi.PBFT, 512)
    c.delay_mode = _abi.DELAY_RANDOM
    c.rng_mode = rng
    c.seed = seed
    c.pbft_rounds = 5
    c.pbft_block_bytes = 1000
    c.pbft_view_change = 0  # the lottery would move the leader differently per stream
    c.stop_ns = -1
    return c


def pbft_block_medians(trace):
    """(replica, block) -> median over nodes of commit t - block t."""
    import numpy as np
    from bcsim import _abi
    T = _abi.TR
    t0 = {(r[0], r[7]): r[1] for r in trace if r[6] == T["PBFT_BLOCK"]}
    per = {}
    for r in trace:
        if r[6] == T["PBFT_COMMIT"] and (r[0], r[9]) in t0:
            per.setdefault((r[0], r[9]), []).append(r[1] - t0[(r[0], r[9])])
    return [int(np.median(v)) for _, v in sorted(per.items())]


def _paxos(args):
    import oracle
    from bcsim import _abi
    from bcsim.montecarlo import commit_latencies
    k, seed = args
    return [int(x) for x in commit_latencies(oracle.run(paxos_cfg(k, seed, _abi.RNG_GLIBC))[0], _abi.PAXOS)]


def _pbft(seed):
    import oracle
    from bcsim import _abi
    return pbft_block_medians(oracle.run(pbft_cfg(seed, _abi.RNG_GLIBC))[0])


def main():
    with mp.get_context("spawn").Pool(min(8, os.cpu_count() or 1)) as pool:
        px = {k: pool.map(_paxos, [(k, s) for s in range(1, PAXOS_SEEDS + 1)]) for k in (1, 2)}
        pb = pool.map(_pbft, range(1, PBFT_SEEDS + 1))
    with open(os.path.join(HERE, "ks_c3_paxos4096.json"), "w") as f:
        json.dump({"n": 4096, "seeds": PAXOS_SEEDS, "rng": "glibc",
                   "latency_ns": {str(k): [x for run in v for x in run] for k, v in px.items()},
                   "per_seed": {str(k): v for k, v in px.items()}}, f)
    with open(os.path.join(HERE, "ks_pbft512.json"), "w") as f:
        json.dump({"n": 512, "seeds": PBFT_SEEDS, "rng": "glibc", "rounds": 5,
                   "block_median_ns": [x for run in pb for x in run], "per_seed": pb}, f)


if __name__ == "__main__":
    main()
