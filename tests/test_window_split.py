"""k_scan window splitting (engine.hip window_split): a node with more arrivals in a cell than
its LDS staging holds (cap_arr) processes them in several time windows.  At N=4096 that is the
PBFT leader's heavy cells; here BCSIM_CAP_ARR=64 (128) forces it on jittered cases of degree > 64,
which must stay bit-exact against the oracle (the window bound is the largest end time with at
most cap arrivals, as the binary search it replaced found)."""
import pytest

import oracle
from bcsim import _abi
from parity_cases import _cfg, cases, compare

pytestmark = pytest.mark.gpu

# name -> (config or None for the parity case of that name, staging capacity, must split).
# The capacity must still hold every arrival of one instant.  PBFT with getRandomDelay():
# a node's PREPAREs arrive on three instants 1 ms apart (~N/3 each), and a cell
# (L ~ 3.1 ms) holds at least two of them, so cap < 2N/3 splits; Raft's three jitter values
# put ~85 of 255 heartbeat replies on one instant; Paxos responses spread over 50 ms
# (run for parity with the smallest window, whether or not a cell overflows it).
SPLIT_CASES = {
    "pbft100_jitter_ctr": (_cfg(_abi.PBFT, 100, delay_mode=_abi.DELAY_RANDOM, rng_mode=_abi.RNG_COUNTER, seed=3,
                                pbft_rounds=4, pbft_block_bytes=3000), 64, True),
    "pbft200_jitter_ctr": (_cfg(_abi.PBFT, 200, delay_mode=_abi.DELAY_RANDOM, rng_mode=_abi.RNG_COUNTER, seed=8,
                                pbft_rounds=3, pbft_block_bytes=2000), 128, True),
    "raft256_jitter_ctr": (_cfg(_abi.RAFT, 256, delay_mode=_abi.DELAY_RANDOM, rng_mode=_abi.RNG_COUNTER, seed=6,
                                t_end_ns=2_000_000_000, cap_ops_per_node=8192), 128, False),
    "paxos256_jitter_rep8": (None, 64, False),
}


@pytest.mark.parametrize("name", sorted(SPLIT_CASES))
def test_split_windows_match_oracle(name, engine_lib, monkeypatch):
    import bcsim
    cfg, cap, must_split = SPLIT_CASES[name]
    cfg = cfg or cases()[name]
    ref = oracle.run(cfg)
    assert ref[2]["error"] == 0
    monkeypatch.setenv("BCSIM_CAP_ARR", str(cap))
    with bcsim.Simulator(cfg) as s:
        s.run()
        got = (s.trace(), s.counters(), s.status())
        split = s.engine_counters()["split_windows"]
    diff = compare(ref, got)
    assert diff is None, f"{name}: {diff}"
    assert len(got[0]) > 0
    assert split > 0 or not must_split, f"{name}: no window was split (the case does not exercise window_split)"
