"""HIP engine vs CPU oracle: bit-exact traces and counters (fixed-delay and
counter-RNG jitter configs).  The oracle is the checker only."""
import pytest

import oracle
from parity_cases import cases, compare, topology

pytestmark = pytest.mark.gpu

CASES = cases()


@pytest.mark.parametrize("name", sorted(CASES))
def test_engine_matches_oracle(name, engine_lib):
    import bcsim
    cfg = CASES[name]
    topo = topology(name)
    ref = oracle.run(cfg, topology=topo)
    got = bcsim.run(cfg, topology=topo)
    assert ref[2]["error"] == 0
    diff = compare(ref, got)
    assert diff is None, f"{name}: {diff}"
    assert len(got[0]) > 0
