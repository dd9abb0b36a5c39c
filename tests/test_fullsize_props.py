"""The bench-configuration properties (tests/fullsize_props.py) hold for the oracle
itself at small n, so they are the reference's behaviour, not the engine's (CPU)."""
import pytest

import oracle
from fullsize_props import bench_config, check_bench_config


@pytest.mark.parametrize("n", [16, 64])
def test_bench_config_properties_hold_for_oracle(n):
    c = bench_config(n)
    tr, cnt, st = oracle.run(c)
    check_bench_config(tr, cnt, st, c)
