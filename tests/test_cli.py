"""The drop-in boundary as shipped: bcsim_cli (blockchain-simulator.cc written
against the NetworkHelper / PointToPointHelper facade, include/network_helper.hpp)
with per-link Delay attributes, so NetworkHelper::SetLinks feeds the per-edge
prop_ns path (prop_const = -1 in the engine).  Its stdout -- the reference's
NS_LOG_INFO lines plus a counters line -- must equal the oracle's run of the same
configuration formatted by the same trace writer."""
import os
import subprocess

import numpy as np
import pytest

import oracle
from bcsim import _abi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "blockchain-simulator_amd", "bcsim_cli")


def cli_topology(n, base_ns, spread_us):
    """The CLI's mesh (blockchain-simulator.cc:34-51 order) with the per-link delay it
    sets before each Install(i, j), j < i: base + 1 us * ((7 i + 3 j) mod (spread + 1))."""
    row = np.arange(n + 1, dtype=np.uint32) * (n - 1)
    col, prop = [], []
    for a in range(n):
        for b in range(n):
            if b == a:
                continue
            i, j = max(a, b), min(a, b)
            col.append(b)
            prop.append(base_ns + 1000 * ((i * 7 + j * 3) % (spread_us + 1)))
    return row, np.array(col, dtype=np.uint32), np.array(prop, dtype=np.int64)


@pytest.mark.gpu
@pytest.mark.parametrize("proto,n,extra", [("pbft", 8, ["--rounds", "12"]), ("raft", 8, [])])
def test_cli_matches_oracle_with_per_link_delays(engine_lib, proto, n, extra):
    import bcsim
    spread = 40
    args = [CLI, "--nodes", str(n), "--protocol", proto, "--fixed-app-delay-ns", "1000000",
            "--delay-spread-us", str(spread)] + extra
    out = subprocess.run(args, capture_output=True, text=True, timeout=120, check=True).stdout
    cfg = _abi.default_config(_abi.PBFT if proto == "pbft" else _abi.RAFT, n)
    cfg.delay_mode = _abi.DELAY_FIXED
    cfg.app_delay_ns = 1_000_000
    if proto == "pbft":
        cfg.pbft_rounds = 12
    else:
        cfg.t_end_ns = 20_000_000_000
    cfg.stop_ns = 10_000_000_000                    # nodeApp.Stop(Seconds(10)) :55
    row, col, prop = cli_topology(n, 3_000_000, spread)
    cfg.link_delay_ns = int(prop[-1])                # the helper's last Delay attribute
    tr, cnt, st = oracle.run(cfg, topology=(row, col, prop))
    assert st["error"] == 0 and len(tr) > 0
    want = "".join(bcsim.format_trace_line(r, cfg) + "\n" for r in tr)
    want += "delivered=%d echoes=%d sends=%d t_last_ns=%d\n" % (
        cnt["delivered_total"], cnt["echoes"], cnt["sends"], cnt["t_last_ns"])
    assert out == want
