"""The engine's fast paths are on by default; each has an off switch that
selects the generic path it restates.  Every switch flipped alone must still give the oracle's
traces and counters -- run in a child process per switch, since some are read once per process
(BCSIM_SPIN, BCSIM_NO_ACTSYNC).  BCSIM_FEW_SCAN=0 puts even the small cases' heavy launches on
the wide-window kernels.  Also: a device error flag raised mid-run (BCSIM_DBG_DEV_ERR) makes
k_next / k_active bail, so the host's mirror spin must fall back to the copy read-back and the
run must end with that error instead of waiting for a mirror word that never comes."""
import os
import subprocess
import sys

import pytest


pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = ["pbft16_fixed_100", "pbft512_small", "pbft12_jitter_ctr", "gossip64_d4_fixed", "gossip512_d8_blocks",
         "paxos16_jitter_rep4", "raft64_fixed"]
SWITCHES = [
    {"BCSIM_L2_OVERLAP": "0"},      # list 2 scanned and linked on the engine stream
    {"BCSIM_CTL_MIRROR": "0"},      # control block read back by copies, no host-mapped mirror
    {"BCSIM_SPIN": "0"},            # plain stream syncs instead of the mirror spin
    {"BCSIM_NO_ACTSYNC": "1"},      # looped grids instead of exact list-length launches
    {"BCSIM_GOSSIP_FRONTIER": "0"}, # k_gossip_cell over every node, not the window's frontier
    {"BCSIM_NO_DEGREG": "1"},       # no regular-degree index arithmetic
    {"BCSIM_MESH_TILE": "0", "BCSIM_FEW_SCAN": "0"},  # k_link_mesh instead of the tiled mesh
    {"BCSIM_SUM": "0", "BCSIM_FEW_SCAN": "0"},        # no record summaries (k_mesh_tile, k_scan_pbft)
    {"BCSIM_NO_DESC": "1"},         # no reply / echo descriptors
    {"BCSIM_SPEC": "0"},            # no speculative k_active behind k_next
    {"BCSIM_L2_OVERLAP": "1"},      # list 2 on the second stream in every window (default: few-node scans)
    {"BCSIM_CHAIN": "0"},           # no device-chained gossip windows (one host sync per window)
    {"BCSIM_FUSE_ACT": "1"},        # k_next builds the speculative lists (opt-in)
    {"BCSIM_LINK_FEW": "0"},        # few-sender windows through k_mesh_prep + k_mesh_row too
]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("env", SWITCHES, ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
def test_switch_matches_oracle(env, engine_lib):
    r = subprocess.run([sys.executable, os.path.join(HERE, "switch_run.py")] + CASES, env={**os.environ, **env},
                       capture_output=True, text=True, timeout=840)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]


@pytest.mark.timeout(120)
@pytest.mark.parametrize("env", [{}, {"BCSIM_CTL_MIRROR": "0"}], ids=["mirror", "copy"])
def test_device_error_ends_run(env, engine_lib):
    import bcsim
    from parity_cases import cases
    old = {k: os.environ.get(k) for k in list(env) + ["BCSIM_DBG_DEV_ERR"]}
    os.environ.update(env, BCSIM_DBG_DEV_ERR="3")
    try:
        with pytest.raises(bcsim.EngineError) as ei:
            bcsim.run(cases()["pbft16_fixed_100"])
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert ei.value.code == -4  # BCSIM_E_OVERFLOW (injected)
