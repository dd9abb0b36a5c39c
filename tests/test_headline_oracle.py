"""The headline path against the oracle at full size (VERDICT r5 "next" #2).

bench.py times PBFT n=4096 on the full mesh (BASELINE configs[3]) through summary entries,
k_mesh_row, k_scan_rt, the speculative k_active behind k_next and the idle-part skip, driven in
50 ms `run(t)` steps.  Here exactly that run (tests/headline_run.py, one child process per engine
switch setting) is compared with the oracle's one-shot run of the same horizon -- 6 steps, 300 ms
simulated, past the first COMMIT wave -- traces and counters bit for bit, once as the bench runs
it (with every skipped idle part re-checked by k_active, BCSIM_CHECK_IDLE=1), once without
summaries (BCSIM_SUM=0) and once without speculation (BCSIM_SPEC=0).  The small parity cases are
driven the same way (run limits mid-cell), speculation on and off.
Reference: pbft-node.cc:166-265 (handlers), :371-411 (SendBlock), blockchain-simulator.cc:34-57.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
STEPS = 6


def _child(args, env, timeout):
    r = subprocess.run([sys.executable, os.path.join(HERE, "headline_run.py")] + args, env={**os.environ, **env},
                       capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    return [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]


@pytest.fixture(scope="module")
def oracle_cache(tmp_path_factory):
    return str(tmp_path_factory.mktemp("headline") / "oracle_c4_6steps.npz")


@pytest.mark.timeout(900)
@pytest.mark.parametrize("env", [{"BCSIM_CHECK_IDLE": "1"}, {"BCSIM_SUM": "0"}, {"BCSIM_SPEC": "0"}],
                         ids=["bench_path", "sum_off", "spec_off"])
def test_c4_pbft4096_bench_steps_match_oracle(env, oracle_cache, engine_lib):
    out = _child([str(STEPS), oracle_cache], env, 840)[-1]
    assert out["diff"] is None, out
    assert out["delivered"] > 50_000_000, out          # past the first PREPARE / COMMIT waves
    if env.get("BCSIM_CHECK_IDLE") == "1":
        assert out["spec_hits"] > 0, out                 # the speculative lists were used
        assert out["idle_parts"] > 0, out                # and idle parts were skipped ...
        assert out["idle_checked"] == out["idle_parts"], out  # ... each verified empty
    if env.get("BCSIM_SPEC") == "0":
        assert out["spec_hits"] == 0, out


@pytest.mark.timeout(600)
@pytest.mark.parametrize("env", [{"BCSIM_CHECK_IDLE": "1"}, {"BCSIM_SPEC": "0", "BCSIM_CHAIN": "0"}],
                         ids=["spec_chain_on", "spec_chain_off"])
def test_small_cases_in_bench_steps_match_oracle(env, engine_lib):
    """PBFT (speculative k_active, idle parts) and gossip (device-chained windows, DESIGN.md §4.2b:
    k_win decides the windows on the device, the run limit ends a chain mid-cell) in 50 ms steps."""
    outs = _child(["cases", "pbft16_fixed_100", "pbft512_small", "pbft100_fixed", "pbft8_rep3_ctr",
                   "gossip64_d4_fixed", "gossip512_d8_blocks", "gossip200_d8_jitter_ctr"], env, 560)
    assert all(o["diff"] is None for o in outs), outs
    gossip = [o for o in outs if o["case"].startswith("gossip") and "jitter" not in o["case"]]
    if env.get("BCSIM_CHECK_IDLE") == "1":
        assert sum(o["spec_hits"] for o in outs) > 0, outs
        assert all(o["idle_checked"] == o["idle_parts"] for o in outs), outs
        assert all(o["chain_windows"] > 0 for o in gossip), gossip           # chains ran (and ended) ...
        assert sum(o["frontier_hits"] for o in gossip) > 0, gossip           # k_next built frontiers
        assert sum(o["host_syncs"] for o in gossip) < sum(o["windows"] for o in gossip), gossip  # fewer syncs
    else:
        assert all(o["chain_windows"] == 0 for o in outs), outs
