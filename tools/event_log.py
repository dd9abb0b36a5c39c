"""DEBUG-ONLY: dump the engine's per-event log (BCSIM_DBG_EVENTS) of a Raft run.

  BCSIM_DBG_EVENTS=<t_max_ns> python tools/event_log.py N T_END_NS OUT.json [app_delay_ns]

Every Raft/Paxos/gossip event handled before t_max adds one trace record of
kind 90 + class (0 arrival, 1 timer, 2 start, 3 stop) with the node state
after the event; diff the files of two builds (GPU vs tools/hipemu).
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "blockchain-simulator_amd")]
import bcsim  # noqa: E402
from bcsim import _abi  # noqa: E402

n, tend, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
ad = int(sys.argv[4]) if len(sys.argv) > 4 else 1_000_000
c = _abi.default_config(_abi.RAFT, n)
c.delay_mode = _abi.DELAY_FIXED
c.app_delay_ns = ad
c.t_end_ns = tend
c.cap_ops_per_node = 8192
tr, cnt, st = bcsim.run(c)
ev = sorted(r for r in tr if r[6] >= 90)
with open(out, "w") as f:
    json.dump(dict(trace=[r for r in tr if r[6] < 90], events=ev, counters=cnt), f)
print(len(ev), "events,", len(tr) - len(ev), "trace records ->", out)
