"""Debug aid: fresh one-shot runs of the engine and the oracle to t_end = T for a grid of T;
prints the counters that differ at each T (case, t0, t1, step in ns)."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "tests"), os.path.join(R, "blockchain-simulator_amd")]
import bcsim  # noqa: E402
import oracle  # noqa: E402
from parity_cases import any_case, compare, topology  # noqa: E402

KEYS = ("delivered_total", "echoes", "sends", "frames_dropped", "msgs_lost", "events")
name, t0, t1, dt = sys.argv[1], int(float(sys.argv[2])), int(float(sys.argv[3])), int(float(sys.argv[4]))
topo = topology(name)
for T in range(t0, t1 + 1, dt):
    cfg = any_case(name)
    cfg.t_end_ns = T
    a = oracle.run(cfg, topology=topo)
    b = bcsim.run(cfg, topology=topo)
    d = {k: (a[1][k], b[1][k]) for k in KEYS if a[1][k] != b[1][k]}
    tr = compare(a, b)
    print(f"T={T / 1e9:.6f} {'EQUAL' if tr is None else 'DIFF'} {d} {'' if tr is None else tr[:200]}", flush=True)
