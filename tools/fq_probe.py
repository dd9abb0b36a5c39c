"""Debug aid: step the HIP engine and the CPU oracle side by side in fixed increments of
simulated time and report the first checkpoint whose counters differ (one case per arg)."""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "tests"), os.path.join(R, "blockchain-simulator_amd")]
import bcsim  # noqa: E402
import oracle  # noqa: E402
from parity_cases import any_case, topology  # noqa: E402

KEYS = ("delivered_total", "echoes", "sends", "frames_dropped", "msgs_lost", "events")
step = int(os.environ.get("STEP_NS", "50000000"))
for name in sys.argv[1:]:
    cfg = any_case(name)
    topo = topology(name)
    t_end = cfg.t_end_ns if cfg.t_end_ns > 0 else cfg.stop_ns
    with bcsim.Simulator(cfg) as g, oracle.OracleSim(cfg) as o:
        if topo is not None:
            g.set_topology(*topo)
            o.set_topology(*topo)
        t, prev = 0, None
        while t < t_end:
            t = min(t + step, t_end)
            g.run(t)
            o.run(t)
            cg, co = g.counters(), o.counters()
            d = {k: (co[k], cg[k]) for k in KEYS if cg[k] != co[k]}
            if d:
                print(f"{name}: first difference by t={t / 1e9:.3f}s (previous checkpoint equal): {d}")
                print("   oracle", {k: co[k] for k in KEYS}, "\n   engine", {k: cg[k] for k in KEYS})
                print("   previous", prev)
                break
            prev = {k: co[k] for k in KEYS}
        else:
            print(f"{name}: equal at every checkpoint up to {t_end / 1e9:.3f}s")
    sys.stdout.flush()
