"""Child process of tests/test_headline_oracle.py: the bench's exact configuration (PBFT n=4096
full mesh, bcsim.preset("c4_pbft4096") as bench.py builds it) driven the way bench.py drives it --
Simulator.run(t) in 50 ms block-interval steps -- under the engine switches of this process's
environment, against the oracle's one-shot run of the same horizon: traces and counters bit for bit.

    python tests/headline_run.py <steps> <oracle.npz|->
    python tests/headline_run.py cases <name> ...     (parity cases, stepped the same way)

The oracle run (~1 min at 6 steps) is cached in <oracle.npz> by the first child and reused by the
next (each switch setting is its own process: some switches are read once per process).  Prints
the loop statistics (windows, speculative hits, idle parts, host syncs) as one JSON line.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "blockchain-simulator_amd")]

PERIOD = 50_000_001  # Seconds(0.05f) in ns (bench.py)


def config(steps):
    import bcsim
    c = bcsim.preset("c4_pbft4096")
    c.stop_ns = -1                      # bench.py make_cfg
    c.pbft_rounds = 5 + 2 * 20 + 4      # bench.py's default driver run (--steps 20 --warmup 5)
    c.t_end_ns = steps * PERIOD
    return c


def oracle_result(c, path):
    import numpy as np
    if path != "-" and os.path.exists(path):
        z = np.load(path, allow_pickle=False)
        trace = [tuple(int(v) for v in r) for r in z["trace"]]
        return trace, json.loads(str(z["counters"]))
    import oracle
    trace, counters = oracle.run(c)[:2]
    if path != "-":
        np.savez(path, trace=np.array(trace, dtype=np.int64), counters=json.dumps(counters))
    return trace, counters


def stepped_cases(names):
    """Parity cases driven in 50 ms run() steps until quiescent (the speculative
    k_active state and the idle-part skip only act when a run stops mid-cell), then to the end,
    against the oracle's one-shot run."""
    import bcsim
    import oracle
    from parity_cases import cases, compare, topology
    allc = cases()
    bad = 0
    for name in names:
        c, topo = allc[name], topology(name)
        with bcsim.Simulator(c) as sim:
            if topo is not None:
                sim.set_topology(*topo)
            k = 0
            while not sim.status()["quiescent"] and k < 400:
                k += 1
                sim.run(k * PERIOD)
            sim.run()
            got = (sim.trace(), sim.counters(), sim.status())
            ls = sim.loop_stats()
            ls["frontier_hits"] = sim.host_stats()["frontier_hits"]
        d = compare(oracle.run(c, topology=topo), got) if got[2]["error"] == 0 else f"status {got[2]}"
        print(json.dumps({"case": name, "steps": k, "diff": d, **ls}), flush=True)
        bad += d is not None
    return 1 if bad else 0


def main():
    if sys.argv[1] == "cases":
        return stepped_cases(sys.argv[2:])
    steps = int(sys.argv[1])
    path = sys.argv[2]
    import bcsim
    from parity_cases import compare
    c = config(steps)
    with bcsim.Simulator(c) as sim:
        for k in range(1, steps + 1):
            sim.run(k * PERIOD)
        got = (sim.trace(), sim.counters(), sim.status())
        ls = sim.loop_stats()
    assert got[2]["error"] == 0, got[2]
    want = oracle_result(c, path)
    d = compare(want, got)
    print(json.dumps({"diff": d, "delivered": got[1]["delivered_total"], "trace": len(got[0]), **ls}), flush=True)
    return 0 if d is None else 1


if __name__ == "__main__":
    sys.exit(main())
