"""Child process of tests/test_switches.py: run parity cases under the environment it was
started with (the engine's A/B switches, some of which are read once per process) and check
each against the oracle.  Prints one line per case; exit status 0 when all match.

    BCSIM_SPIN=0 python tests/switch_run.py pbft16_fixed_100 gossip64_d4_fixed
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "blockchain-simulator_amd")]


def main(names):
    import bcsim
    import oracle
    from parity_cases import cases, compare, topology
    allc = cases()
    bad = 0
    for name in names:
        topo = topology(name)
        got = bcsim.run(allc[name], topology=topo)
        if got[2]["error"] != 0:
            print(f"ERROR {name}: status {got[2]}", flush=True)
            bad += 1
            continue
        d = compare(oracle.run(allc[name], topology=topo), got)
        print(f"{'OK' if d is None else 'DIFF'} {name}{'' if d is None else ': ' + str(d)}", flush=True)
        bad += d is not None
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
