"""Debug aid: compare FQCODEL link-event logs of the engine (BCSIM_FQLOG) and the oracle
(ORACLE_FQLOG): per edge, the first event where the sequences differ (earliest first).
Usage: python tools/fq_log.py CASE T0 T1   (runs both to T1, logging events in [T0, T1))"""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "tests"), os.path.join(R, "blockchain-simulator_amd")]
KIND = {1: "enq", 2: "push", 3: "drop", 4: "wake"}


def load(path):
    a = np.fromfile(path, dtype=np.uint32).reshape(-1, 8)
    t = a[:, 0].astype(np.int64) | (a[:, 1].astype(np.int64) << 32)
    x = a[:, 5].astype(np.int64) | (a[:, 6].astype(np.int64) << 32)
    # (an echo's sub is not part of the model: the oracle logs 0)
    return [(int(t[k]), int(a[k, 2]), int(a[k, 3] >> 24), int(a[k, 3] & 0xFFFFFF), 0 if a[k, 7] else int(a[k, 4]),
             int(x[k]), int(a[k, 7])) for k in range(len(a))]


def main():
    name, t0, t1 = sys.argv[1], int(float(sys.argv[2])), int(float(sys.argv[3]))
    os.environ["BCSIM_FQLOG"] = "/tmp/fq_engine.bin"
    os.environ["ORACLE_FQLOG"] = "/tmp/fq_oracle.bin"
    os.environ["BCSIM_FQLOG_T0"] = str(t0)
    os.environ["BCSIM_FQLOG_T1"] = str(t1)
    import bcsim
    import oracle
    from parity_cases import any_case, topology
    cfg = any_case(name)
    cfg.t_end_ns = t1
    topo = topology(name)
    oracle.run(cfg, topology=topo)
    bcsim.run(cfg, topology=topo)
    eng, ora = load("/tmp/fq_engine.bin"), load("/tmp/fq_oracle.bin")
    print(f"events: engine {len(eng)}, oracle {len(ora)}")
    by = {}
    for src, log in (("e", eng), ("o", ora)):
        for r in log:
            by.setdefault(r[1], {"e": [], "o": []})[src].append(r)
    first = []
    for edge, d in by.items():
        e, o = d["e"], d["o"]
        # (lazy wakes of an empty disc: the engine applies them at the link's next use only)
        k = 0
        # (engine enqueue records carry the op source in x >> 8)
        e = [r if r[2] != 1 else r[:5] + (r[5] & 0xFF,) + r[6:] for r in e]
        while k < min(len(e), len(o)) and e[k] == o[k]:
            k += 1
        if k < max(len(e), len(o)):
            t = min(e[k][0] if k < len(e) else 1 << 62, o[k][0] if k < len(o) else 1 << 62)
            if k >= len(e) and all(r[2] == 4 for r in o[k:]):
                continue
            first.append((t, edge, k))
    first.sort()
    print(f"edges differing: {len(first)} of {len(by)}")
    for t, edge, k in first[:3]:
        e, o = by[edge]["e"], by[edge]["o"]
        print(f"edge {edge}: first difference at index {k} (t={t / 1e9:.9f})")
        for j in range(max(0, k - 4), k + int(os.environ.get('FQ_AFTER', '6'))):
            fe = e[j] if j < len(e) else None
            fo = o[j] if j < len(o) else None
            fmt = lambda r: "-" if r is None else f"{r[0] / 1e9:.9f} {KIND[r[2]]:4s} fr={r[3]:2d} sub={r[4]:6d} x={r[5]} echo={r[6]}"
            print(f"  {'*' if j == k else ' '} E {fmt(fe):70s} | O {fmt(fo)}")


if __name__ == "__main__":
    main()
