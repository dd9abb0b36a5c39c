import sys, time, traceback
import os; R=os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path[:0]=[R, os.path.join(R,'tests'), os.path.join(R,'blockchain-simulator_amd')]
import oracle, bcsim
from parity_cases import cases as _cases, fq_cases, compare, topology
def cases():
    c = _cases(); c.update(fq_cases()); return c
ok = 0
sel = sys.argv[1:]
for name, cfg in sorted(cases().items()):
    if sel and name not in sel: continue
    try:
        t0 = time.time(); topo = topology(name); ref = oracle.run(cfg, topology=topo); t1 = time.time()
        got = bcsim.run(cfg, topology=topo); t2 = time.time()
        d = compare(ref, got)
        print(f"{name:24s} {'OK ' if d is None else 'BAD'} ntr={len(ref[0])}/{len(got[0])} deliv={ref[1]['delivered_total']}/{got[1]['delivered_total']} cpu={t1-t0:.2f}s gpu={t2-t1:.2f}s {d or ''}", flush=True)
        ok += d is None
    except Exception as e:
        print(f"{name:24s} EXC {e}", flush=True)
        if "E_HIP" in str(e) or "illegal" in str(e):
            sys.exit(3)
print("passed", ok)
sys.exit(0 if ok == sum(1 for n in cases() if not sel or n in sel) else 1)
