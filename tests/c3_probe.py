"""GPU probe: the configs[2] batch (Paxos n=4096, 10k replicas, 2 decrees) run in 200 ms chunks
toward quiescence, printing wall time and state per chunk (sizing the quiescence test)."""
import os, sys, time
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "tests"), os.path.join(R, "blockchain-simulator_amd")]
import bcsim
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
c = bcsim.preset("c3_paxos")
c.n_replicas = reps
c.paxos_decrees = 2
c.t_end_ns = 0
w0 = time.time()
with bcsim.Simulator(c) as s:
    t = 0
    while True:
        t += 200_000_000
        s.run(t)
        st, cnt = s.status(), s.counters()
        d = cnt["delivered"]
        print(f"t={t/1e9:.1f}s wall={time.time()-w0:.1f}s q={st['quiescent']} d={d[:6]} dropped={cnt['dropped']}", flush=True)
        if st["quiescent"] or time.time() - w0 > 150 or t >= 12_000_000_000:
            break
