"""DEBUG/MEASUREMENT: run BASELINE configs[2] (Paxos n=4096, jittered links,
multi-decree, R replicas) in 50 ms simulated slices and print progress.

  python tools/c3_probe.py R K [engine_mode]
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "blockchain-simulator_amd")]
import bcsim  # noqa: E402
from bcsim import _abi  # noqa: E402

R, K = int(sys.argv[1]), int(sys.argv[2])
mode = int(sys.argv[3]) if len(sys.argv) > 3 else _abi.ENGINE_SPARSE
n = int(os.environ.get("C3_N", "4096"))
c = bcsim.preset("c3_paxos")
c.n_nodes = n
c.n_replicas = R
c.paxos_decrees = K
c.seed = 5
c.engine_mode = mode
t0 = time.time()
with bcsim.Simulator(c) as s:
    t = 0
    while True:
        t += 50_000_000
        w = time.time()
        s.run(t)
        cnt, st = s.counters(), s.status()
        ks = s.kernel_stats()
        if (t // 50_000_000) % 4 == 0:
            tr = s.trace()
            com = {r[0] for r in tr if r[6] == _abi.TR["PAXOS_COMMIT"]}
            print(f"  replicas with a commit: {len(com)} / {R}", flush=True)
        print(f"t={t / 1e6:.0f}ms wall={time.time() - w:.2f}s msgs={cnt['delivered_total']} cells={st['cells']} "
              f"quiescent={st['quiescent']} " + " ".join(f"{k}={v['us'] / 1e3:.1f}ms/{v['launches']}" for k, v in ks.items()),
              flush=True)
        if st["quiescent"] or time.time() - t0 > 150:
            break
    print(f"total {time.time() - t0:.1f}s msgs={cnt['delivered_total']} rate={cnt['delivered_total'] / (time.time() - t0):.3e}/s",
          flush=True)
