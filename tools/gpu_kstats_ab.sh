#!/bin/bash
# A/B of the kernel-class event timing cost (BCSIM_KSTATS bit mask over scan/link/group/aux)
set -o pipefail
for wl in pbft gossip; do
  for m in 15 2 0; do
    BCSIM_KSTATS=$m timeout -k 10 200 python bench.py --workload $wl --no-cpu-baseline > gpurun_out/ks_${wl}_$m.log 2>&1 || { tail -5 gpurun_out/ks_${wl}_$m.log; exit 1; }
    echo "== $wl KSTATS=$m"; tail -1 gpurun_out/ks_${wl}_$m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3e' % d['value'], round(d['ms_per_step'],3), {k: round(v) for k, v in d['kernel_us'].items()})"
  done
done
