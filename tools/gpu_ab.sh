#!/bin/bash
# GPU A/B helper: parity suite, then the PBFT bench under each env setting given
#   bash tools/gpu_ab.sh "" "BCSIM_BS_LINK=512" ...
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/parity.log 2>&1
rc=$?; tail -2 gpurun_out/parity.log; [ $rc -eq 0 ] || exit 1
k=0
for e in "$@"; do
  k=$((k+1))
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/ab$k.log 2>&1 || { tail -5 gpurun_out/ab$k.log; exit 1; }
  echo "== [$e]"; tail -1 gpurun_out/ab$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3e' % d['value'], round(d['ms_per_step'],3), {k: round(v) for k, v in d['kernel_us'].items()})"
done
