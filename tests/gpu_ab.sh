#!/bin/bash
# GPU A/B: a test selection, then the PBFT bench under each env setting given (one line each).
#   bash tests/gpu_ab.sh <tag> "<pytest args>" "" "BCSIM_MESH_TILE=0" ...
# ("-" as pytest args: no tests)
set -o pipefail
tag=$1; tests=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
if [ "$tests" != "-" ]; then
  timeout -k 10 600 python -u -m pytest $tests -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1
  rc=$?; tail -3 $out/tests.log
  [ $rc -eq 0 ] || exit 1
fi
k=0
for envs in "$@"; do
  k=$((k + 1))
  env $envs timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/bench$k.log 2>&1 || { echo "bench [$envs] failed"; tail -5 $out/bench$k.log; exit 1; }
  echo "[$envs] $(tail -1 $out/bench$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4e msgs/s %.3f ms/step link %.1f us/launch frac %.3f' % (d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac']), {k: round(v) for k, v in d['breakdown']['kernel_us'].items()})")"
done
