#!/bin/bash
# Quick parity + A/B against ab_lib/head.so (the last commit's engine, tools/build_variant.sh):
#   bash tests/gpu_ab_round.sh <tag> [workload]
set -o pipefail
tag=${1:-ab}; wl=${2:-pbft}
out=gpurun_out/$tag; mkdir -p $out
(while sleep 50; do date +%s >> $out/heartbeat; done) & hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_fastpaths.py tests/test_fullsize.py tests/test_gossip.py tests/test_sparse.py -m gpu -x -q --timeout 600 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit 1
bash tests/gpu_ab.sh $tag - "" "BCSIM_LIB=ab_lib/head.so" "" "BCSIM_LIB=ab_lib/head.so" "" "BCSIM_LIB=ab_lib/head.so" || exit 1
for v in "" "BCSIM_LIB=ab_lib/head.so" "" "BCSIM_LIB=ab_lib/head.so"; do
  env $v timeout -k 10 240 python bench.py --workload gossip --steps 20 --warmup 5 --no-cpu-baseline > $out/gossip.log 2>&1 || exit 1
  echo "gossip [$v] $(tail -1 $out/gossip.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4e msgs/s %.3f ms/step' % (d['value'], d['ms_per_step']))")"
done
