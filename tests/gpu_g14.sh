set -o pipefail
o=gpurun_out/g14; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gossip.py tests/test_headline_oracle.py -x -q --timeout 500 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for e in "" "BCSIM_CHAIN=0" "" "BCSIM_CHAIN=0"; do
  env $e timeout -k 10 200 python bench.py --workload gossip --no-cpu-baseline --steps 20 --warmup 5 > $o/g.log 2>&1 || exit 1
  echo "gossip [$e] $(tail -1 $o/g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3f ms/step' % d['ms_per_step'])")"
done
