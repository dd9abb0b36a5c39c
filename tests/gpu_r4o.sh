set -o pipefail
out=gpurun_out/r4o; mkdir -p $out
(while sleep 50; do date +%s >> $out/heartbeat; done) & hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gossip.py tests/test_fastpaths.py tests/test_sparse.py -k "gossip or fast or parity" -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit 1
for v in "" "BCSIM_NO_DEGREG=1" "" "BCSIM_NO_DEGREG=1"; do
  env $v timeout -k 10 240 python bench.py --workload gossip --steps 20 --warmup 5 --no-cpu-baseline > $out/gossip.log 2>&1 || exit 1
  echo "gossip [$v] $(tail -1 $out/gossip.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4e msgs/s %.3f ms/step' % (d['value'], d['ms_per_step']), d['breakdown']['kernel_us'])")"
done
