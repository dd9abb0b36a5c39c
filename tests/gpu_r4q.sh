set -o pipefail
out=gpurun_out/r4q; mkdir -p $out
(while sleep 50; do date +%s >> $out/heartbeat; done) & hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?; tail -3 $out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
bash tests/gpu_ab.sh ab25 - "" "BCSIM_LIB=ab_lib/head.so" "" "BCSIM_LIB=ab_lib/head.so" || exit 1
for v in "" "BCSIM_LIB=ab_lib/head.so"; do
  env $v timeout -k 10 240 python bench.py --workload gossip --steps 20 --warmup 5 --no-cpu-baseline > $out/gossip.log 2>&1 || exit 1
  echo "gossip [$v] $(tail -1 $out/gossip.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4e msgs/s %.3f ms/step' % (d['value'], d['ms_per_step']))")"
done
bash tests/gpu_r4_bench.sh || exit 1
