set -o pipefail
out=gpurun_out/r4k; mkdir -p $out
(while sleep 50; do date +%s >> $out/heartbeat; done) & hb=$!
trap "kill $hb 2>/dev/null" EXIT
bash tests/gpu_bisect.sh "pbft100_fixed pbft16_fixed_100 pbft8_fixed_40 pbft512_small pbft12_jitter_b2 pbft16_fq_100 paxos32_jitter_k4 paxos128_jitter_rep6_k3" "" || exit 1
timeout -k 10 1000 python -u -m pytest tests/test_partition.py -m gpu -x -v --timeout 900 --timeout-method thread > $out/part.log 2>&1; rc=$?; tail -4 $out/part.log; [ $rc -eq 0 ] || exit 1
bash tests/gpu_ab.sh ab21 - "" "BCSIM_SPIN=0" "" "BCSIM_SPIN=0" || exit 1
for v in "" "BCSIM_SPIN=0"; do
  env $v timeout -k 10 240 python bench.py --workload gossip --steps 20 --warmup 5 --no-cpu-baseline > $out/gossip.log 2>&1 || exit 1
  echo "gossip [$v] $(tail -1 $out/gossip.log | cut -c1-200)"
done
bash tests/gpu_ab.sh ab22 - "BCSIM_LIB=ab_lib/nospec.so" "" "BCSIM_LIB=ab_lib/nospec.so" "" || exit 1
BCSIM_WGT=1 timeout -k 10 240 python bench.py --steps 3 --warmup 3 --no-cpu-baseline > $out/wgt.log 2>&1 || exit 1
grep -c wgs $out/wgt.log
