set -o pipefail
out=gpurun_out/ab16; mkdir -p $out
(while sleep 50; do date +%s >> $out/heartbeat; done) & hb=$!
trap "kill $hb 2>/dev/null" EXIT
bash tests/gpu_bisect.sh "gossip200_d8_jitter_ctr gossip24_mesh gossip512_d8_blocks gossip64_d4_b2 gossip64_d4_droptail gossip64_d4_fixed gossip64_d4_fq gossip96_d6_hetero_prop paxos8_fixed_k3 paxos32_jitter_ctr pbft16_fixed_100 pbft16_fq_100 pbft12_fq_jitter raft16_fq_flows2" "" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_fqcodel.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/fq.log 2>&1; rc=$?; tail -2 $out/fq.log
[ $rc -eq 0 -o $rc -eq 1 ] || exit 1
timeout -k 10 400 python -u -m pytest tests/test_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c5" > $out/c5.log 2>&1; rc=$?; tail -2 $out/c5.log
[ $rc -eq 0 -o $rc -eq 1 ] || exit 1
for e in "" "BCSIM_GOSSIP_FRONTIER=0"; do
  env $e timeout -k 10 300 python bench.py --workload gossip --steps 10 --warmup 5 --no-cpu-baseline > $out/g_bench.log 2>&1 || exit 1
  echo "gossip [$e] $(tail -1 $out/g_bench.log | cut -c1-160) $(tail -1 $out/g_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3f ms/step frac %.4f' % (d['ms_per_step'], d['roofline']['frac']))")"
done
for e in "" "BCSIM_PX_FAST=0"; do
  env $e timeout -k 10 400 python bench.py --workload paxos --steps 3 --warmup 4 --no-cpu-baseline > $out/px_bench.log 2>&1 || exit 1
  echo "paxos [$e] $(tail -1 $out/px_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4e msgs/s %.1f ms/step frac %.4f' % (d['value'], d['ms_per_step'], d['roofline']['frac']))")"
done
timeout -k 10 200 python -u tests/c3_probe.py > $out/c3_probe.log 2>&1; tail -3 $out/c3_probe.log
timeout -k 10 600 python bench.py --queue fqcodel --steps 3 --warmup 4 --cpu-budget 10 > $out/fq_bench.log 2>&1; rc=$?; tail -c 300 $out/fq_bench.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests/test_partition.py -m gpu -x -q --timeout 880 --timeout-method thread -k "c4_fq" > $out/fqpart.log 2>&1; tail -3 $out/fqpart.log
