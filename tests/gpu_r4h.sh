set -o pipefail
out=gpurun_out/ab19; mkdir -p $out
(while sleep 50; do date +%s >> $out/heartbeat; done) & hb=$!
trap "kill $hb 2>/dev/null" EXIT
bash tests/gpu_bisect.sh "pbft100_fixed pbft16_fixed_100 pbft8_fixed_40 pbft512_small pbft12_jitter_b2 pbft16_fq_100 raft64_fixed raft16_fixed_b2 paxos32_jitter_ctr paxos8_fixed_k3 gossip64_d4_fixed gossip200_d8_jitter_ctr gossip64_d4_b2" "" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_fastpaths.py tests/test_window_split.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/fast.log 2>&1; rc=$?; tail -2 $out/fast.log
[ $rc -eq 0 -o $rc -eq 1 ] || exit 1
bash tests/gpu_ab.sh ab19 - "" "BCSIM_CTL_MIRROR=0" || exit 1
for e in "" "BCSIM_CTL_MIRROR=0"; do
  env $e timeout -k 10 300 python bench.py --workload gossip --steps 10 --warmup 5 --no-cpu-baseline > $out/g_bench.log 2>&1 || exit 1
  echo "gossip [$e] $(tail -1 $out/g_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4e msgs/s %.3f ms/step frac %.4f' % (d['value'], d['ms_per_step'], d['roofline']['frac']))")"
done
