set -o pipefail
mkdir -p gpurun_out/ab15
bash tests/gpu_bisect.sh "gossip200_d8_jitter_ctr gossip24_mesh gossip512_d8_blocks gossip64_d4_b2 gossip64_d4_droptail gossip64_d4_fixed gossip64_d4_fq gossip96_d6_hetero_prop paxos8_fixed_k3 paxos32_jitter_ctr pbft16_fixed_100" "" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "c5" > gpurun_out/ab15/c5.log 2>&1; rc=$?; tail -2 gpurun_out/ab15/c5.log
[ $rc -eq 0 -o $rc -eq 1 ] || exit 1
for e in "" "BCSIM_GOSSIP_FRONTIER=0"; do
  env $e timeout -k 10 300 python bench.py --workload gossip --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/ab15/g_bench.log 2>&1 || exit 1
  echo "[$e] $(tail -1 gpurun_out/ab15/g_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4e msgs/s %.3f ms/step frac %.4f' % (d['value'], d['ms_per_step'], d['roofline']['frac']))")"
done
