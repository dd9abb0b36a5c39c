#!/bin/bash
# GPU-box workgroup-size sweep of the PBFT n=4096 bench (BCSIM_BS_LINK / BCSIM_BS_SCAN caps),
# after a parity check of the capped (strided) path.  bash tests/gpu_tune.sh
set -o pipefail
mkdir -p gpurun_out/tune
timeout -k 10 240 env BCSIM_BS_LINK=64 BCSIM_BS_SCAN=64 python tests/parity_run.py pbft100_fixed pbft16_fixed_100 raft64_fixed paxos32_jitter_ctr gossip200_d8_jitter_ctr pbft8_rep3_ctr > gpurun_out/tune/parity64.log 2>&1 || { cat gpurun_out/tune/parity64.log; exit 1; }
cat gpurun_out/tune/parity64.log
timeout -k 10 120 python tests/parity_run.py pbft100_fixed > gpurun_out/tune/parity.log 2>&1 || { cat gpurun_out/tune/parity.log; exit 1; }
for cfg in "1024 1024" "512 1024" "256 1024" "1024 512" "1024 256" "512 512" "256 256"; do
  set -- $cfg
  timeout -k 10 120 env BCSIM_BS_LINK=$1 BCSIM_BS_SCAN=$2 python bench.py --no-cpu-baseline > gpurun_out/tune/b_$1_$2.log 2>&1 || exit 1
  echo "link=$1 scan=$2 $(grep '^{' gpurun_out/tune/b_$1_$2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e9,3), 'G msgs/s', d['kernel_us'])")"
done
