set -o pipefail
bash tests/gpu_bisect.sh "raft64_fixed raft16_fq_flows2 gossip64_d4_fixed pbft100_fixed pbft16_fixed_100 pbft8_fixed_40 pbft5_odd pbft512_small pbft8_noecho pbft12_hetero_prop pbft8_compat pbft8_rep3_ctr paxos32_jitter_ctr pbft12_jitter_b2 pbft16_fq_100" "" || exit 1
mkdir -p gpurun_out/ab12
timeout -k 10 400 python -u -m pytest tests/test_fastpaths.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab12/tests.log 2>&1; rc=$?; tail -2 gpurun_out/ab12/tests.log
[ $rc -eq 0 -o $rc -eq 1 ] || exit 1
bash tests/gpu_ab.sh ab12 - "" "BCSIM_L2_OVERLAP=0" "BCSIM_LIB=ab_lib/libbcsim_tile2.so BCSIM_L2_OVERLAP=0" "BCSIM_LIB=ab_lib/ts32.so BCSIM_L2_OVERLAP=0" "BCSIM_LIB=ab_lib/nodefer.so BCSIM_L2_OVERLAP=0" "BCSIM_LIB=ab_lib/ts32nd.so BCSIM_L2_OVERLAP=0" "BCSIM_LIB=ab_lib/ts32nd.so" || exit 1
bash tests/gpu_trace.sh tr12 ""
