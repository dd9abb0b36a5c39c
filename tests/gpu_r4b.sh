set -o pipefail
bash tests/gpu_bisect.sh "pbft100_fixed pbft16_fixed_100 pbft8_fixed_40 pbft5_odd pbft512_small pbft8_noecho pbft12_hetero_prop pbft8_compat pbft8_rep3_ctr pbft12_jitter_b2 raft64_fixed gossip64_d4_fixed" "" || exit 1
mkdir -p gpurun_out/ab13
timeout -k 10 400 python -u -m pytest tests/test_fastpaths.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab13/tests.log 2>&1; rc=$?; tail -2 gpurun_out/ab13/tests.log
[ $rc -eq 0 -o $rc -eq 1 ] || exit 1
bash tests/gpu_ab.sh ab13 - "" "BCSIM_L2_OVERLAP=0" "BCSIM_LIB=ab_lib/rtmaj.so" || exit 1
timeout -k 10 700 python -u -m pytest tests/test_fqcodel.py -m gpu -x -q --timeout 600 --timeout-method thread -k "fullsize" > gpurun_out/ab13/fqfull.log 2>&1; tail -3 gpurun_out/ab13/fqfull.log
