set -o pipefail
out=gpurun_out/ab17; mkdir -p $out
(while sleep 50; do date +%s >> $out/heartbeat; done) & hb=$!
trap "kill $hb 2>/dev/null" EXIT
bash tests/gpu_bisect.sh "pbft100_fixed pbft16_fixed_100 pbft8_fixed_40 pbft5_odd pbft512_small pbft8_noecho pbft12_hetero_prop pbft8_compat pbft8_rep3_ctr pbft12_jitter_b2 pbft16_fq_100 pbft16_droptail_100" "" "BCSIM_FEW_SCAN=0" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_fastpaths.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/fast.log 2>&1; rc=$?; tail -2 $out/fast.log
[ $rc -eq 0 -o $rc -eq 1 ] || exit 1
bash tests/gpu_ab.sh ab17 - "" "BCSIM_SROW=0" "" || exit 1
timeout -k 10 900 python -u -m pytest tests/test_partition.py -m gpu -x -q --timeout 880 --timeout-method thread -k "c4_fq" > $out/fqpart.log 2>&1; tail -3 $out/fqpart.log
