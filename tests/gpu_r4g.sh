set -o pipefail
out=gpurun_out/ab18; mkdir -p $out
(while sleep 50; do date +%s >> $out/heartbeat; done) & hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 900 python -u -m pytest tests/test_sparse.py -m gpu -x -v --timeout 600 --timeout-method thread -k "c3_paxos4096" > $out/c3.log 2>&1; rc=$?; tail -4 $out/c3.log
[ $rc -eq 0 -o $rc -eq 1 ] || exit 1
timeout -k 10 400 python -u -m pytest tests/test_fqcodel.py -m gpu -x -q --timeout 300 --timeout-method thread -k fullsize > $out/fq.log 2>&1; rc=$?; tail -2 $out/fq.log
[ $rc -eq 0 -o $rc -eq 1 ] || exit 1
timeout -k 10 900 python -u -m pytest tests/test_partition.py -m gpu -x -q --timeout 880 --timeout-method thread -k "c4_fq" > $out/fqpart.log 2>&1; rc=$?; tail -3 $out/fqpart.log
[ $rc -eq 0 -o $rc -eq 1 ] || exit 1
bash tests/gpu_trace.sh trg "" "--workload gossip"
