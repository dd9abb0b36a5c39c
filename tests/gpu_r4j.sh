set -o pipefail
out=gpurun_out/r04bench; mkdir -p $out
(while sleep 50; do date +%s >> $out/heartbeat; done) & hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 600 python bench.py --queue fqcodel --steps 3 --warmup 4 --cpu-budget 10 > $out/bench_pbft_fq.log 2>&1; rc=$?; tail -c 300 $out/bench_pbft_fq.log; [ $rc -eq 0 ] || exit 1
bash tests/gpu_prof.sh r04bench/prof --steps 20 --warmup 5 --no-cpu-baseline > $out/prof.log 2>&1; rc=$?; tail -3 $out/prof.log; [ $rc -eq 0 ] || exit 1
bash tests/gpu_r4i.sh || exit 1
timeout -k 10 1000 python -u -m pytest tests/test_partition.py -m gpu -x -v --timeout 900 --timeout-method thread > $out/part.log 2>&1; tail -4 $out/part.log
