set -o pipefail
o=gpurun_out/final6; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -30 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $o/bench_pbft.log 2>&1 || exit 1
tail -1 $o/bench_pbft.log | cut -c1-300
timeout -k 10 240 python bench.py --workload gossip --steps 20 --warmup 5 --no-cpu-baseline > $o/bench_gossip.log 2>&1 || exit 1
tail -1 $o/bench_gossip.log | cut -c1-300
