set -o pipefail
mkdir -p gpurun_out/ab14
timeout -k 10 700 python -u -m pytest tests/test_fqcodel.py -m gpu -x -q --timeout 600 --timeout-method thread -k "fullsize" > gpurun_out/ab14/fqfull.log 2>&1; rc=$?; tail -3 gpurun_out/ab14/fqfull.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py --queue fqcodel --steps 3 --warmup 4 --cpu-budget 10 > gpurun_out/ab14/fq_bench.log 2>&1; rc=$?; tail -c 600 gpurun_out/ab14/fq_bench.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests/test_partition.py -m gpu -x -q --timeout 880 --timeout-method thread -k "c4_fq" > gpurun_out/ab14/fqpart.log 2>&1; tail -3 gpurun_out/ab14/fqpart.log
