set -o pipefail
mkdir -p gpurun_out/ab14
bash tests/gpu_bisect.sh "paxos8_fixed paxos8_fixed0 paxos8_fixed_k3 paxos16_jitter_rep4 paxos32_jitter_ctr paxos32_jitter_k4 paxos128_jitter_rep6_k3 paxos256_jitter_rep8 paxos32_fq_jitter" "" || exit 1
timeout -k 10 700 python -u -m pytest tests/test_fqcodel.py -m gpu -x -q --timeout 600 --timeout-method thread -k "fullsize" > gpurun_out/ab14/fqfull.log 2>&1; rc=$?; tail -3 gpurun_out/ab14/fqfull.log
[ $rc -eq 0 -o $rc -eq 1 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_sparse.py -m gpu -x -q --timeout 580 --timeout-method thread -k "c3_paxos4096_10k" > gpurun_out/ab14/c3.log 2>&1; rc=$?; tail -3 gpurun_out/ab14/c3.log
[ $rc -eq 0 -o $rc -eq 1 ] || exit 1
for e in "" "BCSIM_PX_FAST=0"; do
  env $e timeout -k 10 400 python bench.py --workload paxos --steps 3 --warmup 4 --no-cpu-baseline > gpurun_out/ab14/px_bench$([ -z "$e" ] && echo 1 || echo 0).log 2>&1 || exit 1
  echo "[$e] $(tail -1 gpurun_out/ab14/px_bench$([ -z "$e" ] && echo 1 || echo 0).log | cut -c1-200)"
done
timeout -k 10 600 python bench.py --queue fqcodel --steps 3 --warmup 4 --cpu-budget 10 > gpurun_out/ab14/fq_bench.log 2>&1; rc=$?; tail -c 400 gpurun_out/ab14/fq_bench.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests/test_partition.py -m gpu -x -q --timeout 880 --timeout-method thread -k "c4_fq" > gpurun_out/ab14/fqpart.log 2>&1; tail -3 gpurun_out/ab14/fqpart.log
