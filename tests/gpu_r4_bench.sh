set -o pipefail
out=gpurun_out/r04bench; mkdir -p $out
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $secs "$@" > $out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 $out/$name.log | cut -c1-200
  [ $rc -eq 0 ] || exit 1
}
step bench_pbft 300 python bench.py --steps 20 --warmup 5
step bench_gossip 240 python bench.py --workload gossip
step bench_gossip_pdes1 240 python bench.py --workload gossip --pdes1 --no-cpu-baseline
step bench_paxos 400 python bench.py --workload paxos
step bench_pbft_jitter 300 python bench.py --jitter
step bench_pbft_fq 600 python bench.py --queue fqcodel --steps 3 --warmup 4 --cpu-budget 10
bash tests/gpu_prof.sh r04bench/prof --steps 20 --warmup 5 --no-cpu-baseline > $out/prof.log 2>&1; rc=$?; tail -3 $out/prof.log; exit $rc
