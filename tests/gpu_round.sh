#!/bin/bash
# Round-end GPU evidence: the GPU test suite, the bench lines of every workload (with the
# CPU baseline), and the rocprofv3 kernel trace + PMC passes of the headline.
#   bash tests/gpu_round.sh <tag> [noprof]     (outputs under gpurun_out/<tag>/)
#   (ONLY_PYTEST=1: the suite alone; SKIP_PYTEST=1: the rest -- two calls within gpurun's limit)
set -o pipefail
tag=${1:-round}
out=gpurun_out/$tag
mkdir -p $out
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $secs "$@" > $out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 $out/$name.log | cut -c1-300
  [ $rc -eq 0 ] || exit 1
}
(while sleep 50; do date +%s >> $out/heartbeat; done) & hb=$!
trap "kill $hb 2>/dev/null" EXIT
[ -n "$SKIP_PYTEST" ] || step pytest_gpu 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread
[ -n "$ONLY_PYTEST" ] && exit 0
step bench_pbft 240 python bench.py --steps 20 --warmup 5
step bench_gossip 240 python bench.py --workload gossip --steps 20 --warmup 5
step bench_gossip_pdes1 240 python bench.py --workload gossip --pdes1 --no-cpu-baseline --steps 20 --warmup 5
step bench_pbft_pdes1 240 python bench.py --pdes1 --no-cpu-baseline --steps 20 --warmup 5
step bench_paxos 300 python bench.py --workload paxos
step bench_pbft_jitter 240 python bench.py --jitter
step bench_pbft_fq 400 python bench.py --queue fqcodel --steps 20 --warmup 5 --cpu-budget 10
[ "$2" = "noprof" ] && exit 0
bash tests/gpu_prof_all.sh $tag/prof > $out/prof.log 2>&1 || { tail -5 $out/prof.log; exit 1; }
tail -3 $out/prof.log
