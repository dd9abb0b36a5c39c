set -o pipefail
out=gpurun_out/r03h; mkdir -p $out
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $out/bench_pbft.log 2>&1 || exit 1
tail -1 $out/bench_pbft.log | cut -c1-400
timeout -k 10 240 python bench.py --workload gossip --no-cpu-baseline > $out/bench_gossip.log 2>&1 || exit 1
tail -1 $out/bench_gossip.log | cut -c1-300
timeout -k 10 300 python bench.py --workload paxos --no-cpu-baseline > $out/bench_paxos.log 2>&1 || exit 1
tail -1 $out/bench_paxos.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/trace.log 2>&1 || exit 1
find $out -name "*stats*"
