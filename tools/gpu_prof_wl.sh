# rocprofv3 kernel stats of the gossip and Paxos benches (one run each)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/profwl; mkdir -p $out
timeout -k 10 -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/gossip -o run -- python3 bench.py --workload gossip --no-cpu-baseline > $out/gossip.log 2>&1 || exit 1
echo gossip done
timeout -k 10 -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/paxos -o run -- python3 bench.py --workload paxos --no-cpu-baseline > $out/paxos.log 2>&1 || exit 1
echo paxos done
find $out -name "*kernel_stats.csv"
