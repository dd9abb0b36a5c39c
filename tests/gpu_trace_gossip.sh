set -o pipefail
out=gpurun_out/gtr2; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out -o run -- python3 bench.py --workload gossip --steps 5 --warmup 3 --no-cpu-baseline > $out/log 2>&1; rc=$?; tail -1 $out/log | cut -c1-200; exit $rc
