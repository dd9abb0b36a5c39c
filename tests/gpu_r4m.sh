set -o pipefail
out=gpurun_out/r4m; mkdir -p $out
(while sleep 50; do date +%s >> $out/heartbeat; done) & hb=$!
trap "kill $hb 2>/dev/null" EXIT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --stats -d $out/gtr -o run -- python3 bench.py --workload gossip --steps 5 --warmup 3 --no-cpu-baseline > $out/gtr.log 2>&1; rc=$?; tail -2 $out/gtr.log; [ $rc -eq 0 ] || exit 1
find $out/gtr -name "*.csv" | head
