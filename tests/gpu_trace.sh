#!/bin/bash
# Per-launch kernel trace of the bench (for per-cell analysis: tools/trace_windows.py) + per-WG
# phase timing (BCSIM_WGT=1), under an optional env setting and bench arguments:
#   bash tests/gpu_trace.sh [tag] ["ENV=1 ..."] ["--workload gossip ..."]
set -o pipefail
tag=${1:-trace}; envs=${2:-}; bargs=${3:-}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
env $envs timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out -o kt -- python3 bench.py --no-cpu-baseline --steps 6 --warmup 5 $bargs > $out/bench.log 2>&1 &&
env $envs BCSIM_WGT=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 --warmup 5 $bargs > $out/wgt.log 2>&1
rc=$?
find $out -name "*.csv" | head
exit $rc
