#!/bin/bash
# Per-launch kernel trace of the bench (for per-cell analysis) + per-WG k_link phase timing.
set -o pipefail
mkdir -p gpurun_out/trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -o kt -- python3 bench.py --no-cpu-baseline --steps 6 --warmup 5 > gpurun_out/trace/bench.log 2>&1 &&
BCSIM_WGT=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 6 --warmup 5 > gpurun_out/trace/wgt.log 2>&1
rc=$?
find gpurun_out/trace -name "*.csv" | head
exit $rc
