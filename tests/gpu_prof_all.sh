#!/bin/bash
# Round-end profiles of the three bench workloads (each exactly as bench.py runs it, no CPU
# baseline): kernel trace + stats, then one PMC pass per counter group (tests/gpu_prof.sh), and
# the timed window's kernel statistics (tools/window_stats.py).
#   bash tests/gpu_prof_all.sh <tag>        (outputs under gpurun_out/<tag>/{pbft,gossip,paxos})
set -o pipefail
tag=${1:-prof}
(while sleep 50; do date +%s >> gpurun_out/$tag.heartbeat; done) & hb=$!
trap "kill $hb 2>/dev/null" EXIT
mkdir -p gpurun_out/$tag
run() {
  local w=$1; shift
  bash tests/gpu_prof.sh $tag/$w "$@" --no-cpu-baseline > gpurun_out/$tag/$w.log 2>&1 || { tail -5 gpurun_out/$tag/$w.log; exit 1; }
  python3 tools/window_stats.py gpurun_out/$tag/$w/trace/run_kernel_trace.csv gpurun_out/$tag/$w/trace.log \
    gpurun_out/$tag/$w/window_stats.csv >> gpurun_out/$tag/$w.log 2>&1
  echo "$w: $(tail -1 gpurun_out/$tag/$w.log)"
}
run pbft --steps 20 --warmup 5
run gossip --workload gossip --steps 20 --warmup 5
run paxos --workload paxos
