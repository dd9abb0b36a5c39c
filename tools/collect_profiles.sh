#!/bin/bash
# Copy the round's GPU profiles (tests/gpu_prof_all.sh <tag>) into profiles/ under the names
# bench.py's pmc_traffic() and the docs read:
#   bash tools/collect_profiles.sh <tag> <round, e.g. r06>
set -e
tag=$1; rnd=$2
for pair in pbft:pbft4096 gossip:gossip65536 paxos:paxos4096_r10000; do
  w=${pair%%:*}; name=${pair##*:}; src=gpurun_out/$tag/$w
  [ -d $src ] || { echo "missing $src"; continue; }
  python3 tools/pmc_summary.py $src profiles/${rnd}_pmc_${name}.json
  cp $src/trace/run_kernel_stats.csv profiles/${rnd}_kernel_stats_${name}.csv
  [ -f $src/window_stats.csv ] && cp $src/window_stats.csv profiles/${rnd}_window_stats_${name}.csv
  grep '^{' $src/trace.log | tail -1 > profiles/${rnd}_prof_bench_${name}.json || true
done
ls -la profiles/${rnd}_*
