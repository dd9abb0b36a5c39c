#!/bin/bash
# GPU-box profiling of the bench workload: kernel trace + stats, then one PMC
# pass per counter group (rocprofv3 cannot split counters over passes).
#   bash tests/gpu_prof.sh [tag] [bench args...]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
tag=${1:-prof}; shift
args=${*:---no-cpu-baseline}
out=gpurun_out/$tag
mkdir -p $out
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 -s KILL $secs "$@" > $out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 $out/$name.log
  [ $rc -eq 0 ] || exit 1
}
step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py $args
step pmc_sq 300 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $out/sq -o run -- python3 bench.py $args
step pmc_fetch 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $out/fetch -o run -- python3 bench.py $args
step pmc_write 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum -d $out/write -o run -- python3 bench.py $args
find $out -name "*.csv" | head -20
