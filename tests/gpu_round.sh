#!/bin/bash
# GPU-box validation, one step at a time; stops at the first failure or fault.
#   bash tests/gpu_round.sh [steps...]   (default: checked parity smoke bench prof)
set -o pipefail
mkdir -p gpurun_out
faulted() { grep -q "APERTURE\|illegal memory\|Memory access fault\|HSA_STATUS_ERROR" "$1"; }
run() {
  local name=$1 secs=$2
  shift 2
  echo "== $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] || faulted "gpurun_out/$name.log"; then exit 1; fi
}
steps=${*:-checked parity smoke bench prof}
for st in $steps; do
  case $st in
    checked) run checked 240 env BCSIM_LIB="$PWD/blockchain-simulator_amd/libbcsim_checked.so" BCSIM_SYNC_EACH=1 python tests/parity_run.py ;;
    parity)  run parity 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ;;
    part)    run part 400 python -u -m pytest tests/test_partition.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
    smoke)   run smoke 120 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench1k) run bench1k 300 python bench.py --nodes 1024 --cpu-budget 5 ;;
    bench)   run bench 400 python bench.py ;;
    gprof)   run gprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gprof -o g -- python3 bench.py --workload gossip --no-cpu-baseline --steps 2 --warmup 4 ;;
    mc)      run mc 300 python -u -m pytest tests/test_montecarlo.py -m gpu -x -v --timeout 120 --timeout-method thread ;;
    paxos)   run paxos 400 python bench.py --workload paxos --cpu-budget 10 ;;
    gossip)  run gossip 400 python bench.py --workload gossip --cpu-budget 10 ;;
    newcases) run newcases 300 env BCSIM_LIB="$PWD/blockchain-simulator_amd/libbcsim_checked.so" BCSIM_SYNC_EACH=1 python tests/parity_run.py gossip64_d4_fixed gossip200_d8_jitter_ctr gossip512_d8_blocks gossip24_mesh pbft32_d6_ctr raft48_d6_ctr ;;
    prof)    run prof 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench -- python bench.py --no-cpu-baseline ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
