#!/bin/bash
# PMC passes (one counter group each) over a short PBFT bench: SQ instruction mix / waits of the
# link and scan kernels (tools/pmc_summary.py reads the CSVs)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-pmct}; mkdir -p $out
rocprofv3 --list-avail > $out/avail.txt 2>&1 || true
k=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM"; do
  k=$((k + 1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $grp -d $out/p$k -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 5 > $out/p$k.log 2>&1 || { echo "pass $k failed"; tail -5 $out/p$k.log; exit 1; }
done
find $out -name "*counter_collection.csv" | head
