#!/bin/bash
# Ad-hoc GPU-box check: full parity list, per-workgroup k_link timing, bench.
set -o pipefail
echo "== parity"; timeout -k 5 200 python tests/parity_run.py 2>&1 | cut -c1-150
echo "== wgt"; BCSIM_WGT=1 timeout -k 5 300 python bench.py --no-cpu-baseline --steps 2 --warmup 5 2>&1 | grep -v amdgpu.ids | cut -c1-700 | tail -14
echo "== bench"; timeout -k 5 300 python bench.py --no-cpu-baseline 2>&1 | tail -1
