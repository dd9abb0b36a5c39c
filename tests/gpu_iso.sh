set -o pipefail
BCSIM_WGT=1 timeout -k 5 300 python bench.py --no-cpu-baseline --steps 2 --warmup 5 2>&1 | grep -v amdgpu.ids | cut -c1-600
