# A/B of the k_scan_pbft -> k_link_mesh descriptors (BCSIM_NO_DESC=1: off), PBFT n=4096 bench
set -o pipefail
out=gpurun_out/abdesc; mkdir -p $out
for rep in 1 2; do
  for v in 0 1; do
    BCSIM_NO_DESC=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/d${v}_$rep.log 2>&1 || exit 1
    echo "NO_DESC=$v rep $rep: $(tail -1 $out/d${v}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4e' % d['value'], round(d['ms_per_step'],3), round(d['roofline']['avg_launch_us'],1), {k: round(v) for k, v in d['breakdown']['kernel_us'].items()})")"
  done
done
