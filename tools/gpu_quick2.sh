# quick GPU check: the 2-bucket (tag-wrap) parity cases, fast paths, then the PBFT bench twice
set -o pipefail
out=gpurun_out/quick2; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_fastpaths.py -m gpu -x -q --timeout 200 --timeout-method thread -k "b2 or fast or gossip" > $out/tests.log 2>&1; tail -2 $out/tests.log
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/b$rep.log 2>&1 || exit 1
  tail -1 $out/b$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4e' % d['value'], round(d['ms_per_step'],3), round(d['roofline']['avg_launch_us'],1), round(d['roofline']['frac'],3), {k: round(v) for k, v in d['breakdown']['kernel_us'].items()})"
done
