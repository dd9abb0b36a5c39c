# full GPU suite, then the PBFT bench (driver shape) twice
set -o pipefail
out=gpurun_out/final; mkdir -p $out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 280 --timeout-method thread > $out/pytest.log 2>&1; rc=$?; tail -2 $out/pytest.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $out/b$rep.log 2>&1 || exit 1
  tail -1 $out/b$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.4e' % d['value'], round(d['ms_per_step'],3), round(d['roofline']['avg_launch_us'],1), round(d['roofline']['frac'],3), round(d['roofline']['pipeline']['frac'],3))"
done
