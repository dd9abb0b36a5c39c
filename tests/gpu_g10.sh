set -o pipefail
o=gpurun_out/g10; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_switches.py tests/test_headline_oracle.py tests/test_fastpaths.py -x -q --timeout 600 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for e in "" "BCSIM_LINK_FEW=0" "" "BCSIM_LINK_FEW=0"; do
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $o/p.log 2>&1 || exit 1
  echo "pbft [$e] $(tail -1 $o/p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); l=d['loop']; print('%.3f ms/step launch %.0f wait %.0f us/step, %.1f launches, %.2f syncs/window frac %.3f' % (d['ms_per_step'], l['host_launch_us_per_step'], l['host_wait_us_per_step'], l['launches_per_step'], l['host_syncs_per_window'], d['roofline']['frac']))")"
done
