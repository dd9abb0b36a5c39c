set -o pipefail
o=gpurun_out/g13; mkdir -p $o
BCSIM_PX_CAP=4 timeout -k 10 600 python -u -m pytest tests/test_sparse.py -x -q --timeout 500 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for e in "BCSIM_PX_CAP=4" "" "BCSIM_PX_CAP=4" ""; do
  env $e timeout -k 10 400 python bench.py --workload paxos --no-cpu-baseline > $o/x.log 2>&1 || exit 1
  echo "paxos [$e] $(tail -1 $o/x.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.1f ms/step' % d['ms_per_step'], d['kernel_us'])")"
done
