set -o pipefail
o=gpurun_out/g12; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_sparse.py tests/test_fullsize.py tests/test_montecarlo.py -x -q --timeout 600 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 400 python bench.py --workload paxos --no-cpu-baseline > $o/x.log 2>&1 || exit 1
echo "paxos $(tail -1 $o/x.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.1f ms/step' % d['ms_per_step'], d['kernel_us'], d['breakdown']['kernel_us'])")"
