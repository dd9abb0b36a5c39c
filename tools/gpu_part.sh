# partitioned-run checks + the P=1 partition-machinery gossip bench
set -o pipefail
out=gpurun_out/part; mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_partition.py tests/test_fqcodel.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1; grep -E "passed|failed|FAIL" $out/tests.log | tail -4
timeout -k 10 200 python bench.py --workload gossip --pdes1 --no-cpu-baseline > $out/g1.log 2>&1 || exit 1
tail -1 $out/g1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('pdes1 %.4e' % d['value'], round(d['ms_per_step'],3))"
timeout -k 10 200 python bench.py --workload gossip --no-cpu-baseline > $out/g0.log 2>&1 || exit 1
tail -1 $out/g0.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('plain  %.4e' % d['value'], round(d['ms_per_step'],3))"
