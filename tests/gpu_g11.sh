set -o pipefail
o=gpurun_out/g11; mkdir -p $o
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $o/p.log 2>&1 || exit 1
  echo "pbft $(tail -1 $o/p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); l=d['loop']; print('%.3f ms/step launches %.1f frac %.3f' % (d['ms_per_step'], l['launches_per_step'], d['roofline']['frac']), d['breakdown']['kernel_us'])")"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/pt -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $o/ptrace.log 2>&1 || exit 1
