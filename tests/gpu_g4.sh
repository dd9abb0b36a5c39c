set -o pipefail
o=gpurun_out/g4; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/gt -o kt -- python3 bench.py --workload gossip --no-cpu-baseline --steps 6 --warmup 5 > $o/gtrace.log 2>&1 || exit 1
for e in "" "BCSIM_EXT_EVENTS=0" "" "BCSIM_EXT_EVENTS=0"; do
  env $e timeout -k 10 200 python bench.py --workload gossip --no-cpu-baseline --steps 20 --warmup 5 > $o/g.log 2>&1 || exit 1
  echo "gossip [$e] $(tail -1 $o/g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3f ms/step' % d['ms_per_step'])")"
done
bash tests/gpu_ab.sh g4 - "" "BCSIM_EXT_EVENTS=0" "" "BCSIM_EXT_EVENTS=0"
