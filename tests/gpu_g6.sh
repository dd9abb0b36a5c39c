set -o pipefail
o=gpurun_out/g6; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for e in "" "BCSIM_CHAIN=0" "" "BCSIM_CHAIN=0"; do
  env $e timeout -k 10 200 python bench.py --workload gossip --no-cpu-baseline --steps 20 --warmup 5 > $o/g.log 2>&1 || exit 1
  echo "gossip [$e] $(tail -1 $o/g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3f ms/step' % d['ms_per_step'], d['loop'])")"
done
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $o/p.log 2>&1 || exit 1
echo "pbft $(tail -1 $o/p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%.3f ms/step' % d['ms_per_step'], d['loop'])")"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/gt -o kt -- python3 bench.py --workload gossip --no-cpu-baseline --steps 6 --warmup 5 > $o/gtrace.log 2>&1 || exit 1
BCSIM_CHAIN=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/gt0 -o kt -- python3 bench.py --workload gossip --no-cpu-baseline --steps 6 --warmup 5 > $o/gtrace0.log 2>&1 || exit 1
