# A/B: the round-3 WIP commit (worktree .wt78) vs this tree, PBFT n=4096 bench; then the
# fast-path / full-size / FQCODEL GPU tests of this tree
set -o pipefail
out=$GRAFT_REPO_ROOT/gpurun_out/abold; mkdir -p $out
summ() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%.4e' % d['value'], round(d['ms_per_step'],3), round(d['roofline']['avg_launch_us'],1), {k: round(v) for k, v in d['breakdown']['kernel_us'].items()})" $1; }
for rep in 1 2; do
  (cd .wt78 && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/old$rep.log 2>&1) || exit 1
  echo "old:    $(summ $out/old$rep.log)"
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $out/new$rep.log 2>&1 || exit 1
  echo "new:    $(summ $out/new$rep.log)"
done
timeout -k 10 400 python -u -m pytest tests/test_fastpaths.py tests/test_fullsize.py tests/test_fqcodel.py -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1; tail -2 $out/tests.log
