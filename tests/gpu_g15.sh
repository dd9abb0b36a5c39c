set -o pipefail
o=gpurun_out/g15; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_headline_oracle.py tests/test_gpu_parity.py tests/test_fullsize.py tests/test_switches.py -x -q --timeout 600 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/pt -o run -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > $o/ptrace.log 2>&1 || exit 1
grep k_rebin $o/pt/run_kernel_stats.csv | cut -c1-200
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > $o/p.log 2>&1 || exit 1
tail -1 $o/p.log | cut -c1-400
