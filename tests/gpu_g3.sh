set -o pipefail
o=gpurun_out/g3; mkdir -p $o
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_switches.py tests/test_headline_oracle.py tests/test_fastpaths.py tests/test_fullsize.py -x -q --timeout 600 --timeout-method thread > $o/tests.log 2>&1 || { tail -30 $o/tests.log; exit 1; }
tail -2 $o/tests.log
BCSIM_FDBG=1 timeout -k 10 120 python bench.py --steps 3 --warmup 5 --no-cpu-baseline > $o/fdbg.log 2>&1 || exit 1
bash tests/gpu_ab.sh g3 - "" "BCSIM_FUSE_ACT=0" "" "BCSIM_FUSE_ACT=0"
