set -o pipefail
out=gpurun_out/r4p; mkdir -p $out
(while sleep 50; do date +%s >> $out/heartbeat; done) & hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_fastpaths.py tests/test_fullsize.py -m gpu -x -q --timeout 400 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit 1
bash tests/gpu_ab.sh ab24 - "" "BCSIM_LIB=ab_lib/head.so" "" "BCSIM_LIB=ab_lib/head.so" || exit 1
BCSIM_WGT=1 timeout -k 10 240 python bench.py --steps 3 --warmup 3 --no-cpu-baseline > $out/wgt.log 2>&1 || exit 1
grep "wgs\] cell" $out/wgt.log | head -12
