set -o pipefail
out=gpurun_out/r4s; mkdir -p $out
(while sleep 50; do date +%s >> $out/heartbeat; done) & hb=$!
trap "kill $hb 2>/dev/null" EXIT
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_fastpaths.py tests/test_fullsize.py tests/test_window_split.py tests/test_partition.py -m gpu -x -q --timeout 600 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit 1
bash tests/gpu_ab.sh ab27 - "" "BCSIM_LIB=ab_lib/head.so" "" "BCSIM_LIB=ab_lib/head.so" "" "BCSIM_LIB=ab_lib/head.so" || exit 1
