set -o pipefail
out=gpurun_out/r04suite; mkdir -p $out
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
tail -5 $out/pytest_gpu.log
exit $rc
