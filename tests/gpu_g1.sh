set -o pipefail
mkdir -p gpurun_out/g1
timeout -k 10 900 python -u -m pytest tests/test_headline_oracle.py -x -v --timeout 900 --timeout-method thread > gpurun_out/g1/tests.log 2>&1 || { tail -30 gpurun_out/g1/tests.log; exit 1; }
tail -3 gpurun_out/g1/tests.log
bash tests/gpu_ab.sh g1 - "" "BCSIM_L2_OVERLAP=0" "BCSIM_KSTATS=0" "" "BCSIM_L2_OVERLAP=0" "BCSIM_KSTATS=0"
