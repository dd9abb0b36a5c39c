set -o pipefail
mkdir -p gpurun_out/g2
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/g2/tests.log 2>&1 || { tail -30 gpurun_out/g2/tests.log; exit 1; }
tail -3 gpurun_out/g2/tests.log
bash tests/gpu_ab.sh g2 - "" "BCSIM_FUSE_ACT=0" "BCSIM_L2_OVERLAP=1" "" "BCSIM_FUSE_ACT=0" "BCSIM_L2_OVERLAP=1"
