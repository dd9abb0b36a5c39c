set -o pipefail
mkdir -p gpurun_out/bis
for v in "BCSIM_FEW_SCAN=0" "BCSIM_FEW_SCAN=0 BCSIM_L2_OVERLAP=0" "BCSIM_FEW_SCAN=0 BCSIM_MESH_TILE=0" "BCSIM_FEW_SCAN=0 BCSIM_NO_DESC=1"; do
  echo "== $v"
  env $v timeout -k 10 120 python tests/parity_run.py pbft100_fixed pbft16_fixed_100 pbft8_fixed_40 pbft5_odd 2>&1 | cut -c1-200
  rc=$?; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 3 ] && exit 1
done
exit 0
