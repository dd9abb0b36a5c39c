set -o pipefail
bash tests/gpu_bisect.sh "pbft100_fixed pbft16_fixed_100 pbft8_fixed_40 pbft512_small pbft12_jitter_b2 pbft16_fq_100" "BCSIM_NO_ACTSYNC=1" || exit 1
bash tests/gpu_ab.sh ab20 - "" "BCSIM_NO_ACTSYNC=1" "BCSIM_LIB=ab_lib/wpe6.so" "" "BCSIM_NO_ACTSYNC=1"
