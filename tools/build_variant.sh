#!/bin/bash
# Build an A/B variant of the engine library with extra compile definitions into ab_lib/<name>.so
# (select it at run time with BCSIM_LIB=ab_lib/<name>.so):
#   bash tools/build_variant.sh ts32 -DBCSIM_TILE_TS=32
set -e
name=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/blockchain-simulator_amd
B=$R/ab_lib/build_$name
mkdir -p $B
H=/opt/rocm/bin/hipcc
F="-O3 -std=c++17 -fPIC -Wall -Wno-unused-result -I$R/include"
$H --offload-arch=gfx950 $F "$@" -c $P/csrc/bcsim_capi.hip -o $B/capi.o
for s in host_math network_helper topology; do g++ $F -c $P/csrc/$s.cpp -o $B/$s.o; done
$H --offload-arch=gfx950 -shared -fPIC -o $R/ab_lib/$name.so $B/capi.o $B/host_math.o $B/network_helper.o $B/topology.o \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf $B
echo "ab_lib/$name.so"
