#!/bin/bash
# Build a kernel variant of libpow_gpu.so from a copy of csrc/ for tools/ab_sweep.
#   tools/ab_build.sh <csrc-dir> <out-dir>
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
src=$1; out=$2
mkdir -p "$out"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -mcode-object-version=5 \
  -I "$R/include" -I "$src" "$src"/pow_api.cpp "$src"/pow_board.cpp "$src"/pow_group.cpp "$src"/pow_kernels.hip \
  "$src"/pow_sort.hip "$src"/valu_peak.hip "$src"/pow_aql.cpp ${AB_FLAGS:-} -o "$out/libpow_gpu.so" \
  -L /opt/rocm/lib -lhsa-runtime64 -Wl,-rpath,/opt/rocm/lib
