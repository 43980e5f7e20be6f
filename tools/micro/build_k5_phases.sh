#!/bin/bash
# Diagnostic build of the library with K5 phase stamps (-DPSKV_K5_STAMPS) and
# the k5_phases driver, both under tools/micro/ (git-ignored; they travel to
# the GPU box with the tree).  The product libpskv.so is not touched.
set -euo pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
C=$R/parameter_server_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DPSKV_K5_STAMPS \
  -I "$R/include" -I "$C" "$C/pskv_kernels.hip" "$C/pskv_shard.cpp" "$C/pskv_frames.cpp" \
  -o "$R/tools/micro/libpskv_diag.so"
g++ -O2 -std=c++11 -I "$R/include" "$R/tools/micro/k5_phases.cpp" -L "$R/tools/micro" -lpskv_diag \
  '-Wl,-rpath,$ORIGIN' -o "$R/tools/micro/k5_phases"
echo "built tools/micro/k5_phases"
