#!/bin/bash
# Diagnostic build of the library with K5 phase stamps (-DPSKV_K5_STAMPS) and
# the k5_phases driver, both under tools/micro/ (git-ignored; they travel to
# the GPU box with the tree).  The product libpskv.so is not touched.
#   bash tools/micro/build_k5_phases.sh [OUTDIR [extra hipcc flags...]]
# OUTDIR (default tools/micro) gets libpskv_diag.so and k5_phases side by side
# (rpath $ORIGIN), so variant builds, e.g. -DPSKV_K5A_STREAM=0, can sit beside
# each other for an A/B.
set -euo pipefail
R=$(cd "$(dirname "$0")/../.." && pwd)
C=$R/parameter_server_amd/csrc
O=${1:-$R/tools/micro}
shift || true
mkdir -p "$O"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -DPSKV_K5_STAMPS "$@" \
  -I "$R/include" -I "$C" "$C/pskv_kernels.hip" "$C/pskv_shard.cpp" "$C/pskv_frames.cpp" \
  -o "$O/libpskv_diag.so"
g++ -O2 -std=c++11 -I "$R/include" "$R/tools/micro/k5_phases.cpp" -L "$O" -lpskv_diag \
  '-Wl,-rpath,$ORIGIN' -o "$O/k5_phases"
echo "built $O/k5_phases"
