#!/bin/bash
# Host-side AddressSanitizer build of libpskv.so and the C++ boundary programs
# (tests/cpp), into scratch/asan/ (git-ignored).  Only host code is
# instrumented (-Xarch_host); device code is unchanged.  Run the programs on
# the GPU box with ASAN_OPTIONS=detect_leaks=0 (the HIP runtime's own
# allocations are not ours to report), e.g.
#   bash tools/asan_build.sh && ASAN_OPTIONS=detect_leaks=0 scratch/asan/hip_storage_test
# UBSan (SAN=address,undefined) is built with -fno-sanitize-recover=all, so any
# report ends the program with a non-zero status instead of only being logged.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
SAN=${SAN:-address}  # e.g. SAN=address,undefined
NORECOVER=-fno-sanitize-recover=all
O=$R/scratch/asan
mkdir -p "$O"
CXX=/opt/rocm/llvm/bin/clang++
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared \
  -Xarch_host -fsanitize=$SAN -Xarch_host $NORECOVER -Xarch_host -fno-omit-frame-pointer \
  -I "$R/include" -I "$R/parameter_server_amd/csrc" \
  "$R/parameter_server_amd/csrc/pskv_kernels.hip" "$R/parameter_server_amd/csrc/pskv_shard.cpp" \
  "$R/parameter_server_amd/csrc/pskv_frames.cpp" \
  -o "$O/libpskv.so"
for p in hip_storage_test kv_client_table_test ssp_replay; do
  oracle_link=""  # ssp_replay links the oracle checker as well
  if [ "$p" = ssp_replay ]; then
    oracle_link="-L $R/oracle -loracle -Wl,-rpath,$R/oracle"
  fi
  # shellcheck disable=SC2086  # oracle_link is a word list on purpose
  $CXX -O1 -g -std=c++11 -pthread -fsanitize=$SAN $NORECOVER -fno-omit-frame-pointer \
    -I "$R/include" "$R/tests/cpp/$p.cpp" -o "$O/$p" \
    -L "$O" -lpskv '-Wl,-rpath,$ORIGIN' $oracle_link
done
echo "asan build: $O"
