#!/bin/bash
# A/B two builds of libpskv.so on one box (ab/libpskv_base.so, ab/libpskv_new.so,
# built beforehand; AB_VARIANTS="base x y" alternates ab/libpskv_{base,x,y}.so): alternate them (swapping the in-tree library file, which
# is restored to the tree's own build on exit), 3
# rounds each, under bench.py (default) or, with AB_PROG=zipf, under
# tools/zipf_probe.py (the cfg-3 K5 / K1 kernel times), with AB_PROG=sizes under
# tools/size_probe.py (K2g / K1 fixed cost per launch), with AB_PROG=e2e under
# tools/e2e_probe.py (host-buffer Add / Get).
#   bash tools/ab_lib.sh OUTNAME ["bench.py args"]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/${1:-ab}
ARGS=${2:-"--no-extra --no-cpu-baseline --no-zipf"}
mkdir -p "$OUT"
LIB=$R/parameter_server_amd/libpskv.so
SAVE=$(mktemp) && cp "$LIB" "$SAVE" || exit 1   # the tree's own build, put back at the end
restore() { cp "$SAVE" "$LIB"; rm -f "$SAVE"; }
trap restore EXIT
for i in 1 2 3; do
  for v in ${AB_VARIANTS:-base new}; do
    cp "$R/ab/libpskv_$v.so" "$R/parameter_server_amd/libpskv.so" || exit 1
    if [ "${AB_PROG:-bench}" = sizes ]; then
      timeout -k 10 200 python3 "$R/tools/size_probe.py" > "$OUT/$v$i.log" 2>&1 || exit 2
    elif [ "${AB_PROG:-bench}" = e2e ]; then
      timeout -k 10 200 python3 "$R/tools/e2e_probe.py" > "$OUT/$v$i.log" 2>&1 || exit 2
    elif [ "${AB_PROG:-bench}" = zipf ]; then
      timeout -k 10 200 python3 "$R/tools/zipf_probe.py" > "$OUT/$v$i.log" 2>&1 || exit 2
    else
      timeout -k 10 200 python3 "$R/bench.py" $ARGS > "$OUT/$v$i.json" 2> "$OUT/$v$i.err" || exit 2
    fi
  done
done
echo "ab done"
