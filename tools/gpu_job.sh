#!/bin/bash
# One GPU-box job of named steps, each under its own time limit, stopping at the
# first failure (gpurun runs it as: bash tools/gpu_job.sh OUTDIR STEP...).
#   tests_focus  the parity tests of the dense / repair / golden / replay paths
#   tests_all    pytest -m gpu (everything)
#   align        tools/align_probe.py (window phase cost)
#   emu          bench.py as rank 0 of 8 and of 2 (one rank's cfg-4 share alone)
#   bench        bench.py --steps 20 (the driver's command line)
#   zipf         tools/zipf_probe.py kernel times on cfg 3
#   profile      tools/gpu_profile.sh: rocprofv3 kernel trace + stats, FETCH / WRITE PMC passes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/$1
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    tests_focus) timeout -k 10 300 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
        "$R/tests/test_gpu_parity.py" "$R/tests/test_replay.py" \
        -k "phase or dense or lookalike or repaired or hint or golden or replay or options or dedup or zipf" > "$OUT/tests_focus.log" 2>&1 ;;
    tests_all) timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread "$R/tests" -m gpu \
        > "$OUT/tests_all.log" 2>&1 ;;
    align) timeout -k 10 200 python3 "$R/tools/align_probe.py" 0,1,2,3 20 > "$OUT/align.log" 2>&1 ;;
    emu) PSKV_BENCH_EMULATE=0/8 timeout -k 10 200 python3 "$R/bench.py" --steps 20 --no-zipf --no-cpu-baseline --no-extra \
           > "$OUT/emu08.json" 2> "$OUT/emu08.err" &&
         PSKV_BENCH_EMULATE=0/2 timeout -k 10 200 python3 "$R/bench.py" --steps 20 --no-zipf --no-cpu-baseline --no-extra \
           > "$OUT/emu02.json" 2> "$OUT/emu02.err" ;;
    bench) timeout -k 10 400 python3 "$R/bench.py" --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    profile) bash "$R/tools/gpu_profile.sh" "$(basename "$OUT")/prof" > "$OUT/profile.log" 2>&1 ;;
    zipf) timeout -k 10 300 python3 "$R/tools/zipf_probe.py" "" "PSKV_GET_DEDUP=1" > "$OUT/zipf.log" 2>&1 ;;
    *) echo "unknown step $step"; exit 9 ;;
  esac
  rc=$?
  echo "step $step rc=$rc" >> "$OUT/steps.log"
  [ $rc -eq 0 ] || exit $rc
done
