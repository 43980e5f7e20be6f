#!/bin/bash
# Profile bench.py on the GPU box: kernel trace + stats, then two separate PMC
# passes (FETCH_SIZE, WRITE_SIZE) summarised by tools/collect_pmc.py.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
export TMPDIR=/tmp
OUT=$R/gpurun_out/${1:-prof}
shift || true
mkdir -p "$OUT"
# MODE=cold: the cold form alone (bench.py --cold-only, roofline.cold);
# otherwise the headline step alone (no cold form, Zipf or side measurements)
if [ "${MODE:-headline}" = cold ]; then
  ARGS="--steps 20 --warmup 2 --cold-only $*"
  CONFIG='{"n_gpus": 1, "batches": 64, "batch_keys": 1000000, "sets": 16, "form": "cold", "shard_keys": 1000000000}'
else
  ARGS="--steps 20 --warmup 2 --no-cpu-baseline --no-extra --no-zipf --no-cold $*"
  CONFIG='{"n_gpus": 1, "batches": 64, "batch_keys": 1000000, "sets": 16, "form": "pull-free-slots"}'
fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o trace -- \
  python3 "$R/bench.py" $ARGS > "$OUT/trace.log" 2>&1 || exit 1
timeout -k 5 -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT" -o fetch -- \
  python3 "$R/bench.py" $ARGS > "$OUT/fetch.log" 2>&1 || exit 2
timeout -k 5 -s KILL 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT" -o write -- \
  python3 "$R/bench.py" $ARGS > "$OUT/write.log" 2>&1 || exit 3
python3 "$R/tools/collect_pmc.py" "$OUT/fetch_counter_collection.csv" \
  "$OUT/write_counter_collection.csv" "$OUT/pmc.json" "$CONFIG" > /dev/null || exit 4
echo "profile done: $OUT"
