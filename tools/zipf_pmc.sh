#!/bin/bash
# PMC passes over the cfg-3 (Zipf) general path: wave-state and LDS counters,
# then HBM bytes (FETCH_SIZE / WRITE_SIZE in separate passes).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
export TMPDIR=/tmp
OUT=$R/gpurun_out/${1:-zpmc}
mkdir -p "$OUT"
export PROBE_ROUNDS=2
i=0
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_WAVES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$OUT" -o p$i -- \
    python3 "$R/tools/zipf_probe.py" > "$OUT/p$i.log" 2>&1 || exit $i
done
python3 "$R/tools/pmc_table.py" "$OUT"/p*_counter_collection.csv > "$OUT/table.txt" || exit 9
echo "pmc done: $OUT"
