#!/bin/bash
# One GPU-box job of named steps, each under its own time limit, stopping at the
# first failure (gpurun runs it as: bash tools/gpu_job.sh OUTDIR STEP...).
#   tests_focus  the parity tests of the dense / repair / golden / replay paths
#   tests_all    pytest -m gpu (everything)
#   tests_addget the push-then-pull call tests, the bench-form and two-rank cfg-4 tests, options
#   align        tools/align_probe.py (window phase cost)
#   emu          bench.py as rank 0 of 8 and of 2 (one rank's cfg-4 share alone)
#   emu8all      bench.py as each of the 8 ranks of N = 8 in turn (every rank's cfg-4 share alone)
#   emu_curve    every rank of N = 2 and N = 4 emulated in turn (with emu8all: the estimated scaling curve)
#   emutrace     rocprofv3 kernel trace of rank 0 of 8 (kernel durations and gaps of a small share)
#   smalllat     tools/micro/small_latency (built with g++ against libpskv.so): per-call host Add / Get latency
#   ablat        small_latency under ab/libpskv_{AB_VARIANTS}.so, twice each (the in-tree library restored after)
#   emu_u48      ranks 0 and 1 of N = 8 emulated at UNROLL 8 / 4 (8 / 4 Ki-key chunks for K2g and K1), twice
#   emu_unroll   rank 0 of 8 at 4 x 4 keys per lane (PSKV_UNROLL=4) and at the default 8
#   ztrace       rocprofv3 kernel trace of zipf_probe at K5a 1024 and 512 threads (K5a / K5b split)
#   zpmc         tools/zipf_pmc.sh: wave-state, LDS and HBM counters of the cfg-3 path
#   k5phases     tools/micro/k5_phases (diagnostic build: K5a / K5b phase stamps), assign and accumulate
#   k5dist       the same (assign) on Zipf keys, uniform keys and a uniform pool matched to Zipf's distinct count
#   stamps       tools/step_stamps.py (ab/stamps/libpskv.so, -DPSKV_STEP_STAMPS): K2g / K1 workgroup phase times of
#                rank 0 and 1 of N = 8 and of the N = 1 headline step
#   k5ab         ab/diag_{base,new}/k5_phases (assign, accumulate), then abz: base vs new K5 build phase stamps and times
#   abz          tools/ab_lib.sh with AB_PROG=zipf: ab/libpskv_base.so vs ab/libpskv_new.so on cfg 3, 3 rounds each
#   sizes        tools/size_probe.py: K2g / K1 time against window count (fixed cost per launch)
#   abs          tools/ab_lib.sh with AB_PROG=sizes: base vs new library under tools/size_probe.py
#   abb          tools/ab_lib.sh under bench.py (headline + cold form): base vs new library, 3 rounds
#   abe          the same with rank 0 of N = 8 emulated (PSKV_BENCH_EMULATE=0/8)
#   abocc        bench A/B of ab/libpskv_{base,occ3,occ4b}.so (K2g LDS cap off / 3 / 4 workgroups per CU)
#   abocce       the same on rank 0 of N = 8 emulated
#   abke         bench A/B of ab/libpskv_{base,kearly}.so (K2g keys before its prologue), headline and rank 0 of 8,
#                then the headline with PSKV_EARLY=1 twice
#   graph        tools/graph_probe.py: one rotation of the benchmarked steps as a HIP graph vs launched eagerly
#                (cfg 2 and rank 0 of N = 8)
#   emuzipf      bench.py as rank 0 of 8 and of 4, alone, with the cfg-3 (Zipf) measurement (time-limited)
#   ranks8diag   bench.py as 8 ranks on one GPU: headline only, then with the Zipf measurement
#   ranks8z      every rank of N = 8 alone with cfg 3 (emulated), then bench.py as 8 ranks on one GPU with cfg 3 at
#                GPU_MAX_HW_QUEUES = 1 and 4 (bounded waits, Python stack dumps every 30 s)
#   ranks8q      bench.py as RANKS8_N (8) ranks on one GPU with cfg 3 at GPU_MAX_HW_QUEUES in RANKS8_QUEUES (4)
#   ranks48      bench.py as 4 and as 8 ranks on one GPU (gloo, shared device; --sets 4): the N = 4 / 8 code path
#   zsweep       tools/zipf_probe.py: K5 bucket bits / resolve table / windows / K5a block at the head, 10 rounds
#   foldab       FOLD_REPLAY 1 / 0 interleaved, 3 rounds: the headline (--no-cold) and rank 0 of N = 8 emulated
#   foldcold     FOLD_REPLAY 1 / 0 interleaved, 3 rounds, on the cold form (bench.py --cold-only)
#   wsweep       tools/zipf_probe.py: K5 bucket window bits 11-14 on Zipf keys at 1e8 / 1.25e8 / 5e8 keys and on dense unhinted windows
#   k5tests      the K5 (unhinted Add) parity tests: Zipf, radix, random, accumulate, sentinel, ragged, full-size cfg 3
#   abk1         bench A/B of ab/libpskv_{base,k1occ6,k1occ4}.so (K1 held to 8 / 6 / 4 workgroups per CU), headline and rank 0 of 8
#   fuzz         tests/test_fuzz.py over FUZZ_SCENARIOS (1500) new seeds from FUZZ_SEED0 (3500), single and concurrent
#   sizetrace    rocprofv3 kernel trace of tools/size_probe.py (exact K2g / K4r / K1 durations and gaps)
#   idle         tools/micro/idle_launch: an idle conditional launch's cost between two streaming kernels
#   ztb          tools/zipf_probe.py: K5 bucket count / window width variants at the current K5b
#   sizes_early  tools/size_probe.py with K2g early mode off / on (PSKV_EARLY=0/1), twice
#   emu_early    ranks 0 and 1 of N = 8 emulated with early mode off / auto
#   bench_early  the cfg-2 headline with early mode auto (off there) and forced on, twice
#   fuzz3        1500 more fuzz seeds from 6500 and 8 concurrent groups (own-range K2g, one-load K1)
#   fuzz2        1500 more fuzz seeds from 5000 and 8 concurrent groups (the EARLY knob and look-alikes in play)
#   align_own    tools/align_probe.py with K2g slot-aligned chunks (EARLY=0) vs own-range chunks (EARLY=3), twice
#   zwbits       K5 bucket windows of 2^11 (default) vs 2^12 keys on cfg-3 Zipf and on unhinted dense pushes
#   coldmicro    tools/micro/cold_stream: HBM ceilings of the dense step's access shapes, every byte cold
#   coldbench    bench.py --cold-only (the headline step on a 1e9-key shard: roofline.cold's form)
#   coldopts     the cold form under cache-policy options (NTP off, NT off)
#   ntp_ab       the headline (and its cold form) with K2g parameter stores cached / nt, twice
#   emu_ntp      every rank of N = 8 emulated, K2g parameter stores cached / non-temporal
#   k2g_tune     the headline (+ cold form) under K2g grid / early-load / unroll variants
#   early_cold   the headline (+ cold form, where auto picks early loads) with EARLY auto / 0, twice
#   smoke        __graft_entry__.smoke() (what the driver runs before the bench)
#   shardsize    tools/shard_size_probe.py: K2g / K1 per key on 1e8 / 5e8 / 1e9-key shards (same windows)
#   e2e          tools/e2e_probe.py (host-buffer Add / Get against raw PCIe copy rates)
#   bench        bench.py --steps 20 (the driver's command line)
#   benchdef     bench.py with no arguments (its defaults), timed by the job
#   zipf         tools/zipf_probe.py kernel times on cfg 3
#   zipf_bin     the same for K5a at 1024- and 512-thread workgroups
#   profile      tools/gpu_profile.sh: rocprofv3 kernel trace + stats, FETCH / WRITE PMC passes (headline)
#   profile_cold the same for the cold form (bench.py --cold-only)
#   pmcprobe     tools/pmc_shard_probe.py under one --pmc pass (where the cold form's PMC pass stops)
#   vector       bench.py --vector-only at 1e6 keys (config 1's VectorStorage restatement, CPU, once)
#   asan         tools/asan_build.sh (host ASan + UBSan) and the C++ boundary programs under it
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
OUT=$R/gpurun_out/$1
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for step in "$@"; do
  echo "[$(date +%T)] step $step start"
  echo "[$(date +%T)] step $step start" >> "$OUT/steps.log"
  case $step in
    tests_focus) timeout -k 10 300 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
        "$R/tests/test_gpu_parity.py" "$R/tests/test_replay.py" \
        -k "phase or dense or lookalike or repaired or hint or golden or replay or options or dedup or zipf or radix or sentinel or random" > "$OUT/tests_focus.log" 2>&1 ;;
    tests_addget) timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread \
        "$R/tests/test_add_get.py" "$R/tests/test_dist_gpu.py" "$R/tests/test_gpu_parity.py" \
        "$R/tests/test_bench_multirank_gpu.py" -k "add_get or cfg4 or headline or options or zipf_pulls or two_ranks" \
        > "$OUT/tests_addget.log" 2>&1 ;;
    tests_all) timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread "$R/tests" -m gpu \
        > "$OUT/tests_all.log" 2>&1 ;;
    tests_r6) timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
        "$R/tests/test_dist_gpu.py" "$R/tests/test_serve.py" "$R/tests/test_bench_multirank_gpu.py" \
        -k "rank_shares or holds_staging or bench_ranks_one_gpu" > "$OUT/tests_r6.log" 2>&1 ;;
    tests_k) timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread "$R/tests" -m gpu \
        -k "$TESTS_K" > "$OUT/tests_k.log" 2>&1 ;;
    align) timeout -k 10 200 python3 "$R/tools/align_probe.py" 0,1,2,3 20 > "$OUT/align.log" 2>&1 ;;
    foldcold) mkdir -p "$OUT/foldcold" && for i in 1 2 3; do for f in 1 0; do
          PSKV_FOLD_REPLAY=$f timeout -k 10 200 python3 "$R/bench.py" --steps 50 --cold-only \
            > "$OUT/foldcold/c_f${f}_$i.json" 2> "$OUT/foldcold/c_f${f}_$i.err" || exit 1
        done; done ;;
    foldab) mkdir -p "$OUT/foldab" && for i in 1 2 3; do for f in 1 0; do
          PSKV_FOLD_REPLAY=$f timeout -k 10 200 python3 "$R/bench.py" --steps 100 --no-zipf --no-cpu-baseline \
            --no-extra --no-cold > "$OUT/foldab/h_f${f}_$i.json" 2> "$OUT/foldab/h_f${f}_$i.err" || exit 1
          PSKV_FOLD_REPLAY=$f PSKV_BENCH_EMULATE=0/8 timeout -k 10 200 python3 "$R/bench.py" --steps 100 --no-zipf \
            --no-cpu-baseline --no-extra > "$OUT/foldab/r8_f${f}_$i.json" 2> "$OUT/foldab/r8_f${f}_$i.err" || exit 1
        done; done ;;
    emu) PSKV_BENCH_EMULATE=0/8 timeout -k 10 200 python3 "$R/bench.py" --steps 20 --no-zipf --no-cpu-baseline --no-extra \
           > "$OUT/emu08.json" 2> "$OUT/emu08.err" &&
         PSKV_BENCH_EMULATE=0/2 timeout -k 10 200 python3 "$R/bench.py" --steps 20 --no-zipf --no-cpu-baseline --no-extra \
           > "$OUT/emu02.json" 2> "$OUT/emu02.err" ;;
    emu8all) for r in 0 1 2 3 4 5 6 7; do
          PSKV_BENCH_EMULATE=$r/8 timeout -k 10 200 python3 "$R/bench.py" --steps ${EMU_STEPS:-50} --no-zipf --no-cpu-baseline \
            --no-extra > "$OUT/emu8_$r.json" 2> "$OUT/emu8_$r.err" || exit 1
        done ;;
    emu_curve) for n in 2 4; do for r in $(seq 0 $((n - 1))); do
          PSKV_BENCH_EMULATE=$r/$n timeout -k 10 200 python3 "$R/bench.py" --steps ${EMU_STEPS:-50} --no-zipf --no-cpu-baseline \
            --no-extra > "$OUT/emu${n}_$r.json" 2> "$OUT/emu${n}_$r.err" || exit 1
        done; done ;;
    emutrace) PSKV_BENCH_EMULATE=0/8 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/emutrace" -o run \
          -- python3 "$R/bench.py" --steps 50 --no-zipf --no-cpu-baseline --no-extra > "$OUT/emutrace.log" 2>&1 ;;
    emu_unroll) PSKV_BENCH_EMULATE=0/8 PSKV_UNROLL=4 timeout -k 10 200 python3 "$R/bench.py" --steps 20 --no-zipf \
           --no-cpu-baseline --no-extra > "$OUT/emu08_u4.json" 2> "$OUT/emu08_u4.err" &&
         PSKV_BENCH_EMULATE=0/8 timeout -k 10 200 python3 "$R/bench.py" --steps 20 --no-zipf --no-cpu-baseline \
           --no-extra > "$OUT/emu08_u8.json" 2> "$OUT/emu08_u8.err" ;;
    emu_u48) for rep in 1 2; do for r in 0 1; do for u in 8 4; do
          PSKV_BENCH_EMULATE=$r/8 PSKV_UNROLL=$u timeout -k 10 200 python3 "$R/bench.py" --steps 50 --no-zipf \
            --no-cpu-baseline --no-extra > "$OUT/emu8_${r}_u${u}_$rep.json" 2> "$OUT/emu8_${r}_u${u}_$rep.err" || exit 1
        done; done; done ;;
    smalllat) timeout -k 10 300 "$R/tools/micro/small_latency" > "$OUT/small_latency.log" 2>&1 ;;
    smalllat_sync) for rep in 1 2; do for t in 120000 0; do
          SL_VARIANTS=0,6 PSKV_SYNC_TIMEOUT_MS=$t timeout -k 10 300 "$R/tools/micro/small_latency" \
            > "$OUT/small_latency_t${t}_$rep.log" 2>&1 || exit 1
        done; done ;;
    ablat) L=$R/parameter_server_amd/libpskv.so; cp "$L" "$OUT/.keep.so" &&
        for rep in 1 2; do for v in ${AB_VARIANTS:-base new}; do
          cp "$R/ab/libpskv_$v.so" "$L" &&
          timeout -k 10 300 "$R/tools/micro/small_latency" > "$OUT/small_latency_${v}_$rep.log" 2>&1 || { cp "$OUT/.keep.so" "$L"; exit 1; }
        done; done; cp "$OUT/.keep.so" "$L"; rm -f "$OUT/.keep.so" ;;
    ztrace) for v in ${ZTRACE_BLOCKS:-1024 512}; do
          PSKV_RB_BIN_BLOCK=$v PROBE_ROUNDS=5 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ztrace_$v" \
            -o run -- python3 "$R/tools/zipf_probe.py" > "$OUT/ztrace_$v.log" 2>&1 || exit 1
        done ;;
    zpmc) timeout -k 10 600 bash "$R/tools/zipf_pmc.sh" "$(basename "$OUT")/zpmc" > "$OUT/zpmc.log" 2>&1 ;;
    k5phases) timeout -k 10 200 "$R/tools/micro/k5_phases" 0 > "$OUT/k5_phases_assign.log" 2>&1 &&
        timeout -k 10 200 "$R/tools/micro/k5_phases" 1 > "$OUT/k5_phases_accumulate.log" 2>&1 ;;
    stamps) for spec in 0/8 1/8 0/1; do
          PSKV_LIB_PATH=$R/ab/stamps/libpskv.so timeout -k 10 200 python3 "$R/tools/step_stamps.py" $spec 20 \
            > "$OUT/stamps_${spec/\//of}.log" 2>&1 || exit 1
        done ;;
    k5ab) for v in base new; do for m in 0 1; do
          timeout -k 10 200 "$R/ab/diag_$v/k5_phases" $m > "$OUT/k5_phases_${v}_m$m.log" 2>&1 || exit 1
        done; done &&
        AB_PROG=zipf timeout -k 10 900 bash "$R/tools/ab_lib.sh" "$(basename "$OUT")/abz" > "$OUT/abz.log" 2>&1 ;;
    k5dist) for dist in zipf uniform matched; do
          timeout -k 10 200 "$R/tools/micro/k5_phases" 0 $dist > "$OUT/k5_phases_$dist.log" 2>&1 || exit 1
        done ;;
    ldsrand) timeout -k 10 120 "$R/tools/micro/lds_atomic_rand" > "$OUT/lds_atomic_rand.log" 2>&1 ;;
    abz) AB_PROG=zipf timeout -k 10 900 bash "$R/tools/ab_lib.sh" "$(basename "$OUT")/abz" > "$OUT/abz.log" 2>&1 ;;
    sizes) timeout -k 10 300 python3 "$R/tools/size_probe.py" > "$OUT/size_probe.log" 2>&1 ;;
    abh) AB_PROG=e2e timeout -k 10 900 bash "$R/tools/ab_lib.sh" "$(basename "$OUT")/abh" > "$OUT/abh.log" 2>&1 ;;
    abb) timeout -k 10 900 bash "$R/tools/ab_lib.sh" "$(basename "$OUT")/abb" > "$OUT/abb.log" 2>&1 ;;
    abe) PSKV_BENCH_EMULATE=0/8 timeout -k 10 900 bash "$R/tools/ab_lib.sh" "$(basename "$OUT")/abe" \
          "--no-extra --no-cpu-baseline --no-zipf --steps 50" > "$OUT/abe.log" 2>&1 ;;
    abocc) AB_VARIANTS="base occ3 occ4b" timeout -k 10 900 bash "$R/tools/ab_lib.sh" "$(basename "$OUT")/abocc" \
          > "$OUT/abocc.log" 2>&1 ;;
    abocce) PSKV_BENCH_EMULATE=0/8 AB_VARIANTS="base occ3 occ4b" timeout -k 10 900 bash "$R/tools/ab_lib.sh" \
          "$(basename "$OUT")/abocce" "--no-extra --no-cpu-baseline --no-zipf --no-cold --steps 50" > "$OUT/abocce.log" 2>&1 ;;
    abk1) AB_VARIANTS="base k1occ6 k1occ4" timeout -k 10 900 bash "$R/tools/ab_lib.sh" "$(basename "$OUT")/abk1" \
          > "$OUT/abk1.log" 2>&1 &&
        PSKV_BENCH_EMULATE=0/8 AB_VARIANTS="base k1occ6 k1occ4" timeout -k 10 900 bash "$R/tools/ab_lib.sh" \
          "$(basename "$OUT")/abk1e" "--no-extra --no-cpu-baseline --no-zipf --no-cold --steps 50" > "$OUT/abk1e.log" 2>&1 ;;
    abke) AB_VARIANTS="base kearly" timeout -k 10 900 bash "$R/tools/ab_lib.sh" "$(basename "$OUT")/abke" \
          > "$OUT/abke.log" 2>&1 &&
        PSKV_BENCH_EMULATE=0/8 AB_VARIANTS="base kearly" timeout -k 10 900 bash "$R/tools/ab_lib.sh" \
          "$(basename "$OUT")/abkee" "--no-extra --no-cpu-baseline --no-zipf --no-cold --steps 50" > "$OUT/abkee.log" 2>&1 &&
        for r in 1 2; do PSKV_EARLY=1 timeout -k 10 300 python3 "$R/bench.py" --steps 50 --no-zipf --no-extra \
          --no-cpu-baseline > "$OUT/early1_$r.json" 2> "$OUT/early1_$r.err" || exit 1; done ;;
    graph) timeout -k 10 300 python3 "$R/tools/graph_probe.py" 10 > "$OUT/graph_n1.log" 2>&1 &&
        PSKV_BENCH_EMULATE=0/8 timeout -k 10 300 python3 "$R/tools/graph_probe.py" 10 > "$OUT/graph_r0of8.log" 2>&1 ;;
    emuzipf) PSKV_BENCH_EMULATE=0/4 timeout -k 10 120 python3 "$R/bench.py" --steps 5 --warmup 2 --sets 4 --no-extra \
          --no-cpu-baseline > "$OUT/emuzipf4.json" 2> "$OUT/emuzipf4.err" &&
        PSKV_BENCH_EMULATE=0/8 timeout -k 10 120 python3 "$R/bench.py" --steps 5 --warmup 2 --sets 4 --no-extra \
          --no-cpu-baseline > "$OUT/emuzipf8.json" 2> "$OUT/emuzipf8.err" ;;
    ranks8diag) PSKV_BENCH_BACKEND=gloo PSKV_BENCH_SHARE_GPU=1 timeout -k 10 170 python3 -m torch.distributed.run \
          --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29611 "$R/bench.py" --gpus 8 --steps 5 \
          --warmup 2 --sets 4 --no-zipf --no-extra > "$OUT/ranks8_nozipf.json" 2> "$OUT/ranks8_nozipf.err" &&
        PSKV_BENCH_BACKEND=gloo PSKV_BENCH_SHARE_GPU=1 timeout -k 10 170 python3 -m torch.distributed.run \
          --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29612 "$R/bench.py" --gpus 8 --steps 5 \
          --warmup 2 --sets 4 --no-extra > "$OUT/ranks8_zipf.json" 2> "$OUT/ranks8_zipf.err" ;;
    ranks8z) for r in 1 2 3 4 5 6 7; do
          PSKV_BENCH_EMULATE=$r/8 PSKV_SYNC_TIMEOUT_MS=30000 timeout -k 10 90 python3 "$R/bench.py" --steps 3 \
            --warmup 1 --sets 2 --no-extra --no-cpu-baseline --no-cold > "$OUT/emuz8_$r.json" 2> "$OUT/emuz8_$r.err" || exit 1
        done &&
        for q in ${RANKS8_QUEUES:-1 4}; do
          GPU_MAX_HW_QUEUES=$q PSKV_SYNC_TIMEOUT_MS=40000 PSKV_BENCH_WATCHDOG=30 PSKV_BENCH_BACKEND=gloo \
            PSKV_BENCH_SHARE_GPU=1 timeout -k 10 150 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
            --master-addr 127.0.0.1 --master-port $((29620 + q)) "$R/bench.py" --gpus 8 --steps 3 --warmup 1 --sets 2 \
            --no-extra > "$OUT/ranks8_q$q.json" 2> "$OUT/ranks8_q$q.err" || exit 1
        done ;;
    ranks8q) for q in ${RANKS8_QUEUES:-4}; do
          GPU_MAX_HW_QUEUES=$q PSKV_SYNC_TIMEOUT_MS=40000 PSKV_BENCH_WATCHDOG=30 PSKV_BENCH_BACKEND=gloo \
            PSKV_BENCH_SHARE_GPU=1 timeout -k 10 ${RANKS8_LIMIT:-150} python3 -m torch.distributed.run --nnodes=1 \
            --nproc-per-node ${RANKS8_N:-8} --master-addr 127.0.0.1 --master-port $((29640 + q)) "$R/bench.py" \
            --gpus ${RANKS8_N:-8} --steps 3 --warmup 1 --sets 2 --no-extra \
            > "$OUT/ranks${RANKS8_N:-8}_q$q.json" 2> "$OUT/ranks${RANKS8_N:-8}_q$q.err" || exit 1
        done ;;
    ranks48) for n in 4 8; do
          PSKV_BENCH_BACKEND=gloo PSKV_BENCH_SHARE_GPU=1 timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 \
            --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) "$R/bench.py" --gpus $n --steps 5 \
            --warmup 2 --sets 4 > "$OUT/ranks$n.json" 2> "$OUT/ranks$n.err" || exit 1
        done ;;
    wsweep) for sp in 1e8 1.25e8 5e8; do PROBE_SPACE=$sp PROBE_ROUNDS=10 timeout -k 10 300 python3 -u "$R/tools/zipf_probe.py" "" \
          "PSKV_RB_WBITS=12" "PSKV_RB_WBITS=13" "PSKV_RB_WBITS=14" > "$OUT/wsweep_$sp.log" 2>&1 || exit 1; done &&
        PROBE_WORKLOAD=dense PROBE_ROUNDS=10 timeout -k 10 300 python3 -u "$R/tools/zipf_probe.py" "" "PSKV_RB_WBITS=12" \
          "PSKV_RB_WBITS=13" > "$OUT/wsweep_dense.log" 2>&1 ;;
    zsweep) PROBE_ROUNDS=10 timeout -k 10 500 python3 -u "$R/tools/zipf_probe.py" "" "PSKV_RB_TB=10" "PSKV_RB_APPLY_LOG2=13" \
          "PSKV_RB_WBITS=12" "PSKV_RB_WBITS=10" "PSKV_RB_BIN_BLOCK=512" > "$OUT/zsweep.log" 2>&1 ;;
    k5tests) timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
          "$R/tests/test_gpu_parity.py" "$R/tests/test_fuzz.py" -m gpu \
          -k "zipf or radix or random or accumulate or sentinel or ragged or cfg3 or fuzz" > "$OUT/k5tests.log" 2>&1 ;;
    abs) AB_PROG=sizes timeout -k 10 900 bash "$R/tools/ab_lib.sh" "$(basename "$OUT")/abs" > "$OUT/abs.log" 2>&1 ;;
    fuzz3) FUZZ_SEED0=6500 FUZZ_SCENARIOS=1500 FUZZ_GROUPS=8 timeout -k 10 1000 python3 -u -m pytest \
        "$R/tests/test_fuzz.py" -m gpu -q --timeout 300 --timeout-method thread > "$OUT/fuzz3.log" 2>&1 ;;
    fuzz2) FUZZ_SEED0=5000 FUZZ_SCENARIOS=1500 FUZZ_GROUPS=8 timeout -k 10 1000 python3 -u -m pytest \
        "$R/tests/test_fuzz.py" -m gpu -q --timeout 300 --timeout-method thread > "$OUT/fuzz2.log" 2>&1 ;;
    fuzz) FUZZ_SEED0=${FUZZ_SEED0:-3500} FUZZ_SCENARIOS=${FUZZ_SCENARIOS:-1500} timeout -k 10 1000 python3 -u -m pytest \
        "$R/tests/test_fuzz.py" -m gpu -q --timeout 300 --timeout-method thread > "$OUT/fuzz.log" 2>&1 ;;
    sizetrace) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/sizetrace" -o run \
          -- python3 "$R/tools/size_probe.py" 2,4,8,16,64 20 > "$OUT/sizetrace.log" 2>&1 ;;
    idle) timeout -k 10 120 "$R/tools/micro/idle_launch" > "$OUT/idle_launch.log" 2>&1 ;;
    ztb) timeout -k 10 300 python3 "$R/tools/zipf_probe.py" "" "PSKV_RB_TB=10" "PSKV_RB_TB=10,PSKV_RB_WBITS=12" \
          "PSKV_RB_WBITS=12" > "$OUT/ztb.log" 2>&1 ;;
    sizes_early) for r in 1 2; do for e in 0 1; do
          PSKV_EARLY=$e timeout -k 10 200 python3 "$R/tools/size_probe.py" 2,4,8,16,64 > "$OUT/size_early${e}_$r.log" 2>&1 || exit 1
        done; done ;;
    emu_early) for r in 0 1; do for e in 0 2; do
          PSKV_EARLY=$e PSKV_BENCH_EMULATE=$r/8 timeout -k 10 200 python3 "$R/bench.py" --steps 50 --no-zipf \
            --no-cpu-baseline --no-extra > "$OUT/emu8_${r}_early$e.json" 2> "$OUT/emu8_${r}_early$e.err" || exit 1
        done; done ;;
    bench_early) for r in 1 2; do for e in 2 1; do
          PSKV_EARLY=$e timeout -k 10 200 python3 "$R/bench.py" --steps 50 --no-zipf --no-cpu-baseline --no-extra \
            > "$OUT/bench_early${e}_$r.json" 2> "$OUT/bench_early${e}_$r.err" || exit 1
        done; done ;;
    align_own) for r in 1 2; do for e in 0 3; do
          PSKV_EARLY=$e timeout -k 10 200 python3 "$R/tools/align_probe.py" 0,1,2,3 20 > "$OUT/align_early${e}_$r.log" 2>&1 || exit 1
        done; done ;;
    zwbits) PROBE_ROUNDS=10 timeout -k 10 300 python3 "$R/tools/zipf_probe.py" "" "PSKV_RB_WBITS=12" > "$OUT/zwbits_zipf.log" 2>&1 &&
        PROBE_ROUNDS=10 PROBE_WORKLOAD=dense timeout -k 10 300 python3 "$R/tools/zipf_probe.py" "" "PSKV_RB_WBITS=12" \
          > "$OUT/zwbits_dense.log" 2>&1 ;;
    coldmicro) timeout -k 10 200 "$R/tools/micro/cold_stream" > "$OUT/cold_stream.log" 2>&1 ;;
    coldbench) timeout -k 10 300 python3 "$R/bench.py" --cold-only --steps 50 > "$OUT/cold.json" 2> "$OUT/cold.err" ;;
    coldopts) for o in "" "PSKV_NTP=0" "PSKV_NT=0"; do
          tag=$(echo "x$o" | tr ' =' '__')
          env $o timeout -k 10 300 python3 "$R/bench.py" --cold-only --steps 50 > "$OUT/cold$tag.json" 2> "$OUT/cold$tag.err" || exit 1
        done ;;
    ntp_ab) for r in 1 2; do for e in 0 1; do
          PSKV_NTP=$e timeout -k 10 300 python3 "$R/bench.py" --steps 50 --no-zipf --no-extra \
            --no-cpu-baseline > "$OUT/ntp${e}_$r.json" 2> "$OUT/ntp${e}_$r.err" || exit 1
        done; done ;;
    emu_ntp) for r in 0 1 2 3 4 5 6 7; do for e in 0 1; do
          PSKV_NTP=$e PSKV_BENCH_EMULATE=$r/8 timeout -k 10 200 python3 "$R/bench.py" --steps 50 --no-zipf \
            --no-cpu-baseline --no-extra > "$OUT/emu8_${r}_ntp$e.json" 2> "$OUT/emu8_${r}_ntp$e.err" || exit 1
        done; done ;;
    early_cold) for r in 1 2; do for e in 2 0; do
          PSKV_EARLY=$e timeout -k 10 300 python3 "$R/bench.py" --steps 50 --no-zipf --no-extra --no-cpu-baseline \
            > "$OUT/early${e}_$r.json" 2> "$OUT/early${e}_$r.err" || exit 1
        done; done ;;
    k2g_tune) for o in "" "PSKV_TILE_GRID=4096" "PSKV_UNROLL=4" "PSKV_TILE_GRID=8192"; do
          tag=$(echo "x$o" | tr ' =' '__')
          env $o timeout -k 10 300 python3 "$R/bench.py" --steps 50 --no-zipf --no-extra --no-cpu-baseline \
            > "$OUT/tune$tag.json" 2> "$OUT/tune$tag.err" || exit 1
        done ;;
    smoke) timeout -k 10 300 python3 -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" \
        > "$OUT/smoke.log" 2>&1 ;;
    shardsize) timeout -k 10 400 python3 "$R/tools/shard_size_probe.py" > "$OUT/shard_size.log" 2>&1 &&
        FLUSH=1 timeout -k 10 400 python3 "$R/tools/shard_size_probe.py" > "$OUT/shard_size_flush.log" 2>&1 ;;
    e2e) timeout -k 10 200 python3 "$R/tools/e2e_probe.py" > "$OUT/e2e.log" 2>&1 ;;
    benchdef) t0=$(date +%s); timeout -k 10 900 python3 "$R/bench.py" > "$OUT/benchdef.json" 2> "$OUT/benchdef.err" &&
        echo "bench.py defaults: $(( $(date +%s) - t0 )) s" >> "$OUT/benchdef.err" ;;
    bench) timeout -k 10 400 python3 "$R/bench.py" --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    profile) bash "$R/tools/gpu_profile.sh" "$(basename "$OUT")/prof" > "$OUT/profile.log" 2>&1 ;;
    profile_cold) MODE=cold bash "$R/tools/gpu_profile.sh" "$(basename "$OUT")/prof_cold" > "$OUT/profile_cold.log" 2>&1 ;;
    zipf) timeout -k 10 300 python3 "$R/tools/zipf_probe.py" "" > "$OUT/zipf.log" 2>&1 ;;
    zipf_bin) timeout -k 10 300 python3 "$R/tools/zipf_probe.py" "" "PSKV_RB_BIN_BLOCK=1024" "PSKV_RB_BIN_BLOCK=512" \
        > "$OUT/zipf_bin.log" 2>&1 ;;
    pmcprobe) timeout -k 5 -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcprobe" -o fetch \
          -- python3 "$R/tools/pmc_shard_probe.py" > "$OUT/pmcprobe.log" 2>&1 ;;
    vector) timeout -k 10 600 python3 -u "$R/bench.py" --vector-only --vector-sizes 1000000 \
        > "$OUT/vector_1e6.json" 2> "$OUT/vector_1e6.err" ;;
    asan) SAN=address,undefined timeout -k 10 400 bash "$R/tools/asan_build.sh" > "$OUT/asan_build.log" 2>&1 &&
        A=$R/scratch/asan && export ASAN_OPTIONS=detect_leaks=0 &&
        timeout -k 10 200 "$A/hip_storage_test" > "$OUT/asan_hst.log" 2>&1 &&
        timeout -k 10 200 "$A/kv_client_table_test" --storage hip > "$OUT/asan_kvt.log" 2>&1 &&
        ASAN_OPTIONS=detect_leaks=0:quarantine_size_mb=0 timeout -k 10 200 "$A/ssp_replay" --known-answers \
          --model ssp --staleness 3 --iters 8 --shards 8 --workers 4 > "$OUT/asan_replay.log" 2>&1 &&
        ASAN_OPTIONS=detect_leaks=0:quarantine_size_mb=0 timeout -k 10 200 "$A/ssp_replay" --threads \
          --partition hash --model bsp --iters 8 --shards 8 --workers 4 --features 200000 \
          > "$OUT/asan_replay_hash.log" 2>&1 &&
        { timeout -k 10 200 "$A/ssp_replay" --model ssp --iters 4 --shards 8 --workers 4 \
            > "$OUT/asan_replay_quarantine.log" 2>&1; echo "default quarantine rc=$?" >> "$OUT/asan_replay_quarantine.log"; } ;;
    *) echo "unknown step $step"; exit 9 ;;
  esac
  rc=$?
  echo "step $step rc=$rc" >> "$OUT/steps.log"
  [ $rc -eq 0 ] || exit $rc
done
