set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "inline or known_answers or replay" > gpurun_out/r02_inline_tests.log 2>&1 || { tail -40 gpurun_out/r02_inline_tests.log; exit 1; }
tail -2 gpurun_out/r02_inline_tests.log
timeout -k 10 120 ./tools/micro/small_latency > gpurun_out/r02_small_latency.log 2>&1 || { cat gpurun_out/r02_small_latency.log; exit 2; }
cat gpurun_out/r02_small_latency.log
for v in 1 0; do
  PSKV_ISPIN=$v timeout -k 10 300 parameter_server_amd/bin/ssp_replay --model ssp --staleness 3 --iters 16 --shards 8 --workers 8 > gpurun_out/r02_replay_ispin$v.log 2>&1 || { cat gpurun_out/r02_replay_ispin$v.log; exit 3; }
  tail -2 gpurun_out/r02_replay_ispin$v.log
done
