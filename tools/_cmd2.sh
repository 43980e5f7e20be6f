set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/z2
for e in 0 1 2 3 4 8; do
  PSKV_EXP=$e PROBE_ROUNDS=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/z2 -o e$e -- python3 tools/zipf_probe.py > gpurun_out/z2/e$e.log 2>&1 || exit 1
done
