set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/z1
timeout -k 10 120 rocprofv3 -L > gpurun_out/z1/avail.txt 2>&1 || true
PROBE_ROUNDS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/z1 -o zt -- python3 tools/zipf_probe.py > gpurun_out/z1/probe.log 2>&1
