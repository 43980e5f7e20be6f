set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/z4
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/z4/pytest.log 2>&1 || { tail -30 gpurun_out/z4/pytest.log; exit 1; }
PROBE_ROUNDS=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/z4 -o zt -- python3 tools/zipf_probe.py "" "PSKV_RB_TB=10" > gpurun_out/z4/probe.log 2>&1
