"""bench.py's N > 1 path end to end, as the driver launches it
(`python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr
127.0.0.1 ... bench.py --gpus N`), rehearsed on one GPU: two and four rank
processes,
gloo for the barrier and the reductions, both ranks' shards on cuda:0
(PSKV_BENCH_BACKEND=gloo, PSKV_BENCH_SHARE_GPU=1 — rehearsal knobs the driver
never sets).  Every rank runs cfg 4's self-check (its pulls against a model of
its shard), the timed steps, the Zipf measurement and the
weak-scaled extra; rank 0 prints the one JSON line.  The 8-GPU run is the
driver's; this pins that the multi-rank code path runs and reports what it
should (n_gpus, strong scaling, per-GPU spread, zero push/pull overlap)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 4])
def test_bench_ranks_one_gpu(cuda, world):
    # bounded host waits (SYNC_TIMEOUT_MS): a rank whose work never completes
    # fails with the wait it was in instead of hanging the run
    env = dict(os.environ, PSKV_BENCH_BACKEND="gloo", PSKV_BENCH_SHARE_GPU="1", PSKV_SYNC_TIMEOUT_MS="60000")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "3", "--warmup", "1", "--sets", "4"]
    r = subprocess.run(["timeout", "-k", "10", "400"] + cmd, capture_output=True, text=True, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-5000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == world and res["steps"] == 3 and res["scaling"] == "strong"
    assert res["value"] > 0 and res["unit"] == "GB/s"
    cfg = res["config"]
    assert cfg["key_space"] == 1_000_000_000 and cfg["shard_keys_per_gpu"] == 1_000_000_000 // world
    assert cfg["push_pull_overlap_keys"] == 0
    assert res["per_gpu"]["min_GB/s"] <= res["per_gpu"]["max_GB/s"]
    assert "k_gather" in res["roofline"]["kernels"] and "k_assign_group" in res["roofline"]["kernels"]
    assert "cold" not in res["roofline"]  # the cold form is an N = 1 figure
    assert res["zipf_sparse"]["n_gpus"] == world  # cfg 3 on every rank
    assert res["extra"]["weak_scaled"]["GB/s"] > 0
    # cfg 4's CPU baseline: 8 server threads x 8 MapStorage restatements
    cb = res["cpu_baseline"]
    assert cb["cores"] == 8 and cb["value"] > 0 and cb["kind"] == "port"
    assert cb["one_thread"]["cores"] == 1 and cb["one_thread"]["value"] > 0
