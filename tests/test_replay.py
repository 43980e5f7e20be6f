"""BASELINE config 5 / SURVEY §8f-1: LR-pattern trace through the consistency
models (include/ps/consistency.hpp) over 8 range shards; every Get reply and
the final shard contents must be bit-identical between the CPU oracle storage
and HipStorage<double> (tests/cpp/ssp_replay.cpp)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "parameter_server_amd", "bin", "ssp_replay")


def run(*args):
    if not os.path.exists(EXE):
        import __graft_entry__ as g

        g.build()
    r = subprocess.run(["timeout", "-k", "10", "600", EXE, *args], capture_output=True, text=True)
    return r.returncode, r.stdout + r.stderr


def known_case_names():
    import json

    with open(os.path.join(ROOT, "tests", "golden", "reference_known_answers.json")) as f:
        k = json.load(f)
    return [c["name"] for c in k["model_cases"] + k["util_cases"] + k.get("restatement_cases", [])]


@pytest.mark.parametrize("model", ["ssp", "bsp", "asp"])
def test_replay_cpu_deterministic_and_model_known_answers(model):
    rc, out = run("--cpu-only", "--known-answers", "--model", model, "--iters", "6")
    assert rc == 0, out
    assert "REPLAY OK" in out and "[oracle] model known answers: ok" in out
    # every reference model / util test of the fixture ran and passed
    # (consistency/*_model_test.cpp, util/progress_tracker_test.cpp,
    # util/pending_buffer_test.cpp)
    for name in known_case_names():
        assert f"[oracle] case {name}: ok" in out, name
    if model == "ssp":
        assert "ssp_releases=0 " not in out  # the straggler pattern really exercises staleness


@pytest.mark.gpu
@pytest.mark.parametrize("model,staleness", [("ssp", 3), ("ssp", 0), ("bsp", 0), ("asp", 0)])
def test_replay_hip_vs_cpu(model, staleness):
    rc, out = run("--known-answers", "--model", model, "--staleness", str(staleness), "--iters", "8",
                  "--shards", "8", "--workers", "4")
    assert rc == 0, out
    assert "REPLAY OK (bit-exact)" in out and "[hip] model known answers: ok" in out
    for name in known_case_names():
        assert f"[hip] case {name}: ok" in out, name


@pytest.mark.gpu
@pytest.mark.parametrize("model,staleness,threads", [("ssp", 3, False), ("ssp", 3, True), ("bsp", 0, True)])
def test_replay_example_script_sizes(model, staleness, threads):
    """cfg 5 at the reference example's own sizes
    (scripts/logistic_regression.py.example:31-47): n_features 1e6,
    batch_size 100, 5 workers per node (10 workers: two nodes' worth), over 8
    HBM shards with SSP staleness 3 (and BSP), one server thread per shard in
    the threaded form; every reply and every shard's final contents
    bit-identical to the oracle storage run."""
    args = ["--model", model, "--staleness", str(staleness), "--iters", "6", "--shards", "8",
            "--workers", "10", "--batch", "100", "--features", "1000000"]
    if threads:
        args.append("--threads")
    rc, out = run(*args)
    assert rc == 0, out
    assert "batch=100" in out and "workers=10" in out and "REPLAY OK (bit-exact)" in out


@pytest.mark.parametrize("model", ["ssp", "bsp", "asp"])
def test_replay_threaded_cpu_deterministic(model):
    """One ServerThread per shard (server/server_thread.cpp:20-50): the replies
    of each quiescence window are routed in server order, so two threaded runs
    agree bit for bit."""
    rc, out = run("--cpu-only", "--threads", "--model", model, "--iters", "6", "--workers", "6",
                  "--skew", "2")
    assert rc == 0, out
    assert "REPLAY OK" in out


@pytest.mark.gpu
@pytest.mark.parametrize("model", ["ssp", "bsp"])
def test_replay_threaded_hip_vs_cpu(model):
    """8 server threads drive 8 HipStorage shards concurrently (pskv.h threading
    contract: distinct handles on distinct threads)."""
    rc, out = run("--threads", "--model", model, "--iters", "8", "--shards", "8", "--workers", "4")
    assert rc == 0, out
    assert "REPLAY OK (bit-exact)" in out


@pytest.mark.parametrize("model", ["ssp", "bsp"])
def test_replay_hash_partition_cpu_deterministic(model):
    """The reference Engine's default partitioner (jump consistent hash,
    base/consistent_hashing_partition_manager.hpp) on the worker side; every
    shard owns the whole feature range."""
    rc, out = run("--cpu-only", "--partition", "hash", "--model", model, "--iters", "4",
                  "--features", "200000")
    assert rc == 0, out
    assert "partition=hash" in out and "REPLAY OK" in out


@pytest.mark.gpu
@pytest.mark.parametrize("model,threads", [("bsp", False), ("bsp", True), ("ssp", False)])
def test_replay_hash_partition_hip_vs_cpu(model, threads):
    """The LR app's own configuration (BSP, consistent hashing, Val = double;
    app/logistic_regression.cpp:154, driver/engine.hpp:143-150) over 8 HBM
    shards: every Get reply and every shard's contents bit-identical to the
    oracle storage run."""
    args = ["--partition", "hash", "--model", model, "--iters", "8", "--shards", "8", "--workers", "4",
            "--features", "200000"]
    if threads:
        args.append("--threads")
    rc, out = run(*args)
    assert rc == 0, out
    assert "REPLAY OK (bit-exact)" in out
