"""cfg 5 / SURVEY §8f-1 against an INDEPENDENT restatement of the reference
models (oracle/consistency_ref.py, no code shared with
include/ps/consistency.hpp).

1. The Python models reproduce the reference's own model and util tests
   (tests/golden/reference_known_answers.json), so they are pinned before use.
2. ssp_replay --trace records the model traffic of a replay run -- with the
   oracle storage on CPU here, with the HBM shards (HipStorage<double>) under
   -m gpu -- and every reply it recorded must equal what the Python models
   produce from the same arrivals, and every shard's final contents the dict
   store's.
"""
import os
import struct
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import consistency_ref as cr  # noqa: E402  (test infrastructure: the checker)

EXE = os.path.join(ROOT, "parameter_server_amd", "bin", "ssp_replay")


def _known():
    import json

    with open(os.path.join(ROOT, "tests", "golden", "reference_known_answers.json")) as f:
        return json.load(f)


def _msg(flag, sender, keys=None, vals=None):
    data = []
    if keys is not None:
        data.append(np.asarray(keys, dtype=np.uint32).tobytes())
    if vals is not None:
        data.append(np.asarray(vals, dtype=np.int32).tobytes())
    return cr.Msg(flag, sender, 0, 0, data)


def _model_case_names():
    k = _known()
    return [c["name"] for c in k["model_cases"] + k["restatement_cases"]]


@pytest.mark.parametrize("name", _model_case_names())
def test_models_reproduce_reference_model_tests(name):
    k = _known()
    case = next(c for c in k["model_cases"] + k["restatement_cases"] if c["name"] == name)
    kind = name.split()[0].lower()
    out = []
    md = cr.make_model(kind, cr.MapStore(np.int32), out, staleness=case.get("staleness", 0))
    md.reset(cr.Msg(cr.K_RESET, 9, 0, 0, [np.asarray(case["tids"], dtype=np.uint32).tobytes()]))
    assert out.pop().flag == cr.K_RESET
    for op in case["ops"]:
        if op[0] == "add":
            cr.dispatch(md, _msg(cr.K_ADD, op[1], op[2], op[3]))
        elif op[0] == "get":
            cr.dispatch(md, _msg(cr.K_GET, op[1], op[2]))
        elif op[0] == "clock":
            cr.dispatch(md, _msg(cr.K_CLOCK, op[1]))
        elif op[0] == "pending":  # SSPModel::GetPendingSize(progress)
            assert len(md.pending.get(op[1], [])) == op[2], op
        elif op[0] == "pending_get":  # BSPModel::GetGetPendingSize
            assert len(md.gets) == op[1], op
        elif op[0] == "replies":
            assert len(out) == op[1], op
        else:
            raise AssertionError(op)
    if "replies" in case:
        got = [r for r in out if r.flag == cr.K_GET and len(r.data) == 2]
        assert len(got) == len(case["replies"])
        for r, want in zip(got, case["replies"]):
            assert r.recver == want["recver"]
            if "sender" in want:
                assert r.sender == want["sender"]
            assert np.frombuffer(r.data[0], dtype=np.uint32).tolist() == want["keys"]
            assert np.frombuffer(r.data[1], dtype=np.int32).tolist() == want["vals"]


def test_tracker_reproduces_reference_util_tests():
    k = _known()
    for case in k["util_cases"]:
        if not case["name"].startswith("ProgressTracker"):
            continue
        t = cr.Tracker()
        t.init(case["tids"])
        for op in case["ops"]:
            if op[0] == "num_threads":
                assert len(t.prog) == op[1]
            elif op[0] == "progress":
                assert t.progress(op[1]) == op[2]
            elif op[0] == "valid":
                assert (op[1] in t.prog) == op[2]
            elif op[0] == "min_clock":
                assert t.min_clock == op[1]
            elif op[0] == "advance":
                assert t.advance(op[1]) == op[2], (case["name"], op)
            elif op[0] == "unique_min":
                assert t.unique_min(op[1]) == op[2]
    with pytest.raises(KeyError):  # progresses_.at() on an unknown thread
        t.progress(12345)


def _ranges(shards, n_features, partition):
    if partition == "hash":
        return [(0, n_features)] * shards
    step = n_features // shards
    return [(s * step, n_features if s + 1 == shards else (s + 1) * step) for s in range(shards)]


def _replay_and_check(tmp_path, model, staleness, partition="range", cpu_only=True, workers=4, shards=8,
                      iters=6, batch=30, features=1000000, extra=()):
    if not os.path.exists(EXE):
        import __graft_entry__ as g

        g.build()
    trace = str(tmp_path / f"{model}_{partition}.trace")
    args = [EXE, "--model", model, "--staleness", str(staleness), "--partition", partition,
            "--workers", str(workers), "--shards", str(shards), "--iters", str(iters), "--batch", str(batch),
            "--features", str(features), "--trace", trace, *extra]
    if cpu_only:
        args.append("--cpu-only")
    r = subprocess.run(["timeout", "-k", "10", "600", *args], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "REPLAY OK" in r.stdout
    got = cr.check_trace(trace, model, staleness, _ranges(shards, features, partition))
    assert got["servers"] == shards and got["replies"] > 0
    return got, r.stdout


@pytest.mark.parametrize("model,staleness,partition", [
    ("ssp", 3, "range"), ("ssp", 0, "range"), ("bsp", 0, "range"), ("asp", 0, "range"),
    ("ssp", 3, "hash"), ("bsp", 0, "hash")])
def test_replay_trace_matches_independent_models_cpu(tmp_path, model, staleness, partition):
    got, out = _replay_and_check(tmp_path, model, staleness, partition,
                                 features=1000000 if partition == "range" else 200000)
    if model == "ssp" and staleness == 3:
        assert got["echoes"] > 0  # SSP-released requests were exercised and checked
    print(model, partition, got)


def test_trace_checker_catches_a_changed_reply(tmp_path):
    """The check is not vacuous: one flipped value byte in one recorded Get
    reply makes it fail."""
    _replay_and_check(tmp_path, "ssp", 3)
    trace = tmp_path / "ssp_range.trace"
    raw = bytearray(trace.read_bytes())
    # find a recorded Get reply with values and flip a byte of its first value
    p = 0
    while p < len(raw):
        kind = chr(raw[p])
        if kind == "F":
            _, n = struct.unpack_from("<iQ", raw, p + 1)
            p += 13 + 8 * n
            continue
        s, flag, snd, rcv, mid, nd = struct.unpack_from("<ibiiiI", raw, p + 1)
        q = p + 1 + 21
        lens = []
        for _ in range(nd):
            (ln,) = struct.unpack_from("<Q", raw, q)
            lens.append((q + 8, ln))
            q += 8 + ln
        if kind == "O" and flag == cr.K_GET and nd == 2 and lens[1][1] >= 8:
            raw[lens[1][0] + 3] ^= 0x40
            break
        p = q
    else:
        raise AssertionError("no Get reply in the trace")
    trace.write_bytes(bytes(raw))
    with pytest.raises(AssertionError, match="differs"):
        cr.check_trace(str(trace), "ssp", 3, _ranges(8, 1000000, "range"))


@pytest.mark.gpu
@pytest.mark.parametrize("model,staleness,partition", [
    ("ssp", 3, "range"), ("ssp", 0, "range"), ("bsp", 0, "range"), ("asp", 0, "range"), ("bsp", 0, "hash")])
def test_replay_trace_hip_matches_independent_models(tmp_path, model, staleness, partition):
    """The HBM run's own traffic (HipStorage<double> on 8 shards) checked reply
    by reply against the independent models."""
    got, out = _replay_and_check(tmp_path, model, staleness, partition, cpu_only=False, iters=8,
                                 features=1000000 if partition == "range" else 200000)
    assert "bit-exact" in out
    print(model, partition, got)


@pytest.mark.gpu
def test_replay_trace_hip_example_script_sizes(tmp_path):
    """scripts/logistic_regression.py.example:31-47 sizes (10 workers, batch 100,
    1e6 features), SSP staleness 3 over 8 HBM shards, checked against the
    independent models."""
    got, out = _replay_and_check(tmp_path, "ssp", 3, cpu_only=False, workers=10, iters=6, batch=100)
    assert "batch=100" in out and got["echoes"] > 0
    print(got)
