"""CPU tests of the boundary: libpskv.so loads and exports every symbol
include/pskv.h declares; host-only entry points (range slicing) match the
oracle; the Python mirror of the reference interface behaves like the
reference's template methods.  No kernel is launched here (no GPU)."""
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    with open(os.path.join(ROOT, "include", "pskv.h")) as f:
        txt = f.read()
    return sorted(set(re.findall(r"^\s*(?:[\w\*]+\s+)+\**(pskv_\w+)\(", txt, re.M)))


def test_library_exports_every_declared_symbol():
    from parameter_server_amd import _lib

    syms = header_symbols()
    assert len(syms) >= 20
    assert sorted(_lib.EXPORTED) == syms
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (pskv_\w+)", out))
    missing = [s for s in syms if s not in exported]
    assert not missing, missing


def test_library_is_gfx950_hip_code():
    from parameter_server_amd import _lib

    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", _lib.LIB_PATH],
                         capture_output=True, text=True).stdout
    assert ".hip_fatbin" in out
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_random_access_calibration_library():
    """bench.py's cfg-3 random-access floor (tools/micro/random_access.hip):
    built by __graft_entry__.build() beside libpskv, gfx950 code, exporting the
    two entry points bench.py binds.  Measurement infrastructure only: libpskv
    does not link it."""
    import importlib.util

    spec = importlib.util.spec_from_file_location("pskv_build", os.path.join(ROOT, "parameter_server_amd", "build.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    path = b.build_random_access()
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True).stdout
    assert {"ra_gather", "ra_scatter"} <= set(re.findall(r" T (\w+)", out))
    assert b"gfx950" in open(path, "rb").read()
    from parameter_server_amd import _lib

    deps = subprocess.run(["readelf", "-d", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "random_access" not in deps


def test_abi_version_and_no_device_here():
    from parameter_server_amd import _lib

    assert _lib.lib.pskv_abi_version() == 1
    assert _lib.lib.pskv_device_count() >= 0


def test_bad_arguments_fail_cleanly():
    import ctypes

    from parameter_server_amd import _lib

    h = ctypes.c_void_p()
    assert _lib.lib.pskv_shard_create(0, 10, 5, _lib.PSKV_F32, 0, ctypes.byref(h)) == _lib.PSKV_EINVAL
    assert b"key_begin" in _lib.lib.pskv_last_error()
    assert _lib.lib.pskv_shard_create(0, 0, 100, 7, 0, ctypes.byref(h)) == _lib.PSKV_EINVAL
    assert _lib.lib.pskv_add(None, None, None, 0, 0) == _lib.PSKV_EINVAL
    assert _lib.lib.pskv_sync(None) == _lib.PSKV_EINVAL


def test_shard_without_gpu_raises_loudly():
    import torch

    from parameter_server_amd import PskvError, Shard

    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(PskvError):
        Shard(0, 1000)


def test_range_slice_matches_reference_cases(oracle_mod):
    import json

    from parameter_server_amd import range_slice

    with open(os.path.join(ROOT, "tests", "golden", "reference_known_answers.json")) as f:
        cases = json.load(f)["slice_cases"]
    for c in cases:
        ranges = [tuple(r) for r in c["ranges"]]
        got = [[r, [c["keys"][i] for i in range(s, s + n)]] for r, s, n in range_slice(ranges, c["keys"])]
        assert got == c["expect"], c["cite"]


def test_range_slice_random_vs_oracle(oracle_mod):
    from parameter_server_amd import range_slice

    rng = np.random.default_rng(1)
    for _ in range(200):
        nr = int(rng.integers(1, 9))
        cuts = np.sort(rng.choice(np.arange(1, 2**20), size=nr, replace=False))
        lo = int(rng.integers(0, cuts[0]))
        ranges = [(int(a), int(b)) for a, b in zip(np.r_[lo, cuts[:-1]], cuts)]
        keys = rng.integers(0, 2**20 + 100, size=int(rng.integers(0, 300))).astype(np.uint32)
        if rng.random() < 0.6:
            keys.sort()
        want = oracle_mod.range_slice_ref(ranges, keys)
        got = [(r, [int(k) for k in keys[s:s + n]]) for r, s, n in range_slice(ranges, keys)]
        assert got == want


def _hash_cases():
    import json

    with open(os.path.join(ROOT, "tests", "golden", "reference_known_answers.json")) as f:
        return json.load(f)["hash_slice_cases"]


def test_hash_partition_matches_reference_cases():
    """ConsistentHashingPartitionManager (the reference Engine's default
    partitioner) through the product library: the slices the reference's own
    test asserts (base/consistent_hashing_partition_manager_test.cpp:48-139)."""
    from parameter_server_amd import ConsistentHashingPartitionManager

    for c in _hash_cases():
        pm = ConsistentHashingPartitionManager(c["servers"])
        if "vals" in c:
            got = [[sid, [int(k) for k in kv[0]], [float(v) for v in kv[1]]]
                   for sid, kv in pm.Slice((c["keys"], c["vals"]))]
        else:
            got = [[sid, [int(k) for k in ks]] for sid, ks in pm.Slice(c["keys"])]
        assert got == c["expect"], c["cite"]


def test_oracle_hash_slice_matches_reference_cases(oracle_mod):
    for c in _hash_cases():
        got = [list(x) for x in oracle_mod.hash_slice_ref(c["servers"], c["keys"], c.get("vals"))]
        assert got == c["expect"], c["cite"]


def test_jump_hash_random_vs_oracle(oracle_mod):
    """pskv_jump_hash against the pure-Python restatement: random keys over the
    whole uint32 range (the sentinel 0xFFFFFFFF included), 1..1000 buckets, and
    a batch large enough for the host pool's parallel pieces."""
    from parameter_server_amd import jump_hash

    rng = np.random.default_rng(3)
    for nb in (1, 2, 3, 7, 8, 64, 1000):
        keys = np.concatenate([rng.integers(0, 2**32, size=300), [0, 1, 0xFFFFFFFF]]).astype(np.uint32)
        got = jump_hash(keys, nb)
        want = [oracle_mod.jump_hash_ref(int(k), nb) for k in keys]
        assert got.tolist() == want, nb
    big = rng.integers(0, 2**32, size=(1 << 20) + 12345).astype(np.uint32)
    got = jump_hash(big, 8)
    idx = rng.integers(0, big.size, size=2000)
    assert [int(got[i]) for i in idx] == [oracle_mod.jump_hash_ref(int(big[i]), 8) for i in idx]
    # consistency: growing 8 -> 9 buckets moves only keys into the new bucket
    got9 = jump_hash(big, 9)
    moved = got9 != got
    assert np.all(got9[moved] == 8) and 0.08 < moved.mean() < 0.14
    assert jump_hash(np.zeros(0, np.uint32), 4).size == 0


def test_cpp_boundary_host_cases():
    """tests/cpp/hip_storage_test.cpp range-map cases (host only)."""
    exe = os.path.join(ROOT, "parameter_server_amd", "bin", "hip_storage_test")
    if not os.path.exists(exe):
        from parameter_server_amd import build

        build.build_cpp_tests()
    r = subprocess.run([exe, "--host-only"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout


def test_kv_client_table_host():
    """tests/cpp/kv_client_table_test.cpp on the CPU storage: the reference's
    KVClientTable tests (worker/kv_client_table_test.cpp), typed slicing ==
    the reference's double path, and the worker -> server -> storage system
    test under ASP / SSP / BSP."""
    exe = os.path.join(ROOT, "parameter_server_amd", "bin", "kv_client_table_test")
    if not os.path.exists(exe):
        from parameter_server_amd import build

        build.build_cpp_tests()
    r = subprocess.run(["timeout", "-k", "10", "120", exe, "--host-only"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 failed" in r.stdout


class FakeStorage:
    pass


def test_python_mirror_template_methods():
    """AbstractStorage.Add/Get restate server/abstract_storage.hpp:14-32."""
    from parameter_server_amd import AbstractStorage, CheckError, Flag, Message

    class Fake(AbstractStorage):
        def __init__(self):
            self.added = []

        def SubAdd(self, keys, vals):
            self.added.append((keys.copy(), vals.copy()))

        def SubGet(self, keys):
            return (keys.astype(np.int32) * 10).view(np.uint8)

        def FinishIter(self):
            pass

    s = Fake()
    m = Message()
    m.AddData(np.array([13, 14, 15], np.uint32))
    m.AddData(np.array([1, 2, 3], np.int32))
    s.Add(m)
    assert list(s.added[0][0]) == [13, 14, 15]
    g = Message()
    g.meta.sender, g.meta.recver, g.meta.flag, g.meta.model_id = 2, 0, Flag.kGet, 5
    g.AddData(np.array([7, 8], np.uint32))
    rep = s.Get(g)
    assert (rep.meta.sender, rep.meta.recver, rep.meta.flag, rep.meta.model_id) == (0, 2, Flag.kGet, 5)
    assert len(rep.data) == 2
    assert list(rep.data[1].view(np.int32)) == [70, 80]
    assert np.shares_memory(rep.data[0], g.data[0])  # reply keys alias the request
    with pytest.raises(CheckError):
        s.Add(Message())
    bad = Message()
    bad.AddData(np.array([1], np.uint32))
    bad.AddData(np.array([1], np.uint32))
    with pytest.raises(CheckError):
        s.Get(bad)


def test_python_range_partition_manager_mirror():
    from parameter_server_amd import RangePartitionManager

    pm = RangePartitionManager([0, 1, 2], [(0, 4), (4, 8), (8, 10)])
    sl = pm.Slice((np.array([2, 5, 9], np.uint32), np.array([.2, .5, .9])))
    assert [s for s, _ in sl] == [0, 1, 2]
    assert [float(kv[1][0]) for _, kv in sl] == [.2, .5, .9]
    pm2 = RangePartitionManager([0, 1, 2], [(2, 4), (4, 7), (7, 10)])
    sl2 = pm2.Slice(np.array([2, 8, 9], np.uint32))
    assert [(s, list(k)) for s, k in sl2] == [(0, [2]), (2, [8, 9])]


def test_queue_accounting_per_device(tmp_path):
    """The request server's hardware-queue accounting per device
    (parameter_server_amd/csrc/pskv_queues.h), as a host-only C++
    program built with g++ here: 2 * shards + 1 + extra streams <= GPU_MAX_HW_QUEUES
    on EACH device, with CreateTable's i % ndev binding of 8 server threads
    (driver/engine.hpp:98-110, include/ps/storage_factory.hpp)."""
    import subprocess

    src = os.path.join(ROOT, "tests", "cpp", "queue_accounting_test.cpp")
    exe = str(tmp_path / "queue_accounting_test")
    r = subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-Werror",
                        "-I", os.path.join(ROOT, "parameter_server_amd", "csrc"), src, "-o", exe],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 failed" in r.stdout
