"""GPU parity tests: the HIP path (through the C ABI) against the oracle.

Bar: bit-exact for assign mode (every dtype: the server does no arithmetic),
exact for int32 accumulate, and for float accumulate the recursive-summation
bound stated in DESIGN.md:
    |gpu - ref64| <= 1.01 * (m + 1) * u * (|p0| + sum|v_i|),  u = 2^-24 (f32) / 2^-53 (f64)
with m the number of pushes of that key.
"""
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
DT = {"int32": np.int32, "float32": np.float32, "float64": np.float64}


def tdev(a, cuda, offset=0):
    """numpy -> device tensor (uint32 keys travel as int32 bits).  offset > 0
    returns a view that starts `offset` elements into a larger buffer, so its
    pointer is NOT 16-byte aligned (exercises the scalar kernel variants)."""
    import torch

    a = np.ascontiguousarray(a)
    if a.dtype == np.uint32:
        a = a.view(np.int32)
    t = torch.from_numpy(a.copy())
    if offset:
        pad = torch.zeros(a.size + offset, dtype=t.dtype)
        pad[offset:] = t
        return pad.to(cuda)[offset:]
    return t.to(cuda)


def bits(x):
    x = np.asarray(x)
    return x.view({4: np.uint32, 8: np.uint64}[x.dtype.itemsize])


def assert_bits_equal(got, want, msg=""):
    g, w = bits(got), bits(want)
    if not np.array_equal(g, w):
        bad = np.nonzero(g != w)[0]
        raise AssertionError(f"{msg}: {bad.size} mismatches, first at {bad[:5]}: got {np.asarray(got)[bad[:5]]} "
                             f"want {np.asarray(want)[bad[:5]]}")


def test_cpp_boundary_program(cuda):
    """tests/cpp/hip_storage_test.cpp: the reference's storage unit tests through
    HipStorage<Val> held as std::unique_ptr<AbstractStorage>."""
    exe = os.path.join(ROOT, "parameter_server_amd", "bin", "hip_storage_test")
    r = subprocess.run(["timeout", "-k", "10", "300", exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 failed" in r.stdout


def test_kv_client_table_system_hip(cuda):
    """tests/cpp/kv_client_table_test.cpp with HipStorage<float> shards: worker
    threads with KVClientTable -> sender -> ServerThreads (ASP / SSP / BSP
    models over HBM shards built by CreateTable) -> replies -> CallbackRunner;
    read-your-writes and the final contents of every shard, bit for bit."""
    exe = os.path.join(ROOT, "parameter_server_amd", "bin", "kv_client_table_test")
    r = subprocess.run(["timeout", "-k", "10", "300", exe, "--storage", "hip"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 failed" in r.stdout


def known():
    with open(os.path.join(GOLDEN, "reference_known_answers.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("case", known()["storage_cases"], ids=lambda c: c["name"])
def test_reference_known_answers_hipstorage(cuda, case):
    from parameter_server_amd import HipStorage, Message

    dt = DT[case["dtype"]]
    s = HipStorage(dt, 0, 1 << 20)
    try:
        for op in case["ops"]:
            m = Message()
            m.AddData(np.array(op[1], np.uint32))
            if op[0] == "add":
                m.AddData(np.array(op[2], dt))
                s.Add(m)
            else:
                rep = s.Get(m)
                assert len(rep.data) == 2
                assert list(rep.data[0].view(np.uint32)) == op[1]
                assert_bits_equal(rep.data[1].view(dt), np.array(op[2], dt), case["cite"])
        s.FinishIter()
    finally:
        s.close()


def golden_cases():
    with open(os.path.join(GOLDEN, "assign_vectors.json")) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("layout", [(0, 5000), (2**31 - 700, 2**31 + 700)], ids=["low", "mid"])
@pytest.mark.parametrize("path", ["host", "device", "device_hint", "device_grouped_hint", "device_unaligned"])
@pytest.mark.parametrize("case", golden_cases(), ids=lambda c: c["name"])
def test_golden_vectors(cuda, case, path, layout):
    import parameter_server_amd as ps

    z = np.load(os.path.join(GOLDEN, "assign_vectors.npz"))
    dt = DT[case["dtype"]]
    name = case["name"]
    with ps.Shard(layout[0], layout[1], dt, overflow_slots=1 << 14) as sh:
        adds = [(z[f"{name}/add{j}/keys"], z[f"{name}/add{j}/vals"]) for j in range(case["n_adds"])]
        if path == "host":
            for k, v in adds:
                sh.add(k, v)
        elif path == "device_grouped_hint":
            sh.add_grouped([(tdev(k, cuda), tdev(v, cuda)) for k, v in adds], sorted_hint=True)
        else:
            off = 1 if path == "device_unaligned" else 0
            for k, v in adds:
                sh.add(tdev(k, cuda, off), tdev(v, cuda, off), sorted_hint=(path == "device_hint"))
        q = z[f"{name}/get/keys"]
        got = sh.get(q)
        sh.sync()
    assert_bits_equal(got, z[f"{name}/get/expect"], f"{name}/{path}/{layout}")


@pytest.mark.parametrize("dt", [np.int32, np.float32, np.float64])
def test_random_assign_parity_all_paths(cuda, oracle_mod, dt):
    import torch

    import parameter_server_amd as ps

    rng = np.random.default_rng(123)
    kb, ke = 10_000, 10_000 + 300_000
    ref = oracle_mod.MapStorageRef(dt)
    with ps.Shard(kb, ke, dt, overflow_slots=1 << 16) as sh:
        for step in range(12):
            n = int(rng.integers(0, 70_000))
            kind = step % 4
            if kind == 0:      # unsorted, duplicates, some out of range
                k = rng.integers(kb - 2000, ke + 2000, size=n)
            elif kind == 1:    # sorted with runs of duplicates
                k = np.sort(rng.integers(kb, ke, size=n))
            elif kind == 2:    # contiguous window (dense)
                b = int(rng.integers(kb, ke - n - 1)) if n < ke - kb - 2 else kb
                k = np.arange(b, b + n)
            else:              # sorted but with out-of-range tail -> sorted hint must repair
                k = np.sort(rng.integers(kb, ke + 50, size=n))
            k = k.astype(np.uint32)
            v = (rng.standard_normal(n) * 1e3).astype(dt)
            mode = step % 3
            if mode == 0:
                sh.add(k, v)
            elif mode == 1:
                sh.add(tdev(k, cuda), tdev(v, cuda), sorted_hint=True)
            else:
                sh.add(tdev(k, cuda, 3), tdev(v, cuda, 3), sorted_hint=bool(step & 1))
            ref.add(k, v)
        q = np.concatenate([np.arange(kb - 3000, ke + 3000),
                            rng.integers(0, 2**32, size=5000)]).astype(np.uint32)
        got_h = sh.get(q)
        got_d = sh.get(tdev(q, cuda)).cpu().numpy().view(dt)
        torch.cuda.synchronize()
        sh.sync()
    want = ref.get(q)
    assert_bits_equal(got_h, want, "host get")
    assert_bits_equal(got_d, want, "device get")


def test_sorted_hint_on_unsorted_data_is_repaired(cuda, oracle_mod):
    import parameter_server_amd as ps

    rng = np.random.default_rng(9)
    ref = oracle_mod.MapStorageRef(np.float32)
    with ps.Shard(0, 100_000, np.float32) as sh:
        before = sh.info()["n_general_launches"]
        k = rng.integers(0, 100_000, size=50_000).astype(np.uint32)   # unsorted, duplicates
        v = rng.standard_normal(k.size).astype(np.float32)
        sh.add(tdev(k, cuda), tdev(v, cuda), sorted_hint=True)
        ref.add(k, v)
        got = sh.get(np.arange(100_000, dtype=np.uint32))
        assert sh.info()["n_general_launches"] > before
    assert_bits_equal(got, ref.get(np.arange(100_000, dtype=np.uint32)), "repair")


@pytest.mark.parametrize("nb", [2, 7, 64, 70])
def test_grouped_overlapping_batches_later_wins(cuda, oracle_mod, nb):
    """Grouped sorted Add (K2g key-tile owner): batches overlap; call order decides."""
    import parameter_server_amd as ps

    rng = np.random.default_rng(nb)
    size = 200_000
    dense = np.zeros(size, np.float32)
    batches = []
    for j in range(nb):
        n = int(rng.integers(1, 40_000))
        if j % 3 == 0:
            b = int(rng.integers(0, size - n))
            k = np.arange(b, b + n)
        else:
            k = np.sort(rng.integers(0, size, size=n))
        k = k.astype(np.uint32)
        v = rng.standard_normal(n).astype(np.float32)
        batches.append((k, v))
        oracle_mod.dense_last_wins(dense, 0, k, v)
    with ps.Shard(0, size, np.float32) as sh:
        sh.add_grouped([(tdev(k, cuda), tdev(v, cuda)) for k, v in batches], sorted_hint=True)
        got = sh.get(np.arange(size, dtype=np.uint32))
        info = sh.info()
    assert info["n_sorted_launches"] >= 1
    assert_bits_equal(got, dense, f"grouped nb={nb}")


def test_grouped_get_matches_single(cuda):
    import torch

    import parameter_server_amd as ps

    rng = np.random.default_rng(4)
    with ps.Shard(0, 1 << 20, np.float64) as sh:
        k = np.arange(1 << 20, dtype=np.uint32)
        v = rng.standard_normal(k.size)
        sh.add(k, v)
        qs = [rng.integers(0, 1 << 21, size=int(n)).astype(np.uint32) for n in (1, 5, 4096, 100_001, 0, 77)]
        outs = [torch.empty(q.size, dtype=torch.float64, device=cuda) for q in qs]
        sh.get_grouped([(tdev(q, cuda), o) for q, o in zip(qs, outs)])
        torch.cuda.synchronize()
        for q, o in zip(qs, outs):
            assert_bits_equal(o.cpu().numpy(), sh.get(q), "grouped get")
            want = np.where(q < (1 << 20), v[np.minimum(q, (1 << 20) - 1)], 0.0)
            assert_bits_equal(o.cpu().numpy(), want, "vs numpy")


@pytest.mark.parametrize("dt", [np.int32, np.float32, np.float64])
def test_accumulate_mode(cuda, dt):
    import parameter_server_amd as ps

    rng = np.random.default_rng(77)
    kb, size = 500, 50_000
    p64 = np.zeros(size, np.float64)
    a64 = np.zeros(size, np.float64)
    cnt = np.zeros(size, np.int64)
    acc_i = np.zeros(size, np.int64)
    with ps.Shard(kb, kb + size, dt, mode="accumulate") as sh:
        for step in range(6):
            n = int(rng.integers(1000, 80_000))
            k = (rng.zipf(1.2, size=n) % size + kb).astype(np.uint32) if step % 2 else \
                np.sort(rng.integers(kb, kb + size, size=n)).astype(np.uint32)
            if dt is np.int32:
                v = rng.integers(-2**31, 2**31 - 1, size=n, dtype=np.int64).astype(np.int32)
            else:
                v = rng.standard_normal(n).astype(dt)
            if step % 3 == 2:
                sh.add(tdev(k, cuda), tdev(v, cuda), sorted_hint=True)
            else:
                sh.add(k, v)
            idx = k.astype(np.int64) - kb
            np.add.at(p64, idx, v.astype(np.float64))
            np.add.at(a64, idx, np.abs(v.astype(np.float64)))
            np.add.at(cnt, idx, 1)
            np.add.at(acc_i, idx, v.astype(np.int64))
        got = sh.get(np.arange(kb, kb + size, dtype=np.uint32))
    if dt is np.int32:
        want = ((acc_i + 2**31) % 2**32 - 2**31).astype(np.int32)  # wrap-around sum is exact
        assert_bits_equal(got, want, "int32 accumulate")
    else:
        u = 2.0**-24 if dt is np.float32 else 2.0**-53
        tol = 1.01 * (cnt + 1) * u * a64
        err = np.abs(got.astype(np.float64) - p64)
        assert np.all(err <= tol), f"max err/tol {np.max(err / np.maximum(tol, 1e-300))}"


def _dense_windows(rng, kb, size, n_windows):
    """Overlapping contiguous key windows inside [kb, kb+size): long ones (many
    8 Ki-key chunks), short ones, odd lengths and unaligned starts."""
    out = []
    for w in range(n_windows):
        n = int(rng.choice([1, 3, 1000, 8191, 8192, 20_001, 70_000]))
        first = int(rng.integers(kb, kb + size - n + 1))
        if w % 3 == 0:
            first -= (first - kb) % 4  # 4-aligned offset: the 16-byte RMW path
        out.append(np.arange(first, first + n, dtype=np.uint32))
    return out


@pytest.mark.parametrize("dt", [np.int32, np.float32, np.float64])
@pytest.mark.parametrize("path", ["host", "device_hint", "device_hint_unaligned"])
def test_accumulate_dense_windows_sequential_bits(cuda, dt, path):
    """K7 (dense accumulate): every key gets one RMW summing the covering
    windows in call order, so the result equals sequential accumulation in the
    value dtype BIT FOR BIT (np.add.at is sequential, in dtype arithmetic)."""
    import parameter_server_amd as ps

    rng = np.random.default_rng(5)
    kb, size = 1000, 200_000
    want = np.zeros(size, dt)
    with ps.Shard(kb, kb + size, dt, mode="accumulate") as sh:
        sh.set_timing(True)
        for call in range(4):
            wins = _dense_windows(rng, kb, size, 9 if call % 2 else 1)
            vals = [(rng.integers(-2**31, 2**31 - 1, size=k.size, dtype=np.int64).astype(np.int32)
                     if dt is np.int32 else rng.standard_normal(k.size).astype(dt)) for k in wins]
            if path == "host":
                sh.add_grouped(list(zip(wins, vals)))
            else:
                off = 1 if path.endswith("unaligned") else 0
                sh.add_grouped([(tdev(k, cuda), tdev(v, cuda, off)) for k, v in zip(wins, vals)],
                               sorted_hint=True)
            for k, v in zip(wins, vals):
                np.add.at(want, k.astype(np.int64) - kb, v)
        got = sh.get(np.arange(kb, kb + size, dtype=np.uint32))
        assert sh.kernel_time(_lib_k("ACC_DENSE"))["launches"] > 0, "dense accumulate kernel did not run"
        if path != "host":
            assert sh.kernel_time(_lib_k("DENSE_CHECK"))["launches"] > 0
    assert_bits_equal(got, want, f"dense accumulate {path}")


def _lib_k(name):
    from parameter_server_amd import _lib

    return getattr(_lib, "PSKV_K_" + name)


@pytest.mark.parametrize("dt", [np.int32, np.float32])
def test_accumulate_dense_lookalike_falls_back(cuda, dt):
    """A hinted window whose endpoints look dense but whose inside is not (two
    keys swapped, one key repeated): K6 must reject the group before any RMW,
    and the K4a accumulate applies it instead (order-free: int32 exact, float
    within the stated bound)."""
    import parameter_server_amd as ps

    rng = np.random.default_rng(9)
    kb, size = 0, 100_000
    wins = _dense_windows(rng, kb, size, 6)
    big = [i for i, k in enumerate(wins) if k.size >= 1000][0]
    k = wins[big].copy()
    k[10], k[11] = k[11], k[10]
    k[500] = k[499]
    wins[big] = k
    vals = [(rng.integers(-1000, 1000, size=w.size).astype(np.int32) if dt is np.int32
             else rng.standard_normal(w.size).astype(dt)) for w in wins]
    p64, a64, cnt = np.zeros(size), np.zeros(size), np.zeros(size, np.int64)
    with ps.Shard(kb, kb + size, dt, mode="accumulate") as sh:
        sh.add_grouped([(tdev(w, cuda), tdev(v, cuda)) for w, v in zip(wins, vals)], sorted_hint=True)
        got = sh.get(np.arange(kb, kb + size, dtype=np.uint32))
    for w, v in zip(wins, vals):
        np.add.at(p64, w.astype(np.int64) - kb, v.astype(np.float64))
        np.add.at(a64, w.astype(np.int64) - kb, np.abs(v.astype(np.float64)))
        np.add.at(cnt, w.astype(np.int64) - kb, 1)
    if dt is np.int32:
        assert_bits_equal(got, p64.astype(np.int32), "int32 fallback")
    else:
        tol = 1.01 * (cnt + 1) * 2.0**-24 * a64
        assert np.all(np.abs(got.astype(np.float64) - p64) <= tol)


def test_baseline_size_dense_roundtrip(cuda):
    """cfg 2 at full size: 1e8-float shard, 1M-key contiguous windows at seed-42
    bases; grouped sorted Add then grouped Get returns the last write of every
    key (windows may repeat: later wins), untouched keys read 0."""
    import torch

    import parameter_server_amd as ps
    from parameter_server_amd import workload

    space, J = 100_000_000, 16
    bases = workload.dense_bases(J, space)
    batches = workload.dense_batches(J, space, device=cuda)
    with ps.Shard(0, space, np.float32) as sh:
        sh.add_grouped(batches, sorted_hint=True)
        outs = [torch.empty_like(v) for _, v in batches]
        sh.get_grouped([(k, o) for (k, _), o in zip(batches, outs)])
        last = {}
        for j, b in enumerate(bases):
            last[int(b)] = j
        for j, b in enumerate(bases):
            want = batches[last[int(b)]][1]
            assert torch.equal(outs[j].view(torch.int32), want.view(torch.int32)), f"window {j}"
        # a never-written window reads zeros
        free = next(x for x in range(0, space, 1_000_000) if x not in last)
        z = sh.get(torch.arange(free, free + 1_000_000, dtype=torch.int32, device=cuda))
        assert int(torch.count_nonzero(z)) == 0
        dv = sh.dense_view()
        b0 = int(bases[0])
        assert torch.equal(dv[b0:b0 + 1_000_000].view(torch.int32), outs[0].view(torch.int32))
        sh.sync()


@pytest.mark.parametrize("space,R,steps", [(100_000_000, 16, 20), (1_000_000_000, 4, 6)],
                         ids=["cfg2_1e8", "cold_1e9"])
def test_bench_headline_form_bit_exact(cuda, oracle_mod, space, R, steps):
    """The benchmarked state itself: bench.py's own sets and
    Form — 64 x 1M windows at seed-42-family 1M-aligned bases per set, R sets
    rotated, the sorted-hint grouped Add (K2g dense mode + verification + K4r),
    then the grouped Get (K1) of the window slots the push left free (zero
    push/pull overlap).  Every pull of every step is compared bit for bit with
    the oracle's sequential last-write-wins restatement (map_storage.hpp:22-23;
    never-written keys read 0, :33-37), and at the end the whole dense array.
    cfg2_1e8 is the headline (N = 1, cfg 2); cold_1e9 is roofline.cold's form."""
    import sys

    import torch

    import parameter_server_amd as ps

    sys.path.insert(0, ROOT)
    import bench

    dev = torch.device(cuda)
    J, B = 64, 1_000_000
    n_pulls = [len(bench.plan_pull(0, 1, J, B, r, bench.plan_rank(0, 1, J, B, r)[4])[0]) for r in range(R)]
    sp = None if space == 100_000_000 else space
    sets = [bench.make_set(0, 1, J, B, dev, r, space=sp, n_pull=None if sp is None else n_pulls[r])
            for r in range(R)]
    assert all(bench.overlap_keys(s) == 0 for s in sets)
    ref = np.zeros(space, np.float32)
    host = [[(f, v.cpu().numpy()) for (_, f, _), (_, v) in zip(s["slices"], s["batches"])] for s in sets]
    with ps.Shard(0, space, np.float32) as sh:
        sh.set_stream(torch.cuda.current_stream().cuda_stream)
        form = bench.Form(sh, sets, dev)
        for i in range(steps):
            t = i % R
            for f, v in host[t]:
                oracle_mod.dense_last_wins(ref, 0, np.arange(f, f + v.size, dtype=np.uint32), v)
            form.step(i)
            torch.cuda.synchronize()
            for (_, f, n), o in zip(form.pull_slices[t], form.outs[t]):
                assert_bits_equal(o.cpu().numpy(), ref[f:f + n], f"step {i}: pull of window {f}")
        dense = sh.dense_view().cpu().numpy()
        sh.set_stream(None)
        sh.sync()
    assert_bits_equal(dense, ref, "whole shard after the steps")
    assert np.count_nonzero(ref) > 0


def test_zipf_batches_parity(cuda, oracle_mod):
    """cfg 3 shape at reduced key space: unsorted Zipf(0.99) pushes with heavy
    duplicates go through the default unhinted path (K5: LDS super-chunk dedup,
    key buckets, bucket-owned resolve) and match the oracle."""
    import torch

    import parameter_server_amd as ps
    from parameter_server_amd import workload

    space = 2_000_000
    batches = workload.zipf_batches(4, space, batch=262_144, device=cuda)
    dense = np.zeros(space, np.float32)
    with ps.Shard(0, space, np.float32) as sh:
        sh.add_grouped(batches[:2])
        for k, v in batches[2:]:
            sh.add(k, v)
        for k, v in batches:
            oracle_mod.dense_last_wins(dense, 0, k.cpu().numpy().view(np.uint32), v.cpu().numpy())
        got = sh.get(torch.arange(space, dtype=torch.int32, device=cuda)).cpu().numpy()
    hot = np.bincount(batches[0][0].cpu().numpy().view(np.uint32).astype(np.int64)).max()
    assert hot > 1000  # the hot key really is hot
    assert_bits_equal(got, dense, "zipf")


@pytest.mark.parametrize("ntp", [0, 1])
def test_zipf_pulls(cuda, oracle_mod, ntp):
    """K1 on Zipf pulls (hot keys repeated hundreds of times per chunk),
    out-of-range keys, the sentinel 0xFFFFFFFF, never-written keys, and chunks
    that mix dense runs at every phase with scattered keys — bit-exact against
    the oracle, the parameters written by sorted windows with cached and with
    non-temporal (option NTP) stores.  (Round 3's pull-key dedup variant,
    GET_DEDUP, measured no gain, and its non-temporal parameter loads, GET_NTP,
    lost to NTP; both were removed in round 4.)"""
    import torch

    import parameter_server_amd as ps
    from parameter_server_amd import workload

    space = 2_000_000
    zb = workload.zipf_batches(3, space, batch=300_000, device=cuda)
    ref = oracle_mod.MapStorageRef(np.float32)
    with ps.Shard(0, space, np.float32, overflow_slots=1 << 12, options={"NTP": ntp}) as sh:
        for k, v in zb:
            sh.add(k, v)
            ref.add(k.cpu().numpy().view(np.uint32), v.cpu().numpy())
        extra = np.array([0xFFFFFFFF, space + 5, space + 5, 2**31 + 9], np.uint32)
        xv = np.arange(4, dtype=np.float32) + 0.5
        sh.add(extra, xv)
        ref.add(extra, xv)
        # windows through the sorted device path (K2g: stores cached or nt)
        wins = [np.arange(b, b + 20_000, dtype=np.uint32) for b in (7001, 9003, 40_000, 1_000_001)]
        wv = [np.random.default_rng(int(w[0])).standard_normal(w.size).astype(np.float32) for w in wins]
        sh.add_grouped([(tdev(w, cuda), tdev(v, cuda)) for w, v in zip(wins, wv)], sorted_hint=True)
        for w, v in zip(wins, wv):
            ref.add(w, v)
        q = zb[0][0].cpu().numpy().view(np.uint32).copy()
        q[1000:1000 + 64] = np.arange(5000, 5064, dtype=np.uint32)       # dense runs inside scattered chunks
        q[4096:4096 + 8192] = np.arange(7001, 7001 + 8192, dtype=np.uint32)  # a whole chunk run, phase 1
        q[20480:20480 + 8192] = np.arange(9003, 9003 + 8192, dtype=np.uint32)  # phase 3
        q[7:40] = 0xFFFFFFFF
        q[50:60] = space + 5
        q[-9:] = np.arange(space + 100, space + 109, dtype=np.uint32)     # never written: 0
        outs = [torch.empty(q.size // 2, dtype=torch.float32, device=cuda),
                torch.empty(q.size - q.size // 2, dtype=torch.float32, device=cuda)]
        parts = [tdev(q[:q.size // 2], cuda), tdev(q[q.size // 2:], cuda)]
        sh.get_grouped(list(zip(parts, outs)))
        got = torch.cat(outs).cpu().numpy()
        assert sh.get_option("NTP") == ntp
    assert_bits_equal(got, ref.get(q), f"zipf pulls, NTP {ntp}")


@pytest.mark.parametrize("mode", ["assign", "accumulate"])
def test_cfg3_full_size_zipf_parity(cuda, oracle_mod, mode):
    """cfg 3 at its stated size: a 1e8-key float shard, 8 x 1M unsorted
    Zipf(0.99) pushes (workload.zipf_batches: seed-7 key permutation), as one
    grouped unhinted Add (K5) — the bench's sparse step.  Assign: the WHOLE dense
    array equals the oracle's sequential last-write-wins restatement
    (map_storage.hpp:17-27) bit for bit, and a Get of every pushed key returns
    it.  Accumulate: every key within the stated recursive-summation bound of
    the float64 sum, untouched keys exactly 0."""
    import torch

    import parameter_server_amd as ps
    from parameter_server_amd import workload

    space = 100_000_000
    zb = workload.zipf_batches(8, space, device=cuda)
    keys = [k.cpu().numpy().view(np.uint32) for k, _ in zb]
    vals = [v.cpu().numpy() for _, v in zb]
    with ps.Shard(0, space, np.float32, mode=mode) as sh:
        sh.add_grouped(zb)
        allk = torch.cat([k for k, _ in zb])
        pulled = sh.get(allk).cpu().numpy()
        dense = sh.dense_view().cpu().numpy()
        sh.sync()
    allk_np = np.concatenate(keys).astype(np.int64)
    if mode == "assign":
        ref = np.zeros(space, np.float32)
        for k, v in zip(keys, vals):
            oracle_mod.dense_last_wins(ref, 0, k, v)
        assert_bits_equal(dense, ref, "cfg 3 dense array")
        assert_bits_equal(pulled, ref[allk_np], "cfg 3 pulls")
        return
    p64 = np.zeros(space, np.float64)
    a64 = np.zeros(space, np.float64)
    for k, v in zip(keys, vals):
        oracle_mod.accumulate_ref(p64, a64, 0, k, v)
    cnt = np.bincount(allk_np, minlength=space)
    tol = 1.01 * (cnt + 1) * 2.0**-24 * a64
    err = np.abs(dense.astype(np.float64) - p64)
    assert np.all(err <= tol), f"{int(np.sum(err > tol))} keys outside the bound"
    assert np.all(dense[cnt == 0] == 0)
    assert cnt.max() > 40_000  # the hot key: ~48k hits per batch
    assert_bits_equal(pulled, dense[allk_np], "cfg 3 pulls (accumulate)")


def test_overflow_table_growth_and_edges(cuda, oracle_mod):
    import parameter_server_amd as ps

    rng = np.random.default_rng(31)
    ref = oracle_mod.MapStorageRef(np.float32)
    with ps.Shard(2**32 - 1000, 2**32, np.float32, overflow_slots=64) as sh:
        for step in range(5):
            k = rng.integers(0, 2**32, size=30_000).astype(np.uint32)   # almost all overflow
            k[:10] = 0xFFFFFFFF                                         # the LDS sentinel key, in range
            k[10:20] = 2**32 - 1000
            v = rng.standard_normal(k.size).astype(np.float32)
            sh.add(k, v)                     # host path: the inserting workgroup grows the table
            ref.add(k, v)
            sh.sync()
        info = sh.info()
        assert info["overflow_capacity"] >= 2 * info["overflow_count"] > 0
        q = np.concatenate([k, rng.integers(0, 2**32, size=1000).astype(np.uint32),
                            np.array([0xFFFFFFFF, 0, 2**32 - 1000], np.uint32)])
        got = sh.get(q)
        # empty calls are no-ops
        sh.add(np.zeros(0, np.uint32), np.zeros(0, np.float32))
        assert sh.get(np.zeros(0, np.uint32)).size == 0
        sh.add_grouped([])
    assert_bits_equal(got, ref.get(q), "overflow")


class _AccRef:
    """Accumulate-mode model for int32 (wrap-around sums are exact in any
    order): key -> value, missing keys 0."""

    def __init__(self):
        self.m = {}

    def add(self, k, v):
        for kk, vv in zip(k.tolist(), v.astype(np.int64).tolist()):
            self.m[kk] = (self.m.get(kk, 0) + vv) & 0xFFFFFFFF

    def get(self, k):
        return np.array([self.m.get(kk, 0) for kk in k.tolist()], dtype=np.uint32).view(np.int32)


def _burst(rng, i, kb, ke, n_new, sort):
    """One push: n_new NEW out-of-range keys (below the range and above it;
    fresh every burst), every one repeated 1-3 times, plus in-range keys."""
    below = np.arange(kb - 1 - i * n_new // 2, kb - 1 - (i + 1) * n_new // 2, -1, dtype=np.int64)
    above = ke + 10 + np.arange(i * (n_new - below.size), (i + 1) * (n_new - below.size), dtype=np.int64) * 3
    k = np.concatenate([below, above, rng.integers(kb, ke, size=n_new // 4)])
    k = np.repeat(k, rng.integers(1, 4, size=k.size)).astype(np.uint32)
    if sort:
        k.sort(kind="stable")
    else:
        rng.shuffle(k)
    return k


# one push / device path of the overflow inserters (each a single workgroup that
# reserves room, growing the table on the device): K2g + replay (K4r), the
# replay folded into the Get (K1r), K5's out-of-range bucket, K4 + its
# oor-only replay, the host K5 path and K8 messages
BURST_PATHS = ["sorted_hint", "add_get", "unsorted", "stamps", "host", "inline"]


@pytest.mark.parametrize("mode", ["assign", "accumulate"])
@pytest.mark.parametrize("path", BURST_PATHS)
def test_overflow_burst_parity(cuda, oracle_mod, path, mode):
    """The reference's last range server stores every key the slicer cannot
    place, however many (range_partition_manager.hpp:26-27,
    map_storage.hpp:22-23): bursts of 5,000 NEW out-of-range keys into a
    64-slot table, with no sync between them, through every inserter, match
    the reference bit for bit -- assign against MapStorageRef (last occurrence
    wins), accumulate (int32, exact) against the sequential sum -- read back
    both by device Gets between the bursts and by a host Get at the end; the
    table grew on the device."""
    import torch

    import parameter_server_amd as ps

    rng = np.random.default_rng(100 + 2 * BURST_PATHS.index(path) + (mode == "accumulate"))
    dt = np.float32 if mode == "assign" else np.int32
    ref = oracle_mod.MapStorageRef(dt) if mode == "assign" else _AccRef()
    kb, ke = 1_000_000, 1_010_000
    opts = {"GENERAL": "stamps"} if path == "stamps" else {}
    seen = []
    with ps.Shard(kb, ke, dt, mode=mode, overflow_slots=64, options=opts) as sh:
        for i in range(3):
            k = _burst(rng, i, kb, ke, 5000, sort=path in ("sorted_hint", "add_get"))
            v = (rng.integers(-1000, 1000, size=k.size)).astype(dt)
            if mode == "assign":
                v = (rng.standard_normal(k.size) * 100).astype(dt)
            ref.add(k, v)
            seen.append(k)
            q = np.unique(np.concatenate(seen))
            if path == "inline":  # K8: messages of <= 256 keys
                for j in range(0, k.size, 200):
                    sh.add(k[j:j + 200], v[j:j + 200])
                got = sh.get(q)
            elif path == "host":
                sh.add(k, v)
                got = sh.get(q)
            elif path == "add_get":
                out = torch.empty(q.size, dtype=torch.float32 if dt == np.float32 else torch.int32, device=cuda)
                sh.add_get_grouped([(tdev(k, cuda), tdev(v, cuda))], [(tdev(q, cuda), out)], sorted_hint=True)
                got = out.cpu().numpy()
            else:
                sh.add(tdev(k, cuda), tdev(v, cuda), sorted_hint=path == "sorted_hint")
                got = sh.get(tdev(q, cuda)).cpu().numpy()
            assert_bits_equal(got, ref.get(q), f"{path}/{mode} burst {i}")
        sh.sync()
        info = sh.info()
        n_out = int(np.count_nonzero((q < kb) | (q >= ke)))
        assert info["overflow_count"] == n_out, (info, n_out)
        assert info["overflow_capacity"] >= 2 * n_out > 64
        assert_bits_equal(sh.get(q), ref.get(q), f"{path}/{mode} after sync")


@pytest.mark.parametrize("path", ["unsorted", "sorted_hint"])
def test_overflow_growth_many_doublings_in_one_launch(cuda, path):
    """One device Add of 2 Mi NEW out-of-range keys into a 64-slot table: the
    single inserting workgroup (K5's out-of-range bucket, or the replay behind
    K2g) reserves room for everything it is about to insert, so the table goes
    from 64 slots to >= 4 Mi inside ONE launch (a 65 536-fold growth, the
    whole rehash and fill done by that workgroup) and every key lands; values
    bit-exact (each key once, so last-write-wins is the value itself)."""
    import torch

    import parameter_server_amd as ps

    n = 2 << 20
    rng = np.random.default_rng(77)
    k = (np.uint64(3_000_000) + np.arange(n, dtype=np.uint64) * np.uint64(7)).astype(np.uint32)  # all above the range
    if path == "unsorted":
        rng.shuffle(k)
    v = rng.standard_normal(n).astype(np.float32)
    with ps.Shard(0, 1_000_000, np.float32, overflow_slots=64) as sh:
        sh.add(tdev(k, cuda), tdev(v, cuda), sorted_hint=path == "sorted_hint")
        got = sh.get(tdev(k, cuda)).cpu().numpy()
        torch.cuda.synchronize()
        sh.sync()
        info = sh.info()
        assert info["overflow_count"] == n and info["overflow_capacity"] >= 2 * n, info
        assert_bits_equal(got, v, f"{path}: 2 Mi new out-of-range keys")
        assert_bits_equal(sh.get(k[::97]), v[::97], f"{path}: host Get after sync")


def test_overflow_growth_concurrent_shards(cuda, oracle_mod):
    """The reference runs one server thread per range (simple_id_mapper.cpp:28-31),
    each with its own storage; here 8 shards on 8 threads push device bursts
    of new out-of-range keys at once, so growth requests from several shards'
    kernels (K5's out-of-range bucket, the replay after K2g) are outstanding
    together and the ONE grow service answers them in turn.  Every shard,
    read back on its own thread after each burst and again at the end, matches
    its own MapStorageRef bit for bit."""
    import threading

    import parameter_server_amd as ps

    n_sh, bursts = 8, 3
    shards = [ps.Shard(1_000_000 + 20_000 * i, 1_010_000 + 20_000 * i, np.float32, overflow_slots=64)
              for i in range(n_sh)]
    pushes = [[] for _ in range(n_sh)]
    reads = [[] for _ in range(n_sh)]
    errors = []

    def work(i):
        try:
            sh = shards[i]
            kb, ke = 1_000_000 + 20_000 * i, 1_010_000 + 20_000 * i
            rng = np.random.default_rng(700 + i)
            seen = []
            for b in range(bursts):
                k = _burst(rng, b, kb, ke, 3000, sort=i % 2 == 1)
                v = (rng.standard_normal(k.size) * 100).astype(np.float32)
                pushes[i].append((k, v))
                seen.append(k)
                q = np.unique(np.concatenate(seen))
                sh.add(tdev(k, cuda), tdev(v, cuda), sorted_hint=i % 2 == 1)
                reads[i].append((q, sh.get(tdev(q, cuda)).cpu().numpy()))
            sh.sync()
            reads[i].append((q, sh.get(q)))
        except Exception as e:  # re-raised on the main thread
            errors.append((i, e))

    try:
        th = [threading.Thread(target=work, args=(i,)) for i in range(n_sh)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        assert not any(t.is_alive() for t in th), "a shard thread did not finish"
        assert not errors, errors
        for i, sh in enumerate(shards):
            ref = oracle_mod.MapStorageRef(np.float32)
            for b, (k, v) in enumerate(pushes[i]):
                ref.add(k, v)
                q, got = reads[i][b]
                assert_bits_equal(got, ref.get(q), f"shard {i} burst {b}")
            q, got = reads[i][-1]
            assert_bits_equal(got, ref.get(q), f"shard {i} after sync")
            kb, ke = 1_000_000 + 20_000 * i, 1_010_000 + 20_000 * i
            n_out = int(np.count_nonzero((q < kb) | (q >= ke)))
            info = sh.info()
            assert info["overflow_count"] == n_out and info["overflow_capacity"] >= 2 * n_out > 64, (i, info)
    finally:
        for sh in shards:
            sh.close()


def test_overflow_growth_timeout_fails_loudly(cuda):
    """SYNC_TIMEOUT_MS = 1 bounds a growth request's wait on the device at
    ~1 ms, about the grow service's polling period: a burst far past the table
    either grows in time or drops keys, and then the next sync says so
    (PSKV_ESTATE, "dropped") -- never a silent loss: a sync that succeeds
    means every key is there."""
    import torch

    import parameter_server_amd as ps
    from parameter_server_amd import PskvError, _lib

    rng = np.random.default_rng(5)
    with ps.Shard(0, 1000, np.float32, overflow_slots=64, options={"SYNC_TIMEOUT_MS": 1}) as sh:
        k = np.arange(10_000, 60_000, dtype=np.uint32)
        rng.shuffle(k)
        v = np.ones(k.size, np.float32)
        dk, dv = tdev(k, cuda), tdev(v, cuda)
        sh.add(dk, dv)
        torch.cuda.synchronize()  # the Add ran under the 1 ms device bound
        sh.set_option("SYNC_TIMEOUT_MS", 0)  # (the host waits below are not under test)
        try:
            sh.sync()
            ok = True
        except PskvError as e:
            assert e.code == _lib.PSKV_ESTATE and "dropped" in str(e), str(e)
            ok = False
        if ok:
            assert np.all(sh.get(k) == 1.0)


def test_bounded_waits_report_pending_work(cuda):
    """Every host wait is bounded (option SYNC_TIMEOUT_MS, round 5; VERDICT r4
    item 1): with ~3 s of earlier work on the stream the shard runs on (torch's
    current stream, pskv_set_stream), a sync and a host Get fail with
    PSKV_ESTATE after the 300 ms bound, the message naming the stream waited
    for and the last kernel the shard queued; nothing is cancelled, so once the
    bound is lifted the same shard completes and reads what was written,
    bit-exact."""
    import torch

    import parameter_server_amd as ps
    from parameter_server_amd import PskvError, _lib

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(50_000_000)
    e1.record()
    torch.cuda.synchronize()
    cycles_per_ms = 50_000_000 / max(e0.elapsed_time(e1), 1e-3)
    k = np.arange(0, 5000, 3, dtype=np.uint32)
    v = (k * 0.5).astype(np.float32)
    with ps.Shard(0, 10_000, np.float32, options={"SYNC_TIMEOUT_MS": 300}) as sh:
        assert sh.get_option("SYNC_TIMEOUT_MS") == 300
        sh.set_stream(torch.cuda.current_stream().cuda_stream)
        sh.add(k, v)
        sh.sync()
        # device inputs made BEFORE the sleep: a pageable host-to-device copy
        # made after it would wait for it inside torch
        kd, vd = tdev(k, cuda), tdev(v + 1, cuda)
        torch.cuda.synchronize()
        torch.cuda._sleep(int(3000 * cycles_per_ms))  # ~3 s ahead of the shard's work
        sh.add(kd, vd)  # queued behind it (K5)
        # the sync waits behind the sleep and the queued K5 Add; the host Get
        # of 1000 keys goes out as inline K8 launches and polls their reply
        for what, call, last in (("sync", sh.sync, "K5"), ("host get", lambda: sh.get(k[:1000]), "K8")):
            with pytest.raises(PskvError) as ei:
                call()
            assert ei.value.code == _lib.PSKV_ESTATE, what
            msg = str(ei.value)
            assert "not complete after" in msg and "stream" in msg and last in msg, (what, msg)
        sh.set_option("SYNC_TIMEOUT_MS", 0)  # unbounded: the queued work completes
        sh.sync()
        assert np.array_equal(sh.get(k), v + 1)
        sh.set_stream(None)


def test_size_mismatch_is_rejected(cuda):
    from parameter_server_amd import CheckError, HipStorage, Message

    s = HipStorage(np.float32, 0, 1000)
    m = Message()
    m.AddData(np.array([1, 2, 3], np.uint32))
    m.AddData(np.array([1.0, 2.0], np.float32))
    with pytest.raises(CheckError):
        s.Add(m)
    s.close()


def test_external_stream_and_timing(cuda):
    import torch

    import parameter_server_amd as ps
    from parameter_server_amd import _lib

    st = torch.cuda.Stream()
    with ps.Shard(0, 1 << 22, np.float32) as sh:
        sh.set_stream(st.cuda_stream)
        sh.set_timing(True)
        with torch.cuda.stream(st):
            k = torch.arange(1 << 22, dtype=torch.int32, device=cuda)
            v = torch.rand(1 << 22, device=cuda)
            sh.add(k, v, sorted_hint=True)
            out = sh.get(k)
        st.synchronize()
        assert torch.equal(out, v)
        t = sh.kernel_time(_lib.PSKV_K_GATHER)
        assert t["launches"] == 1 and t["total_ms"] > 0 and t["elements"] == 1 << 22
        sh.set_stream(None)


@pytest.mark.parametrize("nb", [2, 9, 64, 65])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("early", [0, 1])
def test_grouped_dense_windows_mode(cuda, oracle_mod, nb, dtype, early):
    """All batches contiguous windows (dense mode of the grouped sorted Add):
    unaligned bases, overlaps, ragged lengths; later batches win.  early:
    option EARLY forced off / on (K2g's own-range chunks, loads before the
    prologue; f64 ignores it)."""
    import parameter_server_amd as ps

    rng = np.random.default_rng(100 + nb)
    size = 300_000
    dense = np.zeros(size, dtype)
    batches = []
    for j in range(nb):
        n = int(rng.integers(1, 50_000))
        b = int(rng.integers(0, size - n))
        k = np.arange(b, b + n, dtype=np.uint32)
        v = rng.standard_normal(n).astype(dtype)
        batches.append((k, v))
        oracle_mod.dense_last_wins(dense, 0, k, v)
    with ps.Shard(0, size, dtype, options={"EARLY": early}) as sh:
        before = sh.info()["n_general_launches"]
        sh.add_grouped([(tdev(k, cuda), tdev(v, cuda)) for k, v in batches], sorted_hint=True)
        got = sh.get(np.arange(size, dtype=np.uint32))
    assert_bits_equal(got, dense, f"dense windows nb={nb}")


@pytest.mark.parametrize("key_begin", [0, 1, 2, 3])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("early", [0, 1])
def test_dense_windows_every_phase(cuda, oracle_mod, key_begin, dtype, early):
    """cfg 4's producer windows start at any key: windows at every phase against
    the 16-byte parameter slots (the shard's key_begin shifts it once more),
    lengths around the dense chunk (8192 keys) and its multiples, whole windows
    repeated (a later one covers an earlier one), partial overlaps, tiny
    windows; grouped sorted Add (K2g dense mode: phase-shifted slot stores),
    then Gets of every window, of windows at other phases and of the whole
    array (K1: the two-slot loads) — bit-exact against the oracle."""
    import torch

    import parameter_server_amd as ps

    rng = np.random.default_rng(700 + key_begin)
    size = 600_000
    kb = key_begin
    dense = np.zeros(size, dtype)
    wins = []
    for n in (8192 * 3, 8192 * 3 + 1, 8192 * 3 - 1, 8192 * 5 + 2, 8192 + 3, 8191, 8193, 4, 3, 1, 2, 5, 70_001):
        for ph in range(4):
            b = int(rng.integers(0, (size - n) // 4)) * 4 + ph
            wins.append((b, n))
    wins.append(wins[0])                               # repeated whole: the later one wins
    b0, n0 = wins[5]
    wins.append((b0 + 1000, 30_000))                   # partial overlap of a phase-1 window
    rng.shuffle(wins)
    batches = []
    for b, n in wins:
        k = np.arange(kb + b, kb + b + n, dtype=np.uint32)
        v = rng.standard_normal(n).astype(dtype)
        batches.append((k, v))
    with ps.Shard(kb, kb + size, dtype, options={"EARLY": early}) as sh:
        for g in (batches[:27], batches[27:]):         # two grouped calls
            sh.add_grouped([(tdev(k, cuda), tdev(v, cuda)) for k, v in g], sorted_hint=True)
            for k, v in g:
                oracle_mod.dense_last_wins(dense, kb, k, v)
        outs = [torch.empty(k.size, dtype=torch.float32 if dtype == np.float32 else torch.float64,
                            device=cuda) for k, _ in batches]
        sh.get_grouped([(tdev(k, cuda), o) for (k, _), o in zip(batches, outs)])
        for (k, _), o in zip(batches, outs):
            assert_bits_equal(o.cpu().numpy(), dense[k.astype(np.int64) - kb], f"pull of window at {k[0]}")
        for ph in range(4):                            # pulls at other phases than the pushes
            b = int(rng.integers(0, (size - 40_000) // 4)) * 4 + ph
            k = np.arange(kb + b, kb + b + 40_000, dtype=np.uint32)
            assert_bits_equal(sh.get(tdev(k, cuda)).cpu().numpy(), dense[b:b + 40_000], f"pull phase {ph}")
        got = sh.get(np.arange(kb, kb + size, dtype=np.uint32))
    assert_bits_equal(got, dense, f"dense windows at every phase, key_begin {kb}")


def test_grouped_dense_lookalike_is_repaired(cuda, oracle_mod):
    """Endpoints say 'dense window' but the keys are not contiguous (two swapped,
    one duplicated): the per-element check must tag the group for repair."""
    import parameter_server_amd as ps

    rng = np.random.default_rng(8)
    size = 100_000
    dense = np.zeros(size, np.float32)
    batches = []
    for j in range(6):
        b = int(rng.integers(0, size - 20_000))
        k = np.arange(b, b + 20_000, dtype=np.uint32)
        if j == 2:
            k[100], k[200] = k[200], k[100]      # unsorted, same endpoints
        if j == 4:
            k[5000] = k[5001]                    # duplicate, same endpoints
        v = rng.standard_normal(k.size).astype(np.float32)
        batches.append((k, v))
        oracle_mod.dense_last_wins(dense, 0, k, v)
    with ps.Shard(0, size, np.float32) as sh:
        sh.add_grouped([(tdev(k, cuda), tdev(v, cuda)) for k, v in batches], sorted_hint=True)
        got = sh.get(np.arange(size, dtype=np.uint32))
    assert_bits_equal(got, dense, "lookalike")


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("phase", [0, 1, 3])
@pytest.mark.parametrize("early", [0, 1])
def test_grouped_dense_lookalike_never_writes_missing_keys(cuda, oracle_mod, dtype, phase, early):
    """A wrong sorted hint on batches whose endpoints span exactly n - 1 keys
    but which repeat one key and so MISS another, where no other batch of the
    group holds the missing key: the sorted pass must not write the missing
    key (the replay rewrites only the group's own keys), so it keeps its prior
    value (map_storage.hpp:22-23: an Add touches only the keys it carries).
    Whole chunks (>= 8 Ki keys), the chunk holding the window's phase shift,
    partial chunks and the batch tail, at window phases 0 / 1 / 3."""
    import parameter_server_amd as ps

    rng = np.random.default_rng(11 + phase)
    size = 200_000
    prior = rng.standard_normal(size).astype(dtype)
    dense = prior.copy()
    specs = [(1_000 + phase, 30_000, [5, 9_000, 20_000, 29_998]),   # whole chunks + tail
             (60_000 + phase, 8_200, [8_190]),                      # the phase-shift chunk boundary
             (100_000 + phase, 700, [0, 350]),                      # one partial chunk
             (150_000 + phase, 20_000, [])]                         # a clean window
    batches = []
    for b, n, dups in specs:
        k = np.arange(b, b + n, dtype=np.uint32)
        for i in dups:  # k[i] repeats k[i + 1] (same endpoints): key b + i is missing
            if i + 1 < n:
                k[i] = k[i + 1]
            else:
                k[i] = k[i - 1]
        v = rng.standard_normal(n).astype(dtype)
        batches.append((k, v))
    with ps.Shard(0, size, dtype, options={"EARLY": early}) as sh:
        sh.add(np.arange(size, dtype=np.uint32), prior)
        for k, v in batches:
            oracle_mod.dense_last_wins(dense, 0, k, v)
        sh.add_grouped([(tdev(k, cuda), tdev(v, cuda)) for k, v in batches], sorted_hint=True)
        got = sh.get(np.arange(size, dtype=np.uint32))
    assert_bits_equal(got, dense, f"lookalike missing keys, phase {phase}")


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("n", [4, 700, 30_000])
def test_host_sorted_group_with_duplicates_spanning_n_minus_1(cuda, oracle_mod, dtype, n):
    """HOST batches (the reference's zmq frames) that are sorted, so the CPU
    check passes them to the sorted path, but repeat a key and miss another, so
    their endpoints span exactly n - 1 keys like a dense window: the grouped
    Add must still give the LAST occurrence of the repeated key and leave the
    missing key alone (map_storage.hpp:22-23).  E.g. keys [5, 6, 6, 8]."""
    import parameter_server_amd as ps

    rng = np.random.default_rng(n)
    size = 200_000
    prior = rng.standard_normal(size).astype(dtype)
    dense = prior.copy()
    batches = []
    for j, b in enumerate((1_000, 40_000, 70_001)):
        k = np.arange(b, b + n, dtype=np.uint32)
        if j != 1:  # batch 1 stays a true dense window
            i = n // 2 if n > 4 else 1
            k[i + 1] = k[i]  # sorted, a repeat of k[i], key b + i + 1 missing
        v = rng.standard_normal(n).astype(dtype)
        batches.append((k, v))
    with ps.Shard(0, size, dtype, options={"INLINE": 0}) as sh:  # n = 4 too: the staged path
        sh.add(np.arange(size, dtype=np.uint32), prior)
        for k, v in batches:
            oracle_mod.dense_last_wins(dense, 0, k, v)
        sh.add_grouped(batches)  # host buffers: the CPU check proves them sorted
        got = sh.get(np.arange(size, dtype=np.uint32))
    assert_bits_equal(got, dense, f"host sorted look-alike, n={n}")


@pytest.mark.parametrize("mode,dtype", [("assign", np.float32), ("assign", np.float64),
                                        ("accumulate", np.float64), ("accumulate", np.int32)])
def test_radix_path_hot_bucket_many_rounds(cuda, oracle_mod, mode, dtype):
    """K5: every key in ONE key bucket (and the out-of-range bucket), far more
    entries than the apply workgroup's LDS table holds -> multi-round apply."""
    import parameter_server_amd as ps

    opts = {"GENERAL": "radix"}  # K5 for accumulate too

    rng = np.random.default_rng(55)
    size = 1 << 25                      # bucket width 64 Ki keys
    kb = 1000
    batches = []
    for j in range(12):
        n = 60_000 + j
        k = rng.integers(kb, kb + 65_536, size=n)          # dense bucket 0
        k[:500] = rng.integers(kb + size, 2**32, size=500)  # out-of-range bucket
        k = k.astype(np.uint32)
        if dtype is np.int32:
            v = rng.integers(-2**31, 2**31 - 1, size=n, dtype=np.int64).astype(np.int32)
        else:
            v = rng.standard_normal(n).astype(dtype)
        batches.append((k, v))
    q = np.unique(np.concatenate([k for k, _ in batches]))
    with ps.Shard(kb, kb + size, dtype, mode=mode, overflow_slots=1 << 15, options=opts) as sh:
        sh.add_grouped([(tdev(k, cuda), tdev(v, cuda)) for k, v in batches])
        got = sh.get(q)
        sh.sync()
    if mode == "assign":
        ref = oracle_mod.MapStorageRef(dtype)
        for k, v in batches:
            ref.add(k, v)
        assert_bits_equal(got, ref.get(q), "radix assign")
    else:
        acc = {}
        for k, v in batches:
            for kk, vv in zip(k.tolist(), v.tolist()):
                acc[kk] = acc.get(kk, 0) + vv
        want = np.array([acc[int(x)] for x in q])
        if dtype is np.int32:
            assert_bits_equal(got, ((want + 2**31) % 2**32 - 2**31).astype(np.int32), "radix int acc")
        else:
            assert np.allclose(got, want, rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("mode", ["assign", "accumulate"])
@pytest.mark.parametrize("path", ["host", "device_hint", "device_hint_single", "device_unhinted"])
def test_windows_ending_at_top_of_key_space(cuda, oracle_mod, mode, path):
    """Dense windows and sorted batches that end at key 0xFFFFFFFF in a shard
    whose key_end is 2^32: no uint32 wrap in the window / density / tile
    arithmetic of K2, K2g, K6/K7 or the host checks.  int32 values: assign and
    accumulate are both bit-exact."""
    import parameter_server_amd as ps

    rng = np.random.default_rng(2024)
    kb = 2**32 - (1 << 20)
    ref = np.zeros(1 << 20, np.int64)
    batches = []
    for j in range(9):
        if j % 3 == 0:
            n = int(rng.choice([1, 7, 4096, 70_001]))
            k = np.arange(2**32 - n, 2**32, dtype=np.uint64).astype(np.uint32)      # window to the top
        elif j % 3 == 1:
            f = int(rng.integers(kb, 2**32 - 50_000))
            k = np.arange(f, f + 50_000, dtype=np.uint64).astype(np.uint32)         # window below
        else:
            k = np.sort(rng.integers(2**32 - 300_000, 2**32, size=40_000)).astype(np.uint32)  # sorted, dups
            k[-3:] = 0xFFFFFFFF
        v = rng.integers(-2**31, 2**31 - 1, size=k.size, dtype=np.int64).astype(np.int32)
        batches.append((k, v))
    for k, v in batches:
        idx = k.astype(np.int64) - kb
        if mode == "assign":
            oracle_mod.dense_last_wins(ref, kb, k, v.astype(np.int64))
        else:
            np.add.at(ref, idx, v.astype(np.int64))
    want = ((ref + 2**31) % 2**32 - 2**31).astype(np.int32)
    with ps.Shard(kb, 2**32, np.int32, mode=mode) as sh:
        if path == "host":
            sh.add_grouped(batches)
        elif path == "device_hint":
            sh.add_grouped([(tdev(k, cuda), tdev(v, cuda)) for k, v in batches], sorted_hint=True)
        elif path == "device_hint_single":
            for k, v in batches:
                sh.add(tdev(k, cuda), tdev(v, cuda), sorted_hint=True)
        else:
            sh.add_grouped([(tdev(k, cuda), tdev(v, cuda)) for k, v in batches])
        got = sh.get(np.arange(kb, 2**32, dtype=np.uint64).astype(np.uint32))
    assert_bits_equal(got, want, f"{mode} {path} top of key space")


@pytest.mark.parametrize("layout", ["sentinel_dense", "sentinel_overflow"])
@pytest.mark.parametrize("path", ["device", "host"])
def test_accumulate_sentinel_key_duplicates(cuda, layout, path):
    """Key 0xFFFFFFFF (the LDS tables' EMPTY, kept in a side word) pushed many
    times in one batch: its duplicates fold into ONE entry per super-chunk
    (regression: every duplicate used to claim ownership of the side word)."""
    import parameter_server_amd as ps

    kb, ke = (2**32 - 1000, 2**32) if layout == "sentinel_dense" else (0, 1000)
    for n_ff in (1, 2, 5, 3000):
        k = np.array([kb + 5] * 3 + [2**32 - 1] * n_ff + [2**32 - 2] * 2, np.uint32)
        v = np.arange(1, k.size + 1, dtype=np.int32)
        with ps.Shard(kb, ke, np.int32, mode="accumulate", overflow_slots=1 << 10) as sh:
            if path == "device":
                sh.add_grouped([(tdev(k, cuda), tdev(v, cuda))])
            else:
                sh.add(k, v)
            got = sh.get(np.array([kb + 5, 2**32 - 1, 2**32 - 2], np.uint32))
        want = np.array([v[:3].sum(), v[3:3 + n_ff].sum(), v[-2:].sum()], np.int64).astype(np.int32)
        assert_bits_equal(got, want, f"sentinel x{n_ff}")


@pytest.mark.parametrize("mode", ["assign", "accumulate"])
def test_many_ragged_batches_grouped(cuda, oracle_mod, mode):
    """150 ragged batches in one grouped Add and one grouped Get (more than the
    64 a launch's kernarg holds, so both calls are cut into several launches):
    empty, 1-key and 20 K-key batches, unsorted with duplicates and
    out-of-range keys.  int32 values: assign and accumulate are bit-exact."""
    import torch

    import parameter_server_amd as ps

    rng = np.random.default_rng(150)
    kb, size = 1000, 300_000
    batches = []
    for j in range(150):
        n = int(rng.choice([0, 1, 2, 17, 999, 20_000]))
        k = rng.integers(0, kb + size + 5000, size=n).astype(np.uint32)
        v = rng.integers(-2**31, 2**31 - 1, size=n, dtype=np.int64).astype(np.int32)
        batches.append((k, v))
    q_batches = [rng.integers(0, kb + size + 5000, size=int(rng.choice([0, 1, 3000]))).astype(np.uint32)
                 for _ in range(150)]
    if mode == "assign":
        ref = oracle_mod.MapStorageRef(np.int32)
        for k, v in batches:
            ref.add(k, v)
        wants = [ref.get(q) for q in q_batches]
    else:
        acc = {}
        for k, v in batches:
            for kk, vv in zip(k.tolist(), v.tolist()):
                acc[kk] = acc.get(kk, 0) + vv
        wrap = lambda x: ((np.asarray(x, np.int64) + 2**31) % 2**32 - 2**31).astype(np.int32)
        wants = [wrap([acc.get(int(x), 0) for x in q]) for q in q_batches]
    with ps.Shard(kb, kb + size, np.int32, mode=mode, overflow_slots=1 << 16) as sh:
        sh.add_grouped([(tdev(k, cuda), tdev(v, cuda)) for k, v in batches])
        outs = [torch.empty(q.size, dtype=torch.int32, device=cuda) for q in q_batches]
        sh.get_grouped([(tdev(q, cuda), o) for q, o in zip(q_batches, outs)])
        torch.cuda.synchronize()
        for j, (o, w) in enumerate(zip(outs, wants)):
            assert_bits_equal(o.cpu().numpy(), w, f"{mode} batch {j}")


def test_radix_accumulate_full_key_space_edges(cuda):
    """K5 accumulate on the reference's argument-less storage (the whole uint32
    key space in one shard, 16 GiB of int32 in HBM): the K5b -> K5c pair
    hand-off carries key offset 0xFFFFFFFF and 0 like any other; int32 sums
    wrap and are exact."""
    import parameter_server_amd as ps

    rng = np.random.default_rng(91)
    batches = []
    for j in range(5):
        n = 200_000 + 17 * j
        k = rng.integers(0, 2**32, size=n, dtype=np.uint64)
        k[:3000] = rng.choice(np.array([0, 1, 2**32 - 1, 2**32 - 2, 2**31], np.uint64), size=3000)
        k = k.astype(np.uint32)
        v = rng.integers(-2**31, 2**31 - 1, size=n, dtype=np.int64).astype(np.int32)
        batches.append((k, v))
    acc = {}
    for k, v in batches:
        for kk, vv in zip(k.tolist(), v.tolist()):
            acc[kk] = acc.get(kk, 0) + vv
    q = np.array(sorted(acc) + [12345, 2**32 - 3], dtype=np.uint32)
    want = np.array([acc.get(int(x), 0) for x in q], np.int64)
    want = ((want + 2**31) % 2**32 - 2**31).astype(np.int32)
    with ps.Shard(0, 2**32, np.int32, mode="accumulate") as sh:
        sh.add_grouped([(tdev(k, cuda), tdev(v, cuda)) for k, v in batches])
        got = sh.get(q)
    assert_bits_equal(got, want, "full key space accumulate")


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_radix_accumulate_zipf_split_launches(cuda, dtype):
    """cfg-3-shaped accumulate through K5 (bin, resolve, pair apply): Zipf
    pushes over several launch pieces (> 8 M keys for 4-byte values), checked
    against float64 sums with the recursive-summation bound."""
    import torch

    import parameter_server_amd as ps

    rng = np.random.default_rng(123)
    size = 20_000_000
    n_total = 9_000_000 if dtype is np.float32 else 4_600_000
    perm_seed = 5
    ranks = rng.zipf(1.1, size=n_total) % size
    keys = ((ranks * 2654435761 + perm_seed) % size).astype(np.uint32)
    vals = rng.standard_normal(n_total).astype(dtype)
    cut = n_total // 3
    idx = keys.astype(np.int64)
    p64 = np.bincount(idx, weights=vals.astype(np.float64), minlength=size)
    a64 = np.bincount(idx, weights=np.abs(vals.astype(np.float64)), minlength=size)
    cnt = np.bincount(idx, minlength=size)
    with ps.Shard(0, size, dtype, mode="accumulate") as sh:
        sh.add_grouped([(tdev(keys[:cut], cuda), tdev(vals[:cut], cuda)),
                        (tdev(keys[cut:], cuda), tdev(vals[cut:], cuda))])
        got = sh.get(torch.arange(size, dtype=torch.int32, device=cuda)).cpu().numpy()
    u = 2.0**-24 if dtype is np.float32 else 2.0**-53
    tol = 1.01 * (cnt + 1) * u * a64
    err = np.abs(got.astype(np.float64) - p64)
    assert np.all(err <= tol), f"max err/tol {np.max(err / np.maximum(tol, 1e-300))}"


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_radix_path_long_runs(cuda, oracle_mod, dtype):
    """K5 resolve with runs longer than its registers hold (few, narrow key
    buckets; every super-chunk puts ~45 entries into each) but few enough
    entries for one table: the strided single-round path."""
    import parameter_server_amd as ps

    rng = np.random.default_rng(77)
    kb, size = 5000, 4096
    dense = np.zeros(size, dtype)
    batches = []
    for j in range(3):
        k = rng.integers(kb, kb + size, size=5000 + j).astype(np.uint32)
        v = rng.standard_normal(k.size).astype(dtype)
        batches.append((k, v))
        oracle_mod.dense_last_wins(dense, kb, k, v)
    with ps.Shard(kb, kb + size, dtype) as sh:
        sh.add_grouped([(tdev(k, cuda), tdev(v, cuda)) for k, v in batches])
        got = sh.get(np.arange(kb, kb + size, dtype=np.uint32))
    assert_bits_equal(got, dense, "long runs")


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_radix_path_split_launches(cuda, oracle_mod, dtype):
    """An unsorted group larger than one K5 launch (1024 super-chunks: 8 M keys
    for 4-byte values, 4 M for 8-byte) is cut into consecutive pieces, a batch
    split across two of them; duplicates across the cut keep call order."""
    import torch

    import parameter_server_amd as ps

    rng = np.random.default_rng(99)
    size = 3_000_000
    n_big = 9_000_000 if dtype is np.float32 else 4_500_000
    big = rng.integers(0, size, size=n_big).astype(np.uint32)
    vb = rng.standard_normal(n_big).astype(dtype)
    small = rng.integers(0, size, size=700_000).astype(np.uint32)
    vs = rng.standard_normal(small.size).astype(dtype)
    dense = np.zeros(size, dtype)
    oracle_mod.dense_last_wins(dense, 0, small, vs)
    oracle_mod.dense_last_wins(dense, 0, big, vb)
    with ps.Shard(0, size, dtype) as sh:
        sh.add_grouped([(tdev(small, cuda), tdev(vs, cuda)), (tdev(big, cuda), tdev(vb, cuda))])
        got = sh.get(torch.arange(size, dtype=torch.int32, device=cuda)).cpu().numpy()
    assert_bits_equal(got, dense, "split")


def test_general_path_stamps_variant_matches(cuda, oracle_mod):
    """The K4 stamp path (shard option GENERAL = stamps) as the unhinted
    general path."""
    import parameter_server_amd as ps

    rng = np.random.default_rng(66)
    ref = oracle_mod.MapStorageRef(np.float32)
    with ps.Shard(0, 500_000, np.float32, overflow_slots=1 << 14, options={"GENERAL": "stamps"}) as sh:
        assert sh.get_option("GENERAL") == 0
        for _ in range(4):
            k = rng.integers(0, 520_000, size=90_000).astype(np.uint32)
            v = rng.standard_normal(k.size).astype(np.float32)
            sh.add(tdev(k, cuda), tdev(v, cuda))
            ref.add(k, v)
        q = np.arange(0, 520_000, dtype=np.uint32)
        got = sh.get(q)
    assert_bits_equal(got, ref.get(q), "stamps path")


@pytest.mark.parametrize("dtype", [np.int32, np.float32])
def test_accumulate_stamps_variant_k4a(cuda, dtype):
    """K4a accumulate (LDS chunk sums + one atomic add per distinct key per
    chunk), selected by the shard option GENERAL = stamps: int32 exact, float
    within bound."""
    import parameter_server_amd as ps

    rng = np.random.default_rng(67)
    size = 300_000
    p64, a64, cnt = np.zeros(size), np.zeros(size), np.zeros(size, np.int64)
    with ps.Shard(0, size, dtype, mode="accumulate", options={"GENERAL": "stamps"}) as sh:
        for _ in range(3):
            k = (rng.zipf(1.3, size=120_000) % size).astype(np.uint32)
            v = (rng.integers(-1000, 1000, size=k.size).astype(np.int32) if dtype is np.int32
                 else rng.standard_normal(k.size).astype(dtype))
            sh.add(tdev(k, cuda), tdev(v, cuda))
            np.add.at(p64, k.astype(np.int64), v.astype(np.float64))
            np.add.at(a64, k.astype(np.int64), np.abs(v.astype(np.float64)))
            np.add.at(cnt, k.astype(np.int64), 1)
        got = sh.get(np.arange(size, dtype=np.uint32))
    if dtype is np.int32:
        assert_bits_equal(got, p64.astype(np.int32), "k4a int32")
    else:
        tol = 1.01 * (cnt + 1) * 2.0**-24 * a64
        assert np.all(np.abs(got.astype(np.float64) - p64) <= tol)


def _pinned(a):
    """numpy view of a page-locked copy of a (torch pinned host memory)."""
    import torch

    a = np.ascontiguousarray(a)
    t = torch.from_numpy(a.view(np.int32) if a.dtype == np.uint32 else a).pin_memory()
    out = t.numpy()
    return out.view(np.uint32) if a.dtype == np.uint32 else out


@pytest.mark.parametrize("pinned_path", ["dma", "default"])
@pytest.mark.parametrize("pageable_path", ["dma", "staged"])
@pytest.mark.parametrize("mode", ["assign", "accumulate"])
def test_pinned_host_buffers_direct_dma(cuda, oracle_mod, mode, pageable_path, pinned_path):
    """Page-locked caller buffers (the zmq frames after the SURVEY §8f-3 mailbox
    change): same results as pageable buffers, for sorted, dense and unsorted
    batches, Add and Get.  pinned_path "dma": Adds and Gets DMA'd directly
    from / to them at every size; "default": Adds below 2 MiB take the staging
    copy and Gets up to 8 MiB run K1 on them in place (zero copy)."""
    import parameter_server_amd as ps

    opts = {}
    if pinned_path == "dma":
        opts.update(DMA_MIN_BYTES_PINNED=0, FRAME_ZC_MAX_BYTES=0)
    # pageable buffers go by direct DMA (forced at every size: by default only
    # calls of >= 32 MiB (Add) / 32 KiB (Get) do) or through pinned staging
    opts.update(PAGEABLE_DMA=1 if pageable_path == "dma" else 0, DMA_MIN_BYTES=0, DMA_MIN_BYTES_GET=0)
    rng = np.random.default_rng(71)
    kb, size = 10, 400_000
    batches = []
    for j in range(6):
        if j % 3 == 0:
            f = int(rng.integers(kb, kb + size - 50_000))
            k = np.arange(f, f + 50_000, dtype=np.uint32)                       # dense window
        elif j % 3 == 1:
            k = np.sort(rng.integers(kb, kb + size, size=30_000)).astype(np.uint32)  # sorted
        else:
            k = rng.integers(0, kb + size + 1000, size=30_000).astype(np.uint32)    # unsorted, overflow
        v = rng.integers(-500, 500, size=k.size).astype(np.float64)
        batches.append((k, v))
    q = np.arange(0, kb + size + 1000, dtype=np.uint32)
    outs = {}
    for kind in ("pageable", "pinned"):
        with ps.Shard(kb, kb + size, np.float64, mode=mode, overflow_slots=1 << 14, options=opts) as sh:
            bb = batches if kind == "pageable" else [(_pinned(k), _pinned(v)) for k, v in batches]
            sh.add_grouped(bb[:3])
            for k, v in bb[3:]:
                sh.add(k, v)
            qq = q if kind == "pageable" else _pinned(q)
            o = np.zeros(q.size, np.float64) if kind == "pageable" else _pinned(np.zeros(q.size, np.float64))
            sh.get_grouped([(qq, o)])
            outs[kind] = o.copy()
            outs[kind + "_single"] = sh.get(qq)
    assert_bits_equal(outs["pinned"], outs["pageable"], "pinned vs pageable")
    assert_bits_equal(outs["pinned_single"], outs["pageable"], "pinned single get")
    if mode == "assign":
        ref = oracle_mod.MapStorageRef(np.float64)
        for k, v in batches:
            ref.add(k, v)
        assert_bits_equal(outs["pinned"], ref.get(q), "pinned vs oracle")


# ---------------------------------------------------------------- K8 inline
# Small host messages (<= 256 keys per Add, <= 512 per Get) travel inside the
# kernel arguments.  They are the reference's live traffic shape (one LR
# sample's features per message, app/logistic_regression.cpp:411,490).

def _small_messages(rng, kb, ke, count, max_n=256):
    """Host messages of 0..max_n keys: duplicates, out-of-range keys on both
    sides, the overflow sentinel 0xFFFFFFFF."""
    out = []
    for i in range(count):
        n = int(rng.integers(0, max_n + 1)) if i % 5 else max_n
        k = rng.integers(kb - 50, ke + 50, size=n).astype(np.uint32)
        if n > 4 and i % 3 == 0:
            k[: n // 4] = k[0]                   # a hot key, repeated
        if n > 2 and i % 7 == 0:
            k[-1] = 0xFFFFFFFF
            k[-2] = int(rng.integers(0, 2**32))
        out.append(k)
    return out


@pytest.mark.parametrize("dt", [np.int32, np.float32, np.float64])
def test_inline_small_messages_assign(cuda, oracle_mod, dt):
    """K8 assign: last write wins within and across messages, missing keys 0,
    overflow keys kept; the same message stream through the staged path
    (PSKV_INLINE=0) gives the same bits."""
    import parameter_server_amd as ps
    from parameter_server_amd import _lib

    rng = np.random.default_rng(808)
    kb, ke = 1000, 1000 + 4096
    msgs = _small_messages(rng, kb, ke, 120)
    vals = [(rng.standard_normal(k.size) * 100).astype(dt) for k in msgs]
    ref = oracle_mod.MapStorageRef(dt)
    staged = ps.Shard(kb, ke, dt, overflow_slots=64, options={"INLINE": 0})
    staged.set_timing(True)
    try:
        with ps.Shard(kb, ke, dt, overflow_slots=64) as sh:
            sh.set_timing(True)
            replies = []
            for i, (k, v) in enumerate(zip(msgs, vals)):
                sh.add(k, v)
                staged.add(k, v)
                ref.add(k, v)
                if i % 10 == 9:                       # interleaved small Gets
                    q = np.concatenate([k[:40], rng.integers(kb - 60, ke + 60, size=40)]).astype(np.uint32)
                    replies.append((sh.get(q), staged.get(q), ref.get(q)))
            q = np.concatenate([np.arange(kb - 60, ke + 60), [0xFFFFFFFF]]).astype(np.uint32)
            big = sh.get(q)                             # > 512 keys: staged Get
            assert sh.kernel_time(_lib.PSKV_K_INLINE_ADD)["launches"] == sum(1 for k in msgs if k.size)
            assert sh.kernel_time(_lib.PSKV_K_INLINE_GET)["launches"] == len(replies)
            sh.sync()
        assert staged.kernel_time(_lib.PSKV_K_INLINE_ADD)["launches"] == 0
        big_staged = staged.get(q)
    finally:
        staged.close()
    for a, b, w in replies:
        assert_bits_equal(a, w, "inline get")
        assert_bits_equal(b, w, "staged get")
    assert_bits_equal(big, ref.get(q), "full read after inline adds")
    assert_bits_equal(big_staged, ref.get(q), "full read after staged adds")


@pytest.mark.parametrize("max_n,chunks", [(256, "1"), (2048, "8")])
@pytest.mark.parametrize("dt", [np.int32, np.float32, np.float64])
def test_inline_accumulate_sequential_bits(cuda, dt, max_n, chunks):
    """K8 accumulate: the first occurrence of a key adds every occurrence in
    index order, so the result equals sequential accumulation in the value
    dtype BIT FOR BIT (np.add.at), overflow keys included."""
    import parameter_server_amd as ps

    rng = np.random.default_rng(909)
    kb, ke = 0, 2048
    msgs = _small_messages(rng, kb, ke, 80, max_n=max_n)
    want = np.zeros(ke - kb, dt)
    want_ovf = {}
    # INLINE_ADD_CHUNKS 8: messages of up to 8 launches
    with ps.Shard(kb, ke, dt, mode="accumulate", overflow_slots=64, options={"INLINE_ADD_CHUNKS": int(chunks)}) as sh:
        for k in msgs:
            v = (rng.integers(-2**31, 2**31 - 1, size=k.size, dtype=np.int64).astype(np.int32)
                 if dt is np.int32 else rng.standard_normal(k.size).astype(dt))
            sh.add(k, v)
            inr = k < ke
            np.add.at(want, k[inr].astype(np.int64) - kb, v[inr])
            for key, val in zip(k[~inr], v[~inr]):
                with np.errstate(over="ignore"):
                    want_ovf[int(key)] = dt(want_ovf.get(int(key), dt(0)) + val)
        got = sh.get(np.arange(kb, ke, dtype=np.uint32))
        ok = np.array(sorted(want_ovf), np.uint32)
        got_ovf = sh.get(ok)
    assert_bits_equal(got, want, "inline accumulate (dense)")
    assert_bits_equal(got_ovf, np.array([want_ovf[int(x)] for x in ok], dt), "inline accumulate (overflow)")


@pytest.mark.parametrize("n", [255, 256, 257, 511, 512, 513, 1024, 1025, 2048, 2049])
def test_inline_size_boundaries(cuda, oracle_mod, n):
    """Messages at and beyond the inline limits (an Add of at most 256 keys in
    one launch, a Get in launches of 512 keys, at most 2 of them, so 1024
    keys; grouped calls count their batches together; beyond them the pinned
    staging copy) agree with the oracle."""
    import parameter_server_amd as ps
    from parameter_server_amd import _lib

    rng = np.random.default_rng(n)
    ref = oracle_mod.MapStorageRef(np.float64)
    with ps.Shard(0, 3000, np.float64) as sh:
        sh.set_timing(True)
        k = rng.integers(0, 3100, size=n).astype(np.uint32)
        v = rng.standard_normal(n)
        sh.add(k, v)
        ref.add(k, v)
        # grouped: three batches, n keys in all
        parts = np.split(np.arange(n), [n // 3, 2 * n // 3])
        k2 = rng.integers(0, 3100, size=n).astype(np.uint32)
        v2 = rng.standard_normal(n)
        sh.add_grouped([(k2[p], v2[p]) for p in parts])
        for p in parts:
            ref.add(k2[p], v2[p])
        outs = [np.empty(p.size) for p in parts]
        sh.get_grouped([(k2[p], o) for p, o in zip(parts, outs)])
        got = sh.get(k)
        adds = sh.kernel_time(_lib.PSKV_K_INLINE_ADD)["launches"]
        gets = sh.kernel_time(_lib.PSKV_K_INLINE_GET)["launches"]
    assert adds == (2 if n <= 256 else 0)
    assert gets == (2 * -(-n // 512) if n <= 1024 else 0)
    assert_bits_equal(got, ref.get(k), "single")
    for p, o in zip(parts, outs):
        assert_bits_equal(o, ref.get(k2[p]), "grouped")


@pytest.mark.parametrize("spin", ["1", "0"])
def test_inline_get_reply_paths(cuda, oracle_mod, spin):
    """The inline Get's two completion forms: the polled sequence word the
    kernel publishes after its reply (default) and a plain stream wait
    (PSKV_ISPIN=0); with timing on, the polled form is bypassed too."""
    import parameter_server_amd as ps

    rng = np.random.default_rng(11)
    ref = oracle_mod.MapStorageRef(np.float32)
    with ps.Shard(0, 1 << 16, np.float32, options={"ISPIN": int(spin)}) as sh:
        for i in range(300):
            k = rng.integers(0, 1 << 17, size=int(rng.integers(1, 300))).astype(np.uint32)
            v = rng.standard_normal(k.size).astype(np.float32)
            sh.add(k, v)
            ref.add(k, v)
            if i == 150:
                sh.set_timing(True)
            q = rng.integers(0, 1 << 17, size=int(rng.integers(1, 513))).astype(np.uint32)
            assert_bits_equal(sh.get(q), ref.get(q), f"get {i}")


def test_batch_beyond_2_to_32_elements(cuda):
    """Maximum sizes: ONE device batch of 2^32 + 2^20 elements (keys i mod 2^32
    over a shard of the whole uint32 key space, int32 values), so the batch is
    cut into pieces below the 32-bit per-launch counts and the first 2^20 keys
    are written twice — the later occurrence must win.  Add without a hint (K5
    over ~525 K super-chunks), then a Get of the same 2^32 + 2^20 keys.  (The
    tensors are filled and checked in pieces of 2^28: torch's own kernels are
    not used on more than 2^31 elements at once.)"""
    import torch

    import parameter_server_amd as ps

    n, P = (1 << 32) + (1 << 20), 1 << 28
    keys = torch.empty(n, dtype=torch.int32, device=cuda)
    vals = torch.empty(n, dtype=torch.int32, device=cuda)
    for off in range(0, n, P):
        m = min(P, n - off)
        k = torch.arange(off, off + m, dtype=torch.int64, device=cuda) % (1 << 32)
        keys[off:off + m] = torch.where(k >= 1 << 31, k - (1 << 32), k).to(torch.int32)  # uint32 bits
        vals[off:off + m] = 1 if off < 1 << 32 else 2
    assert int(keys[(1 << 32) + 5]) == 5 and int(keys[(1 << 31) + 1]) == -(1 << 31) + 1
    with ps.Shard(0, 1 << 32, np.int32) as sh:
        sh.add(keys, vals)
        del vals
        out = sh.get(keys)
        torch.cuda.synchronize()
        sh.sync()
    del keys
    # keys below 2^20 were pushed twice (value 1, then 2): they read 2 in both places
    for off in range(0, n, P):
        m = min(P, n - off)
        want = torch.ones(m, dtype=torch.int32, device=cuda)
        lo = max(0, min(m, (1 << 20) - off))
        want[:lo] = 2                         # the first 2^20 positions
        if off >= 1 << 32:
            want[:] = 2                       # the repeated tail
        assert torch.equal(out[off:off + m], want), off


@pytest.mark.parametrize("n", [1025, 1500, 4096, 8193, 70_000, 120_000])
def test_zero_copy_get_sizes(cuda, oracle_mod, n):
    """Medium pageable host Gets (past the inline size, <= 1 MiB of keys and
    values) run K1 over pinned staging: the keys read and the values written
    across PCIe by the kernel.  Partial chunks, unaligned sizes, missing and
    out-of-range keys, grouped and single; against the oracle and against the
    DMA path (PSKV_ZC_MAX_BYTES=0)."""
    import parameter_server_amd as ps

    rng = np.random.default_rng(n)
    kb, ke = 5000, 5000 + 200_000
    k = rng.integers(0, ke + 3000, size=300_000).astype(np.uint32)
    v = rng.standard_normal(k.size)
    ref = oracle_mod.MapStorageRef(np.float64)
    ref.add(k, v)
    q = rng.integers(0, ke + 3000, size=n).astype(np.uint32)
    q[:3] = [0xFFFFFFFF, ke + 2999, kb]
    res = {}
    for zc in ("default", "0"):
        with ps.Shard(kb, ke, np.float64, overflow_slots=1 << 16,
                      options={"ZC_MAX_BYTES": 0} if zc == "0" else None) as sh:
            sh.add(k, v)
            parts = np.array_split(q, 3)
            outs = [np.empty(p.size) for p in parts]
            sh.get_grouped(list(zip(parts, outs)))
            res[zc] = (sh.get(q), np.concatenate(outs))
    want = ref.get(q)
    for zc, (single, grouped) in res.items():
        assert_bits_equal(single, want, f"single {zc}")
        assert_bits_equal(grouped, want, f"grouped {zc}")


def test_c_abi_error_paths_leave_the_shard_usable(cuda, oracle_mod):
    """Every argument error of the C ABI returns PSKV_EINVAL with a message and
    changes nothing (the reference aborts on these through CHECK,
    abstract_storage.hpp:15,20 / map_storage.hpp:20; HipStorage keeps that by
    aborting on a non-zero status): null pointers with n > 0, null batch arrays,
    unknown or contradictory flags, bad timing ids, bad create arguments.  The
    shard then still answers exactly like the oracle."""
    import ctypes

    import parameter_server_amd as ps
    from parameter_server_amd import _lib

    L = _lib.lib
    rng = np.random.default_rng(5)
    kb, ke = 100, 100 + 10_000
    ref = oracle_mod.MapStorageRef(np.float32)
    k = rng.integers(0, 20_000, size=3000).astype(np.uint32)
    v = rng.standard_normal(3000).astype(np.float32)
    out = np.zeros(3000, np.float32)
    with ps.Shard(kb, ke, np.float32) as sh:
        sh.add(k, v)
        ref.add(k, v)
        h = sh.handle
        kp, vp, op = k.ctypes.data, v.ctypes.data, out.ctypes.data
        bad = [
            ("pskv_add: null keys", lambda: L.pskv_add(h, None, vp, 10, _lib.PSKV_HOST)),
            ("pskv_add: null keys", lambda: L.pskv_add(h, kp, None, 10, _lib.PSKV_HOST)),
            ("pskv_get: null keys", lambda: L.pskv_get(h, None, 10, op, _lib.PSKV_HOST)),
            ("pskv_get: null keys", lambda: L.pskv_get(h, kp, 10, None, _lib.PSKV_HOST)),
            ("unknown flags", lambda: L.pskv_add(h, kp, vp, 10, 0x8)),
            ("unknown flags", lambda: L.pskv_add(h, kp, vp, 10, _lib.PSKV_DEVICE | _lib.PSKV_HOST_FRAME)),
            ("unknown flags", lambda: L.pskv_get(h, kp, 10, op, 0x40)),
            ("null batches", lambda: L.pskv_add_grouped(h, None, 3, _lib.PSKV_HOST)),
            ("null batches", lambda: L.pskv_get_grouped(h, None, 3, _lib.PSKV_HOST)),
            ("bad argument", lambda: L.pskv_kernel_time(h, 999, None, None, None)),
            ("null argument", lambda: L.pskv_shard_info(h, None)),
        ]
        for msg, call in bad:
            assert call() == _lib.PSKV_EINVAL, msg
            assert msg.encode() in L.pskv_last_error(), (msg, L.pskv_last_error())
        arr = (_lib.PskvBatch * 2)(_lib.PskvBatch(kp, vp, 5), _lib.PskvBatch(None, vp, 5))
        assert L.pskv_add_grouped(h, arr, 2, _lib.PSKV_HOST) == _lib.PSKV_EINVAL
        # nothing above changed the shard; empty calls are legal no-ops
        assert L.pskv_add(h, None, None, 0, _lib.PSKV_HOST) == _lib.PSKV_OK
        assert L.pskv_get(h, None, 0, None, _lib.PSKV_HOST) == _lib.PSKV_OK
        sh.sync()
        q = np.concatenate([k, rng.integers(0, 2**32, size=500).astype(np.uint32)])
        assert_bits_equal(sh.get(q), ref.get(q), "after rejected calls")
    hh = ctypes.c_void_p()
    for args, msg in [((0, 5, 5, _lib.PSKV_F32, 0), b"key_begin"),
                      ((0, 0, 2**32 + 1, _lib.PSKV_F32, 0), b"key_begin"),
                      ((0, 0, 100, 9, 0), b"dtype"),
                      ((0, 0, 100, _lib.PSKV_F32, 5), b"mode"),
                      ((1000, 0, 100, _lib.PSKV_F32, 0), b"device")]:
        assert L.pskv_shard_create(*args, ctypes.byref(hh)) == _lib.PSKV_EINVAL, args
        assert msg in L.pskv_last_error(), (args, L.pskv_last_error())
    ref.close()


def test_shard_options_api(cuda, monkeypatch, capfd):
    """pskv_set_option / pskv_get_option: every option by name, round trip,
    unknown names and out-of-range values rejected with PSKV_EINVAL (the shard
    unchanged), the environment as the creation default -- where an invalid
    value is reported on stderr and ignored, never a failed creation;
    the options removed in round 4 (GET_DEDUP, RB_INSERT, FUSE: measured losers) are
    unknown names now."""
    import parameter_server_amd as ps
    from parameter_server_amd import PskvError, _lib

    names = ["GENERAL", "UNROLL", "GET_UNROLL", "NT", "NTP", "EARLY", "PAGEABLE_DMA", "DMA_MIN_BYTES", "DMA_MIN_BYTES_GET",
             "DMA_MIN_BYTES_PINNED", "ZC_MAX_BYTES", "FRAME_ZC_MAX_BYTES", "INLINE", "INLINE_ADD_CHUNKS",
             "INLINE_GET_CHUNKS", "ISPIN", "SERVE", "SERVE_IDLE_US", "TILE_SHIFT", "TILE_GRID", "RB_WBITS",
             "RB_NBD", "RB_TB", "RB_APPLY_LOG2", "RB_BIN_BLOCK", "SYNC_TIMEOUT_MS", "FOLD_REPLAY"]
    with ps.Shard(0, 1000, np.float32) as sh:
        for n in names:
            sh.set_option(n, sh.get_option(n))  # every default is a valid value
        sh.set_option("GENERAL", "stamps")
        assert sh.get_option("GENERAL") == 0
        sh.set_option("SERVE", 1)  # INLINE_ADD_CHUNKS was set explicitly above: it stays
        assert sh.get_option("INLINE_ADD_CHUNKS") == 1
        sh.set_option("ZC_MAX_BYTES", 12345)
        assert sh.get_option("ZC_MAX_BYTES") == 12345
        for n, bad in (("UNROLL", 5), ("GET_UNROLL", 6), ("RB_APPLY_LOG2", 12), ("TILE_SHIFT", 3), ("INLINE", 2),
                        ("RB_BIN_BLOCK", 768), ("FOLD_REPLAY", 2), ("NOPE", 1), ("GET_DEDUP", 1), ("RB_INSERT", 1), ("GET_NTP", 1), ("FUSE", 1)):
            before = sh.get_option(n) if n in names else None
            with pytest.raises(PskvError) as ei:
                sh.set_option(n, bad)
            assert ei.value.code == _lib.PSKV_EINVAL
            if before is not None:
                assert sh.get_option(n) == before
        k = np.arange(100, dtype=np.uint32)
        sh.add(k, k.astype(np.float32))
        assert np.array_equal(sh.get(k), k.astype(np.float32))
    with ps.Shard(0, 1000, np.float32, options={"SERVE": 1}) as sh:
        assert sh.get_option("INLINE_ADD_CHUNKS") == 2  # the server's small-Add default
    # the environment: valid values become creation defaults, invalid ones are
    # reported and ignored (the shard is created with the built-in default)
    monkeypatch.setenv("PSKV_UNROLL", "4")
    monkeypatch.setenv("PSKV_TILE_SHIFT", "5")      # out of range
    monkeypatch.setenv("PSKV_GENERAL", "bogus")     # unknown name
    monkeypatch.setenv("PSKV_RB_BIN_BLOCK", "1024x")  # not a number
    monkeypatch.setenv("PSKV_GET_NTP", "1")         # a retired option
    capfd.readouterr()
    with ps.Shard(0, 1000, np.float32) as sh:
        assert sh.get_option("UNROLL") == 4
        assert sh.get_option("TILE_SHIFT") == 0
        assert sh.get_option("GENERAL") == 1
        assert sh.get_option("RB_BIN_BLOCK") == 1024
        k = np.arange(100, dtype=np.uint32)
        sh.add(k, k.astype(np.float32) + 1)
        assert np.array_equal(sh.get(k), k.astype(np.float32) + 1)
    err = capfd.readouterr().err
    for var in ("PSKV_TILE_SHIFT", "PSKV_GENERAL", "PSKV_RB_BIN_BLOCK", "PSKV_GET_NTP"):
        assert f"ignoring environment {var}=" in err, err
    assert "retired option" in err, err
    assert "PSKV_UNROLL" not in err
