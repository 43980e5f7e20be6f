"""CPU tests: pin the oracle (the CPU restatement) to the reference's own known
answers, and check its restatements against each other.  No GPU."""
import json
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
DT = {"int32": np.int32, "float32": np.float32, "float64": np.float64}


def known():
    with open(os.path.join(GOLDEN, "reference_known_answers.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("kind", ["map", "vector"])
@pytest.mark.parametrize("case", known()["storage_cases"], ids=lambda c: c["name"])
def test_oracle_reference_known_answers(oracle_mod, kind, case):
    dt = DT[case["dtype"]]
    ref = (oracle_mod.MapStorageRef if kind == "map" else oracle_mod.VectorStorageRef)(dt)
    for op in case["ops"]:
        if op[0] == "add":
            ref.add(np.array(op[1], np.uint32), np.array(op[2], dt))
        else:
            got = ref.get(np.array(op[1], np.uint32))
            want = np.array(op[2], dt)  # SArray<float>({0.1,...}) rounds the double literal to float
            assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), (case["cite"], got, want)


@pytest.mark.parametrize("case", known()["slice_cases"], ids=lambda c: c["cite"][:40])
def test_range_slice_ref_known_answers(oracle_mod, case):
    got = oracle_mod.range_slice_ref([tuple(r) for r in case["ranges"]], case["keys"])
    assert [[r, ks] for r, ks in got] == case["expect"], case["cite"]
    # the C restatement assigns the same range to every key
    ra = oracle_mod.range_assign([tuple(r) for r in case["ranges"]], case["keys"])
    flat = [r for r, ks in case["expect"] for _ in ks]
    assert list(ra) == flat


def test_range_assign_matches_python(oracle_mod):
    rng = np.random.default_rng(3)
    for _ in range(50):
        nr = int(rng.integers(1, 6))
        cuts = np.sort(rng.choice(np.arange(1, 1000), size=nr, replace=False))
        ranges = [(int(a), int(b)) for a, b in zip(np.r_[int(rng.integers(0, 50)), cuts[:-1]], cuts)]
        keys = rng.integers(0, 1100, size=int(rng.integers(0, 200)))
        if rng.random() < 0.5:
            keys = np.sort(keys)
        py = oracle_mod.range_slice_ref(ranges, keys)
        flat = [r for r, ks in py for _ in ks]
        assert list(oracle_mod.range_assign(ranges, keys)) == flat


@pytest.mark.parametrize("dt", [np.int32, np.float32, np.float64])
def test_vector_and_map_storage_are_equivalent(oracle_mod, dt):
    """both reference storages are last-write-wins with default 0."""
    rng = np.random.default_rng(11)
    m, v = oracle_mod.MapStorageRef(dt), oracle_mod.VectorStorageRef(dt)
    for _ in range(6):
        n = int(rng.integers(0, 700))
        k = rng.integers(0, 900, size=n).astype(np.uint32)
        x = (rng.standard_normal(n) * 1000).astype(dt)
        m.add(k, x)
        v.add(k, x)
        q = rng.integers(0, 1000, size=500).astype(np.uint32)
        assert np.array_equal(m.get(q).view(np.uint8), v.get(q).view(np.uint8))
    assert v.size() >= m.size()


def test_dense_last_wins_matches_map(oracle_mod):
    rng = np.random.default_rng(5)
    m = oracle_mod.MapStorageRef(np.float32)
    dense = np.zeros(4000, np.float32)
    for _ in range(10):
        n = int(rng.integers(1, 3000))
        k = (rng.zipf(1.5, size=n) % 4000).astype(np.uint32)
        x = rng.standard_normal(n).astype(np.float32)
        m.add(k, x)
        oracle_mod.dense_last_wins(dense, 0, k, x)
    q = np.arange(4000, dtype=np.uint32)
    assert np.array_equal(m.get(q).view(np.uint32), dense.view(np.uint32))


def test_golden_vectors_reproduce_with_both_restatements(oracle_mod):
    z = np.load(os.path.join(GOLDEN, "assign_vectors.npz"))
    with open(os.path.join(GOLDEN, "assign_vectors.json")) as f:
        meta = json.load(f)
    for c in meta["cases"]:
        dt = DT[c["dtype"]]
        for cls in (oracle_mod.MapStorageRef, oracle_mod.VectorStorageRef):
            ref = cls(dt)
            for j in range(c["n_adds"]):
                ref.add(z[f"{c['name']}/add{j}/keys"], z[f"{c['name']}/add{j}/vals"])
            got = ref.get(z[f"{c['name']}/get/keys"])
            assert np.array_equal(got.view(np.uint8), z[f"{c['name']}/get/expect"].view(np.uint8)), c


def test_oracle_rejects_mismatched_sizes(oracle_mod):
    ref = oracle_mod.MapStorageRef(np.float32)
    with pytest.raises(ValueError):
        ref.add(np.arange(3, dtype=np.uint32), np.zeros(2, np.float32))


def test_bench_step_bytes_and_single_gpu_sets():
    """bench.py's algorithmic byte accounting (counting what a step
    must move: Add n*4 keys + u*V last values + u*V parameter writes, Get
    q*(4+2V)) and the N = 1 window sets: 1M-aligned bases inside the 1e8-key
    shard, set 0 on the config's seed 42, the other sets on distinct seeds; the
    pull of each step is every window slot its push left free, each once — zero
    push/pull overlap (the Get must read parameters the step did not
    write) — so a step touches the whole 400 MB shard."""
    import sys

    sys.path.insert(0, ROOT)
    import bench
    from parameter_server_amd import workload

    add, get = bench.step_bytes(64_000_000, 48_000_000, 64_000_000)
    assert add == 64_000_000 * 4 + 2 * 48_000_000 * 4 and get == 64_000_000 * 12
    assert bench.step_bytes(10, 7, 3, vb=8) == (10 * 4 + 2 * 7 * 8, 3 * 20)
    seen = []
    for r in range(4):
        ks, lo, hi, slices, bases = bench.plan_rank(0, 1, 64, 1_000_000, r)
        assert (ks, lo, hi) == (100_000_000, 0, 100_000_000)
        assert all(b % 1_000_000 == 0 and 0 <= b <= 99_000_000 for b in bases)
        assert [(w, f, n) for w, f, n in slices] == [(j, int(b), 1_000_000) for j, b in enumerate(bases)]
        seen.append(tuple(int(b) for b in bases))
        pull, pbases = bench.plan_pull(0, 1, 64, 1_000_000, r, bases)
        pushed = set(int(b) for b in bases)
        assert len(pull) == 100 - len(pushed) and len(set(int(b) for b in pbases)) == len(pull)
        assert not pushed & set(int(b) for b in pbases)
        assert sorted(pushed | set(int(b) for b in pbases)) == list(range(0, 100_000_000, 1_000_000))
        s = {"slices": slices, "pull": pull}
        assert bench.overlap_keys(s) == 0
        # the cold form: the same draw on a 1e9-key shard, as many pulls
        _, _, hi9, sl9, b9 = bench.plan_rank(0, 1, 64, 1_000_000, r, space=1_000_000_000)
        p9, pb9 = bench.plan_pull(0, 1, 64, 1_000_000, r, b9, space=1_000_000_000, n_pull=len(pull))
        assert hi9 == 1_000_000_000 and len(p9) == len(pull)
        assert bench.overlap_keys({"slices": sl9, "pull": p9}) == 0
    assert len(set(seen)) == 4
    assert seen[0] == tuple(int(b) for b in workload.dense_bases(64, 100_000_000, 1_000_000, seed=42))
    # an overlapping pull is detected
    assert bench.overlap_keys({"slices": [(0, 5, 10)], "pull": [(0, 12, 10)]}) == 3


def test_disjoint_and_complement_windows():
    from parameter_server_amd import workload

    push = workload.global_windows(64, 1_000_000_000, 1_000_000, seed=1000)
    pull = workload.disjoint_windows(push, 64, 1_000_000_000, 1_000_000, seed=7)
    assert pull.shape == (64,) and int(pull.min()) >= 0 and int(pull.max()) <= 999_000_000
    iv = sorted([(int(b), int(b) + 1_000_000) for b in pull])
    assert all(iv[i][1] <= iv[i + 1][0] for i in range(len(iv) - 1))  # pulls pairwise disjoint
    assert all(e <= int(p) or int(p) + 1_000_000 <= int(b)
               for p in pull for b, e in ((int(x), int(x) + 1_000_000) for x in push))
    assert list(workload.disjoint_windows(push, 64, 1_000_000_000, 1_000_000, seed=7)) == list(pull)
    c = workload.complement_windows([0, 20, 20, 60], 0, 100, 20, seed=3)
    assert sorted(int(x) for x in c) == [40, 80]
    assert len(workload.complement_windows([0], 0, 100, 20, seed=3, n_max=2)) == 2
    c2 = workload.complement_windows([1000, 1040], 1000, 1100, 20, seed=1)
    assert sorted(int(x) for x in c2) == [1020, 1060, 1080]
    # an unaligned push window touches two slots: neither is pulled
    c3 = workload.complement_windows([10, 65], 0, 100, 20, seed=2)
    assert sorted(int(x) for x in c3) == [40]
    # a pull that cannot fit raises instead of drawing for ever
    with pytest.raises(ValueError, match="found no place"):
        workload.disjoint_windows([0, 30, 60], 2, 100, 30, seed=1, max_draws=1000)


def test_interval_union_and_global_windows():
    from parameter_server_amd import workload

    assert workload.interval_union([]) == 0
    assert workload.interval_union([(5, 3), (0, 2), (6, 4), (20, 0)]) == 2 + 5
    assert workload.interval_union([(0, 10), (2, 3)]) == 10
    b = workload.global_windows(64, 1_000_000_000, 1_000_000, seed=1000)
    assert b.shape == (64,) and int(b.min()) >= 0 and int(b.max()) <= 999_000_000
    # producer s draws with seed 1000 + s: the same stream whatever the count
    assert list(workload.global_windows(3, 1_000_000_000, 1_000_000, seed=1000)) == list(b[:3])
    assert any(int(x) % 4 for x in b)  # any alignment


def test_bench_default_window_sets():
    """bench.py's --sets default: 16 window sets at N = 1, 64 at N > 1 (fresh
    cfg-4 draws: the largest rank's share over the timed steps approaches the
    mean), an explicit value wins."""
    import bench

    assert bench.parse([]).sets is None
    assert bench.parse(["--sets", "4"]).sets == 4
    assert bench.default_sets(None, 1) == 16 and bench.default_sets(None, 8) == 64
    assert bench.default_sets(4, 8) == 4 and bench.default_sets(1, 1) == 2
