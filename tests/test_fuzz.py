"""Differential fuzzing of the HIP path against the oracle.

Each scenario draws a shard (key range incl. the ends of the uint32 space and a
one-key shard, dtype, mode, a tuning knob that selects another host or kernel
path) and a random sequence of calls — single, grouped (beyond the 64-batch
launch group), host, device (unaligned pointers, right and WRONG sorted hints),
inline-sized and large, uniform / Zipf / sorted / dense-window / out-of-range /
sentinel keys, sorted look-alikes of windows (a repeated key hiding a missing
one), bursts of thousands of NEW out-of-range keys into a 64-slot overflow
table with no sync between calls (round 6: the table grows on the device),
empty batches, clears — and checks every Get against the reference state
right away (and at the end every out-of-range key any call pushed):

  assign      the oracle's MapStorage restatement (server/map_storage.hpp:17-45),
              bit-exact
  accumulate  a float64 running sum per key with the recursive-summation bound
              of DESIGN.md §2; int32 exact (wrap-around)

Seeded: a failure names its scenario and step, and reruns identically.
"""

import os

import numpy as np
import pytest

from test_gpu_parity import assert_bits_equal, tdev

pytestmark = pytest.mark.gpu

# scenarios in the default suite (~30 s on MI355X); FUZZ_SCENARIOS=N runs more
N_SCENARIOS = int(os.environ.get("FUZZ_SCENARIOS", "160"))
SEED0 = int(os.environ.get("FUZZ_SEED0", "0"))  # first scenario seed (longer runs: new seeds)
N_STEPS = 18
N_GROUPS = int(os.environ.get("FUZZ_GROUPS", "4"))  # concurrent groups of 6 shards
# shard options (pskv_set_option) that route calls through other host or
# kernel paths; each scenario takes one
KNOBS = [{}, {}, {}, {"SERVE": 1}, {"GENERAL": "stamps"}, {"INLINE": 0},
         {"UNROLL": 4}, {"PAGEABLE_DMA": 1}, {"ZC_MAX_BYTES": 0},
         {"RB_APPLY_LOG2": 13}, {"RB_BIN_BLOCK": 512}, {"GET_UNROLL": 8}, {"GET_UNROLL": 4}, {"EARLY": 1}, {"EARLY": 0}, {"NTP": 0},
         {"TILE_GRID": 1024}, {"NT": 0}, {"FOLD_REPLAY": 0}]
SIZES = [0, 1, 5, 100, 256, 257, 1024, 2049, 5000, 40_000, 300_000]
U32 = 1 << 32


class AccRef:
    """Accumulate reference over any uint32 key: float64 sums, |v| sums and
    push counts (the tolerance), int64 sums for int32 (wrap at the end)."""

    def __init__(self, dt):
        self.dt = dt
        self.clear()

    def clear(self):
        self.sum, self.abs, self.cnt = {}, {}, {}

    def add(self, keys, vals):
        if keys.size == 0:
            return
        v = vals.astype(np.int64 if self.dt is np.int32 else np.float64)
        u, inv = np.unique(keys, return_inverse=True)
        s = np.zeros(u.size, v.dtype)
        a = np.zeros(u.size, np.float64)
        c = np.zeros(u.size, np.int64)
        np.add.at(s, inv, v)  # any order: the tolerance covers every order
        np.add.at(a, inv, np.abs(v.astype(np.float64)))
        np.add.at(c, inv, 1)
        for k, sk, ak, ck in zip(u.tolist(), s.tolist(), a.tolist(), c.tolist()):
            self.sum[k] = self.sum.get(k, 0) + sk
            self.abs[k] = self.abs.get(k, 0.0) + ak
            self.cnt[k] = self.cnt.get(k, 0) + ck

    def check(self, keys, got, what):
        ks = keys.tolist()
        if self.dt is np.int32:
            want = np.array([((self.sum.get(k, 0) + 2**31) % 2**32) - 2**31 for k in ks], np.int64)
            assert_bits_equal(got, want.astype(np.int32), what)
            return
        u = 2.0**-24 if self.dt is np.float32 else 2.0**-53
        want = np.array([self.sum.get(k, 0.0) for k in ks], np.float64)
        tol = np.array([1.01 * (self.cnt.get(k, 0) + 1) * u * self.abs.get(k, 0.0) for k in ks])
        err = np.abs(np.asarray(got, np.float64) - want)
        bad = np.nonzero(~(err <= tol))[0]
        assert bad.size == 0, f"{what}: {bad.size} keys beyond tolerance, first {[ks[i] for i in bad[:5]]}"


def _keys(rng, kb, ke, n, kind):
    size = ke - kb
    if n == 0:
        return np.empty(0, np.uint32)
    if kind in ("dense", "lookalike") and n <= size:
        first = int(rng.integers(kb, ke - n + 1))
        k = np.arange(first, first + n, dtype=np.uint64).astype(np.uint32)
        if kind == "lookalike" and n >= 3:
            # still sorted, but a key repeats its predecessor and so hides a
            # missing one: the endpoints usually still span n - 1 keys, like a
            # window (the sorted / dense paths must not treat it as one)
            for i in rng.integers(0, n - 1, size=int(rng.integers(1, 4))).tolist():
                k[i + 1] = k[i]
        return k
    if kind == "burst" and size < U32:
        # fresh out-of-range keys: uniform over [0, kb) and [ke, 2^32), half
        # of the bursts sorted (the hinted device path then tags and replays)
        x = rng.integers(0, U32 - size, size=n, dtype=np.int64)
        k = np.where(x < kb, x, x + size)
        if rng.random() < 0.5:
            k = np.sort(k)
        return k.astype(np.uint32)
    if kind == "zipf":
        hot = rng.integers(kb, ke, size=min(size, 64), dtype=np.int64)
        k = hot[(rng.zipf(1.3, size=n) - 1) % hot.size]
    else:
        k = rng.integers(kb, ke, size=n, dtype=np.int64)
    if kind in ("sorted", "dense", "lookalike"):
        k = np.sort(k)
    if kind == "oor":
        # a few keys outside the shard (both sides when they exist), the
        # sentinel 0xFFFFFFFF and 0, repeated
        m = max(1, min(n // 8, 300))
        pool = [U32 - 1, 0]
        if kb > 0:
            pool += [kb - 1] + rng.integers(0, kb, size=8, dtype=np.int64).tolist()
        if ke < U32:
            pool += [ke] + rng.integers(ke, U32, size=8, dtype=np.int64).tolist()
        idx = rng.choice(n, size=m, replace=False)
        k[idx] = rng.choice(np.array(pool, np.int64), size=m)
    return k.astype(np.uint32)


def _vals(rng, dt, n):
    if dt is np.int32:
        return rng.integers(-2**31, 2**31, size=n, dtype=np.int64).astype(np.int32)
    return (rng.standard_normal(n) * 10.0 ** rng.integers(-3, 4)).astype(dt)


def _scenario(seed):
    rng = np.random.default_rng(1_000_003 * seed + 17)
    dt = [np.int32, np.float32, np.float64][seed % 3]
    mode = "accumulate" if seed % 5 in (1, 3) else "assign"
    size = int(rng.choice([1, 17, 4096, 65_536, 250_000]))
    kb = int(rng.choice([0, 1000, 2**31 - 7, U32 - size]))
    knobs = KNOBS[seed % len(KNOBS)]
    return rng, dt, mode, kb, kb + size, knobs


@pytest.mark.parametrize("seed", range(SEED0, SEED0 + N_SCENARIOS))
def test_fuzz_against_oracle(cuda, oracle_mod, seed):
    rng, dt, mode, kb, ke, knobs = _scenario(seed)
    _run(cuda, oracle_mod, seed, rng, dt, mode, kb, ke, knobs)


@pytest.mark.parametrize("group", range(N_GROUPS))
def test_fuzz_concurrent_shards(cuda, oracle_mod, group):
    """Six scenarios at once, each on its own shard of the same GPU from its
    own host thread (pskv.h: distinct handles may be used concurrently — the
    reference runs one storage per ServerThread, simple_id_mapper.cpp:28-31):
    the shared host staging pool, frame pool and device must not mix them up.
    ctypes releases the GIL for every library call, so the calls overlap."""
    import threading

    errs = []

    def worker(seed):
        try:
            rng, dt, mode, kb, ke, knobs = _scenario(seed)  # options are per shard: no races
            _run(cuda, oracle_mod, seed, rng, dt, mode, kb, ke, knobs)
        except BaseException as e:  # noqa: B902 - re-raised in the main thread
            errs.append(e)

    ts = [threading.Thread(target=worker, args=(100_000 + 6 * group + i,)) for i in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in ts), "a worker thread did not finish"
    if errs:
        raise errs[0]


def _run(cuda, oracle_mod, seed, rng, dt, mode, kb, ke, knobs):
    import torch

    import parameter_server_amd as ps

    ref = oracle_mod.MapStorageRef(dt) if mode == "assign" else AccRef(dt)
    keep = []  # device buffers stay alive until the final sync (stream-ordered use)
    kinds = ["uniform", "zipf", "sorted", "dense", "oor", "lookalike", "burst"]
    pushed_out = []  # out-of-range keys of every push (checked at the end)
    where = f"seed {seed} ({np.dtype(dt).name} {mode} [{kb}, {ke}) {knobs})"

    def check(q, got, step):
        what = f"{where} step {step}"
        if mode == "assign":
            assert_bits_equal(got, ref.get(q), what)
        else:
            ref.check(q, got, what)

    slots = int(rng.choice([64, 64, 1 << 14]))  # mostly the smallest table: it must grow on the device
    where = where[:-1] + f", {slots} overflow slots)"

    def pushed(k):
        out = k[(k < kb) | (k.astype(np.uint64) >= ke)]
        if out.size:
            pushed_out.append(out)

    with ps.Shard(kb, ke, dt, mode=mode, overflow_slots=slots, options=knobs) as sh:
        for step in range(N_STEPS):
            op = rng.choice(["add", "add", "add_dev", "add_grouped", "add_grouped_dev", "add_get_dev",
                             "get", "get_dev", "get_grouped", "clear"],
                            p=[.15, .07, .15, .11, .11, .08, .11, .09, .09, .04])
            kind = str(rng.choice(kinds))
            if op == "clear":
                sh.clear()
                pushed_out.clear()
                if mode == "assign":
                    ref.close()
                ref = oracle_mod.MapStorageRef(dt) if mode == "assign" else AccRef(dt)
            elif op in ("add", "add_dev"):
                n = int(rng.choice(SIZES))
                k, v = _keys(rng, kb, ke, n, kind), _vals(rng, dt, n)
                if op == "add":
                    sh.add(k, v)
                else:
                    off = int(rng.choice([0, 0, 1, 3]))
                    hint = bool(rng.random() < 0.6)  # also WRONG hints: repaired
                    dk, dv = tdev(k, cuda, off), tdev(v, cuda, off)
                    keep += [dk, dv]
                    sh.add(dk, dv, sorted_hint=hint)
                    if rng.random() < 0.3:
                        sh.sync()  # (not needed for room: the table grows on the device)
                ref.add(k, v)
                pushed(k)
            elif op in ("add_grouped", "add_grouped_dev"):
                nb = int(rng.choice([1, 2, 7, 64, 65, 70]))
                dense = kind in ("dense", "lookalike")
                batches = []
                for _ in range(nb):
                    n = int(rng.choice([0, 1, 33, 1000, 8192, 20_001] if not dense else [1, 1000, 8192, 30_000]))
                    batches.append((_keys(rng, kb, ke, n, kind if dense else str(rng.choice(kinds))),
                                    None))
                batches = [(k, _vals(rng, dt, k.size)) for k, _ in batches]
                if op == "add_grouped":
                    sh.add_grouped(batches)
                else:
                    dev = [(tdev(k, cuda), tdev(v, cuda)) for k, v in batches]
                    keep += [t for kv in dev for t in kv]
                    sh.add_grouped(dev, sorted_hint=bool(rng.random() < 0.7))
                    if rng.random() < 0.3:
                        sh.sync()
                for k, v in batches:
                    ref.add(k, v)
                    pushed(k)
            elif op == "add_get_dev":
                # pskv_add_get_grouped: the grouped Add then the grouped Get;
                # the pulls see the pushes of the same call
                nb = int(rng.choice([1, 5, 64, 67]))
                dense = kind in ("dense", "lookalike")
                adds = []
                for _ in range(nb):
                    n = int(rng.choice([0, 1, 1000, 8192, 30_000] if dense else [0, 1, 33, 8192, 20_001]))
                    k = _keys(rng, kb, ke, n, kind if dense else str(rng.choice(kinds)))
                    adds.append((k, _vals(rng, dt, k.size)))
                qs = []
                for _ in range(int(rng.choice([1, 3, 64, 66]))):
                    if adds and rng.random() < 0.4:  # a pull of pushed keys (maybe a slice of a window)
                        k = adds[int(rng.integers(0, len(adds)))][0]
                        a = int(rng.integers(0, k.size + 1))
                        qs.append(k[a:a + int(rng.integers(0, 9000))].copy())
                    else:
                        qs.append(_keys(rng, kb, ke, int(rng.choice([0, 1, 300, 5000, 8192])), str(rng.choice(kinds))))
                dev_a = [(tdev(k, cuda), tdev(v, cuda)) for k, v in adds]
                dev_q = [tdev(q, cuda) for q in qs]
                tdt = {np.dtype(np.int32): torch.int32, np.dtype(np.float32): torch.float32,
                       np.dtype(np.float64): torch.float64}[np.dtype(dt)]
                outs = [torch.empty(q.size, dtype=tdt, device=cuda) for q in qs]
                keep += [t for kv in dev_a for t in kv] + dev_q + outs
                sh.add_get_grouped(dev_a, list(zip(dev_q, outs)), sorted_hint=bool(rng.random() < 0.8))
                for k, v in adds:
                    ref.add(k, v)
                    pushed(k)
                for q, o in zip(qs, outs):
                    check(q, o.cpu().numpy(), step)
                if rng.random() < 0.3:
                    sh.sync()
            elif op == "get":
                q = _keys(rng, kb, ke, int(rng.choice(SIZES)), kind)
                check(q, sh.get(q), step)
            elif op == "get_dev":
                q = _keys(rng, kb, ke, int(rng.choice(SIZES)), kind)
                out = sh.get(tdev(q, cuda, int(rng.choice([0, 1]))))
                check(q, out.cpu().numpy(), step)
            else:
                nb = int(rng.choice([1, 3, 64, 66]))
                qs = [_keys(rng, kb, ke, int(rng.choice([0, 1, 300, 5000])), str(rng.choice(kinds)))
                      for _ in range(nb)]
                outs = [np.empty(q.size, dt) for q in qs]
                sh.get_grouped(list(zip(qs, outs)))
                for q, o in zip(qs, outs):
                    check(q, o, step)
        # the whole state at the end: every key of a small shard (or a sample)
        # plus every out-of-range key any call used
        q = np.arange(kb, ke, dtype=np.uint64).astype(np.uint32) if ke - kb <= 65_536 else \
            _keys(rng, kb, ke, 100_000, "uniform")
        if pushed_out:
            o = np.unique(np.concatenate(pushed_out))
            q = np.concatenate([q, o if o.size <= 200_000 else rng.choice(o, 200_000, replace=False)])
        check(q, sh.get(q), "final")
        sh.sync()
        torch.cuda.synchronize()
    if mode == "assign":
        ref.close()
