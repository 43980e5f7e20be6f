"""K10 fused grouped Add + Get (pskv_add_get_grouped; round 4): one launch for
a grouped sorted Add followed by a grouped Get.  Bar: the same bits as the
separate calls (option FUSE = 0) and as the oracle's sequential restatement
(map_storage.hpp:22-23 last write wins, :33-37 never-written keys read 0) for
every shape the fused launch treats differently —
  * pulls disjoint from the pushes (the benchmarked step) and pulls inside the
    push windows at every key phase, including keys several windows cover
    (the Get answers covered keys from the pushed values: the LAST window wins);
  * scattered pulls: out-of-range (overflow) keys, never-written keys, the
    sentinel 0xFFFFFFFF, partial chunks;
  * push groups that are sorted but not windows (tile mode: the in-launch grid
    barrier), wrong sorted hints and window look-alikes (K10r: replay, then
    the Get answered again);
  * more than 64 batches on either side (several launch groups)."""
import numpy as np
import pytest

from test_gpu_parity import assert_bits_equal

pytestmark = pytest.mark.gpu

KB, KE = 1000, 1000 + 3_000_000  # shard [KB, KE)


def _dev(a, cuda):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32 if a.dtype == np.uint32 else a.dtype)).to(cuda)


def _run(cuda, oracle_mod, pre, pushes, pulls, fuse, hint=True):
    """Apply `pre` (setup Adds, separate calls), then one add_get_grouped of
    `pushes` / `pulls` on a fresh float32 shard; return the pulled values and
    the oracle's."""
    import torch

    import parameter_server_amd as ps
    from parameter_server_amd import _lib

    ref = oracle_mod.MapStorageRef(np.float32)
    with ps.Shard(KB, KE, np.float32, overflow_slots=1 << 16, options={"FUSE": fuse}) as sh:
        for k, v in pre:
            sh.add(k, v)
            ref.add(k, v)
        adds = [(_dev(k, cuda), _dev(v, cuda)) for k, v in pushes]
        outs = [torch.full((q.size,), -7.0, dtype=torch.float32, device=cuda) for q in pulls]
        gets = [(_dev(q, cuda), o) for q, o in zip(pulls, outs)]
        sh.reset_timing()
        sh.set_timing(True, kernels=[_lib.PSKV_K_ADD_GET])
        sh.add_get_grouped(adds, gets, sorted_hint=hint)
        torch.cuda.synchronize()
        fused_launches = sh.kernel_time(_lib.PSKV_K_ADD_GET)["launches"]
        sh.set_timing(False)
        got = [o.cpu().numpy() for o in outs]
        # the shard after the call, too
        probe = np.unique(np.concatenate([k for k, _ in pushes] + list(pulls) +
                                         [np.arange(KB, KB + 5000, dtype=np.uint32)]))
        after = sh.get(probe)
        sh.sync()
    for k, v in pushes:
        ref.add(k, v)
    want = [ref.get(q) for q in pulls]
    return got, want, after, ref.get(probe), fused_launches


def _windows(rng, n, length, phase_max=4):
    bases = rng.integers(KB, KE - length - 4, size=n)
    bases = bases - bases % 4 + rng.integers(0, phase_max, size=n)
    return [np.arange(b, b + length, dtype=np.uint32) for b in bases]


def _vals(rng, n):
    return (rng.standard_normal(n) * 10).astype(np.float32)


def _check(cuda, oracle_mod, pre, pushes, pulls, expect_fused=True, hint=True):
    res = {}
    for fuse in (1, 0):
        got, want, after, after_ref, launches = _run(cuda, oracle_mod, pre, pushes, pulls, fuse, hint)
        for j, (g, w) in enumerate(zip(got, want)):
            assert_bits_equal(g, w, f"FUSE={fuse}: pull batch {j}")
        assert_bits_equal(after, after_ref, f"FUSE={fuse}: shard after the call")
        res[fuse] = (got, launches)
    assert res[0][1] == 0
    if expect_fused:
        assert res[1][1] >= 1, "the fused launch did not run"
    for a, b in zip(res[0][0], res[1][0]):
        assert_bits_equal(a, b, "FUSE 1 vs 0")


def test_fused_disjoint_pulls(cuda, oracle_mod):
    """The benchmarked shape: window pushes, pulls of windows no push touches."""
    rng = np.random.default_rng(1)
    pre = [(np.arange(KB, KE, dtype=np.uint32), _vals(rng, KE - KB))]
    pushes = [(k, _vals(rng, k.size)) for k in _windows(rng, 12, 65_536, phase_max=1)]
    pushed = np.unique(np.concatenate([k for k, _ in pushes]))
    pulls = []
    while len(pulls) < 10:
        b = int(rng.integers(KB, KE - 40_000)) & ~3
        q = np.arange(b, b + 40_000, dtype=np.uint32)
        if not np.isin(q, pushed).any():
            pulls.append(q)
    _check(cuda, oracle_mod, pre, pushes, pulls)


@pytest.mark.parametrize("phase", [0, 1, 3])
def test_fused_pulls_inside_push_windows(cuda, oracle_mod, phase):
    """Pulls that read keys the same call pushes (at every window phase), keys
    several overlapping windows cover (the last one wins), and the windows'
    edges, partial chunks included."""
    rng = np.random.default_rng(10 + phase)
    pre = [(np.arange(KB, KB + 400_000, dtype=np.uint32), _vals(rng, 400_000))]
    w0 = np.arange(KB + 100 + phase, KB + 100 + phase + 50_000, dtype=np.uint32)
    w1 = np.arange(KB + 20_000 + phase, KB + 20_000 + phase + 70_000, dtype=np.uint32)  # overlaps w0
    w2 = np.arange(KB + 40_001, KB + 40_001 + 9_000, dtype=np.uint32)                   # inside both
    w3 = np.arange(KB + 300_000 + phase, KB + 300_000 + phase + 8192 * 3, dtype=np.uint32)
    pushes = [(w, _vals(rng, w.size)) for w in (w0, w1, w2, w3)]
    pulls = [
        np.arange(KB, KB + 120_000, dtype=np.uint32),                  # spans all three overlapping windows
        np.arange(KB + 40_001 - 3, KB + 40_001 + 9_003, dtype=np.uint32),  # around w2's edges
        w3.copy(),                                                     # exactly a pushed window
        np.arange(KB + 299_990 + phase, KB + 300_010 + phase, dtype=np.uint32),  # a window's start, tiny
        np.sort(rng.integers(KB, KB + 120_000, size=30_000)).astype(np.uint32),   # sorted scattered
    ]
    _check(cuda, oracle_mod, pre, pushes, pulls)


def test_fused_scattered_pulls_overflow_sentinel(cuda, oracle_mod):
    """Scattered pull keys: overflow keys (written before), never-written keys
    (0), the sentinel, keys in the pushed windows, partial chunks."""
    rng = np.random.default_rng(5)
    ovk = np.concatenate([rng.integers(0, KB, size=300), rng.integers(KE, 1 << 32, size=300),
                          [0xFFFFFFFF]]).astype(np.uint32)
    pre = [(ovk, _vals(rng, ovk.size)), (np.arange(KB, KB + 200_000, dtype=np.uint32), _vals(rng, 200_000))]
    pushes = [(k, _vals(rng, k.size)) for k in _windows(rng, 6, 30_000)]
    q = np.concatenate([rng.integers(KB, KE, size=50_000), ovk, np.concatenate([k for k, _ in pushes])[::7],
                        rng.integers(KE, 1 << 32, size=100)]).astype(np.uint32)
    rng.shuffle(q)
    pulls = [q[:8192 * 3], q[8192 * 3:8192 * 3 + 777], q[8192 * 3 + 777:]]
    _check(cuda, oracle_mod, pre, pushes, pulls)


def test_fused_tile_mode_grid_barrier(cuda, oracle_mod):
    """A push group of sorted batches that are not windows (duplicates, gaps):
    the fused launch runs the Add's tile mode, then its grid barrier, then the
    Get — which must see every tile's writes."""
    rng = np.random.default_rng(7)
    pre = [(np.arange(KB, KE, dtype=np.uint32), _vals(rng, KE - KB))]
    pushes = []
    for n in (200_000, 150_000, 5, 90_000):
        k = np.sort(rng.integers(KB, KE, size=n)).astype(np.uint32)
        pushes.append((k, _vals(rng, n)))
    keys = np.concatenate([k for k, _ in pushes])
    pulls = [np.sort(keys[::3]), keys[::5].copy(), np.arange(KB, KB + 100_000, dtype=np.uint32)]
    _check(cuda, oracle_mod, pre, pushes, pulls)


def test_fused_wrong_hint_and_lookalike_repaired(cuda, oracle_mod):
    """A wrong sorted hint (an unsorted batch) and a window look-alike (spans
    n - 1 keys but repeats one): the fused launch tags the group, K10r replays
    it and answers the Get again — the pulls of the pushed keys see the
    sequential last-write-wins values."""
    rng = np.random.default_rng(9)
    pre = [(np.arange(KB, KB + 500_000, dtype=np.uint32), _vals(rng, 500_000))]
    w = np.arange(KB + 1000, KB + 1000 + 100_000, dtype=np.uint32)
    look = np.arange(KB + 200_001, KB + 200_001 + 50_000, dtype=np.uint32)
    look[20_000] = look[19_999]  # repeats a key, misses another: still spans n - 1
    bad = rng.permutation(np.arange(KB + 300_000, KB + 340_000, dtype=np.uint32))
    pushes = [(w, _vals(rng, w.size)), (look, _vals(rng, look.size)), (bad, _vals(rng, bad.size)),
              (w[5000:9000].copy(), _vals(rng, 4000))]
    pulls = [np.arange(KB, KB + 400_000, dtype=np.uint32), look.copy(), bad[::3].copy()]
    _check(cuda, oracle_mod, pre, pushes, pulls)


def test_fused_many_batches_and_empty(cuda, oracle_mod):
    """70 push windows and 70 pull batches (two launch groups each side), some
    empty: the last Add group fuses with the first Get group, the rest run
    apart, in order."""
    rng = np.random.default_rng(13)
    pushes = [(k, _vals(rng, k.size)) for k in _windows(rng, 70, 9_000)]
    pushes[3] = (np.zeros(0, np.uint32), np.zeros(0, np.float32))
    pulls = [np.arange(b, b + 5_000, dtype=np.uint32) for b in rng.integers(KB, KE - 5_000, size=70)]
    pulls[10] = np.zeros(0, np.uint32)
    pulls[69] = np.concatenate([k for k, _ in pushes[60:]])  # the fused Add group's own keys
    _check(cuda, oracle_mod, [], pushes, pulls)


def test_fused_falls_back_where_it_cannot_fuse(cuda, oracle_mod):
    """No hint, or an unaligned batch: the separate paths, the same results."""
    rng = np.random.default_rng(21)
    pushes = [(k, _vals(rng, k.size)) for k in _windows(rng, 4, 20_000)]
    pulls = [np.arange(KB, KB + 60_000, dtype=np.uint32)]
    got, want, after, after_ref, launches = _run(cuda, oracle_mod, [], pushes, pulls, fuse=1, hint=False)
    assert launches == 0
    assert_bits_equal(got[0], want[0], "unhinted")
    assert_bits_equal(after, after_ref, "unhinted, shard")
