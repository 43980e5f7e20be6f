"""K9 request server (PSKV_SERVE=1): small host messages through a ring in
page-locked memory that one resident workgroup polls, instead of one kernel
launch per message.  Same bar as K8: assign bit-exact against
the oracle, accumulate bit-identical to the sequential loop; plus the
protocol's own edges: regular (large) calls between ring requests (the server
is stopped before them and restarted behind them), a server that leaves on
its idle timer while requests are posted, overflow growth (the server holds
the table by value), several shards on one device, and teardown.
"""
import time

import numpy as np
import pytest

from test_gpu_parity import _small_messages, assert_bits_equal

pytestmark = pytest.mark.gpu


@pytest.fixture
def serve():
    """The shard options that turn the request server on."""
    return {"SERVE": 1}


@pytest.mark.parametrize("dt", [np.int32, np.float32, np.float64])
def test_serve_messages_assign(cuda, oracle_mod, dt, serve):
    """Adds and Gets of 0..256 / up to 1024 keys, duplicates, out-of-range and
    sentinel keys, with a large Add and a large Get (the regular path) every
    25 messages."""
    import parameter_server_amd as ps

    rng = np.random.default_rng(4242)
    kb, ke = 1000, 1000 + 50_000
    msgs = _small_messages(rng, kb, ke, 150)
    ref = oracle_mod.MapStorageRef(dt)
    checks = []
    with ps.Shard(kb, ke, dt, overflow_slots=64, options=serve) as sh:
        for i, k in enumerate(msgs):
            v = (rng.standard_normal(k.size) * 100).astype(dt)
            sh.add(k, v)
            ref.add(k, v)
            if i % 7 == 3:
                q = np.concatenate([k[:300], rng.integers(kb - 60, ke + 60, size=int(rng.integers(1, 700)))])
                q = q.astype(np.uint32)
                checks.append((sh.get(q), ref.get(q)))
            if i % 25 == 24:  # the regular path between ring requests
                big_k = rng.integers(kb, ke, size=20_000).astype(np.uint32)
                big_v = (rng.standard_normal(big_k.size) * 100).astype(dt)
                sh.add(big_k, big_v)
                ref.add(big_k, big_v)
                q = rng.integers(kb - 60, ke + 60, size=5000).astype(np.uint32)
                checks.append((sh.get(q), ref.get(q)))
        q = np.concatenate([np.arange(kb - 60, ke + 60), [0xFFFFFFFF]]).astype(np.uint32)
        checks.append((sh.get(q), ref.get(q)))
        sh.sync()
    for j, (got, want) in enumerate(checks):
        assert_bits_equal(got, want, f"check {j}")


@pytest.mark.parametrize("dt", [np.int32, np.float32, np.float64])
def test_serve_accumulate_sequential_bits(cuda, dt, serve):
    """Accumulate through the ring: the first occurrence adds every occurrence
    in index order, so the result equals np.add.at in the value dtype."""
    import parameter_server_amd as ps

    rng = np.random.default_rng(99)
    kb, ke = 0, 2048
    msgs = _small_messages(rng, kb, ke, 120)
    want = np.zeros(ke - kb, dt)
    want_ovf = {}
    with ps.Shard(kb, ke, dt, mode="accumulate", overflow_slots=64, options=serve) as sh:
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
    assert_bits_equal(got, want, "served accumulate (dense)")
    assert_bits_equal(got_ovf, np.array([want_ovf[int(x)] for x in ok], dt), "served accumulate (overflow)")


def test_serve_idle_restart_and_ring_wrap(cuda, oracle_mod, serve):
    """A 50 us idle timer: the server leaves between most calls and is
    restarted, including while requests are queued; bursts longer than the
    ring (64 slots) wrap it."""
    import parameter_server_amd as ps

    serve = dict(serve, SERVE_IDLE_US=50)
    rng = np.random.default_rng(5)
    ref = oracle_mod.MapStorageRef(np.float32)
    with ps.Shard(0, 10_000, np.float32, options=serve) as sh:
        for i in range(40):
            for _ in range(int(rng.integers(1, 150))):  # a burst of Adds, up to 2+ ring laps
                k = rng.integers(0, 10_000, size=int(rng.integers(1, 40))).astype(np.uint32)
                v = rng.standard_normal(k.size).astype(np.float32)
                sh.add(k, v)
                ref.add(k, v)
            if i % 3 == 0:
                time.sleep(0.001)  # idle: the server leaves
            q = rng.integers(0, 10_000, size=300).astype(np.uint32)
            assert_bits_equal(sh.get(q), ref.get(q), f"round {i}")


def test_serve_overflow_growth(cuda, oracle_mod, serve):
    """Small messages full of out-of-range keys grow the overflow table many
    times: ~40 K new keys from 64 slots, 200 messages.  With the request
    server (K9) one resident launch takes the messages and grows the table
    itself, request after request through the same mailbox (round 6); with
    K8 every launch reserves for its own message."""
    import parameter_server_amd as ps

    rng = np.random.default_rng(17)
    ref = oracle_mod.MapStorageRef(np.float64)
    with ps.Shard(0, 1000, np.float64, overflow_slots=64, options=serve) as sh:
        for _ in range(200):
            k = rng.integers(0, 200_000, size=200).astype(np.uint32)
            v = rng.standard_normal(k.size)
            sh.add(k, v)
            ref.add(k, v)
        q = rng.integers(0, 200_000, size=1000).astype(np.uint32)
        got = sh.get(q)
        sh.sync()
        assert sh.info()["overflow_capacity"] >= 2 * sh.info()["overflow_count"]
    assert_bits_equal(got, ref.get(q), "overflow")


@pytest.mark.parametrize("nshards", [2, 4])
def test_serve_several_shards_one_device(cuda, oracle_mod, serve, nshards):
    """Shards on one GPU, messages interleaved across them, and device-path
    calls on some in between.  A resident server holds the hardware queue its
    stream maps to, so the server engages only while a device has at most
    GPU_MAX_HW_QUEUES / 2 shards (2 by default); with 4 the shards fall back
    to the K8 launches, with the same results."""
    import torch

    import parameter_server_amd as ps

    rng = np.random.default_rng(8)
    shards = [ps.Shard(s * 1000, (s + 1) * 1000, np.float64, options=serve) for s in range(nshards)]
    refs = [oracle_mod.MapStorageRef(np.float64) for _ in shards]
    try:
        for i in range(400):
            s = int(rng.integers(0, nshards))
            k = rng.integers(s * 1000, s * 1000 + 1100, size=int(rng.integers(1, 64))).astype(np.uint32)
            v = rng.standard_normal(k.size)
            shards[s].add(k, v)
            refs[s].add(k, v)
            if i % 50 == 49:
                dk = torch.arange(s * 1000, s * 1000 + 1000, dtype=torch.int32, device=cuda)
                dv = torch.full((1000,), float(i), dtype=torch.float64, device=cuda)
                shards[s].add(dk, dv, sorted_hint=True)
                refs[s].add(dk.cpu().numpy().view(np.uint32), dv.cpu().numpy())
        for s, (sh, ref) in enumerate(zip(shards, refs)):
            q = np.arange(s * 1000, s * 1000 + 1100, dtype=np.uint32)
            assert_bits_equal(sh.get(q), ref.get(q), f"shard {s}")
    finally:
        for sh in shards:
            sh.close()


def test_serve_start_waits_for_slow_stream_work(cuda, oracle_mod, serve):
    """A server launch queued behind > 2 s of earlier work on the shard's stream
    (here a spin kernel on the legacy default stream, which the shard's blocking
    stream orders behind) is not "stuck": srv_wait starts its start-timeout
    clock only once that dependency has completed (a long replay of a
    broken sorted hint followed by a small served Get used to fail with
    PSKV_ESTATE after 2 s)."""
    import torch

    import parameter_server_amd as ps

    rng = np.random.default_rng(31)
    ref = oracle_mod.MapStorageRef(np.float32)
    # calibrate the spin kernel (it counts shader clocks)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(100_000_000)
    e1.record()
    torch.cuda.synchronize()
    cycles_per_ms = 100_000_000 / max(e0.elapsed_time(e1), 1e-3)
    with ps.Shard(0, 10_000, np.float32, options=dict(serve, SERVE_IDLE_US=1000)) as sh:
        k = rng.integers(0, 10_000, size=100).astype(np.uint32)
        v = rng.standard_normal(k.size).astype(np.float32)
        sh.add(k, v)
        ref.add(k, v)
        assert_bits_equal(sh.get(k), ref.get(k), "before")
        time.sleep(0.05)  # the server idles out
        torch.cuda._sleep(int(4000 * cycles_per_ms))  # ~4 s of earlier work
        t0 = time.perf_counter()
        k2 = rng.integers(0, 10_000, size=100).astype(np.uint32)
        v2 = rng.standard_normal(k2.size).astype(np.float32)
        sh.add(k2, v2)  # relaunches the server behind the spin kernel
        ref.add(k2, v2)
        q = rng.integers(0, 10_000, size=300).astype(np.uint32)
        got = sh.get(q)
        waited = time.perf_counter() - t0
    assert_bits_equal(got, ref.get(q), "after the slow dependency")
    assert waited > 2.0, f"the dependency did not delay the served calls ({waited:.2f} s): the test lost its point"


def test_serve_wait_is_bounded(cuda, oracle_mod, serve):
    """The request server's waits are bounded too (SYNC_TIMEOUT_MS):
    a served Get queued behind ~3 s of earlier work on the shard's stream
    fails with PSKV_ESTATE naming the server's dependency once the 500 ms
    bound has passed, where it used to spin for as long as the dependency
    ran; once that work has drained the same shard serves the Get,
    bit-exact."""
    import torch

    import parameter_server_amd as ps
    from parameter_server_amd import PskvError, _lib

    rng = np.random.default_rng(37)
    ref = oracle_mod.MapStorageRef(np.float32)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(50_000_000)
    e1.record()
    torch.cuda.synchronize()
    cycles_per_ms = 50_000_000 / max(e0.elapsed_time(e1), 1e-3)
    with ps.Shard(0, 10_000, np.float32, options=dict(serve, SERVE_IDLE_US=1000, SYNC_TIMEOUT_MS=500)) as sh:
        k = rng.integers(0, 10_000, size=100).astype(np.uint32)
        v = rng.standard_normal(k.size).astype(np.float32)
        sh.add(k, v)
        ref.add(k, v)
        assert_bits_equal(sh.get(k), ref.get(k), "before")
        time.sleep(0.05)  # the server idles out
        torch.cuda._sleep(int(3000 * cycles_per_ms))  # ~3 s of earlier work on the legacy stream
        k2 = rng.integers(0, 10_000, size=100).astype(np.uint32)
        v2 = rng.standard_normal(k2.size).astype(np.float32)
        sh.add(k2, v2)  # relaunches the server behind the spin kernel
        ref.add(k2, v2)
        q = rng.integers(0, 10_000, size=300).astype(np.uint32)
        with pytest.raises(PskvError) as ei:
            sh.get(q)
        assert ei.value.code == _lib.PSKV_ESTATE
        assert "request-server" in str(ei.value) and "not complete after" in str(ei.value), str(ei.value)
        # the earlier work drains (the server then idles out); every later
        # call of the shard succeeds again, nothing was cancelled
        torch.cuda.synchronize()
        sh.set_option("SYNC_TIMEOUT_MS", 0)
        assert_bits_equal(sh.get(q), ref.get(q), "after the earlier work drained")


def test_timed_out_get_holds_staging(cuda, oracle_mod):
    """A staged host Get that gives up on its D2H wait (SYNC_TIMEOUT_MS) leaves
    its H2D, K1 and D2H queued on the pinned staging buffer; the next host Get
    must not write its keys there until that work has drained.
    The second Get is larger, so its keys cover the first one's value region
    in the staging: without the hold the first Get's late D2H lands on them
    before they are DMA'd, and the second Get answers other keys."""
    import torch

    import parameter_server_amd as ps
    from parameter_server_amd import PskvError, _lib

    rng = np.random.default_rng(53)
    ref = oracle_mod.MapStorageRef(np.float32)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(50_000_000)
    e1.record()
    torch.cuda.synchronize()
    cycles_per_ms = 50_000_000 / max(e0.elapsed_time(e1), 1e-3)
    # staged Gets only: no inline (K8), no zero copy, no direct pageable DMA
    opts = dict(INLINE=0, ZC_MAX_BYTES=0, PAGEABLE_DMA=0, SYNC_TIMEOUT_MS=500)
    n = 1_000_000
    with ps.Shard(0, n, np.float32, options=opts) as sh:
        k = np.arange(n, dtype=np.uint32)
        v = rng.standard_normal(n).astype(np.float32)
        sh.add(k, v)
        ref.add(k, v)
        sh.sync()
        q1 = rng.integers(0, n, size=20_000).astype(np.uint32)
        q2 = rng.integers(0, n, size=200_000).astype(np.uint32)
        torch.cuda._sleep(int(2000 * cycles_per_ms))  # ~2 s of earlier work on the legacy stream
        with pytest.raises(PskvError) as ei:
            sh.get(q1)
        assert ei.value.code == _lib.PSKV_ESTATE and "not complete after" in str(ei.value), str(ei.value)
        sh.set_option("SYNC_TIMEOUT_MS", 0)
        got = sh.get(q2)  # waits for the held staging, then stages its own keys
        assert_bits_equal(got, ref.get(q2), "Get after a timed-out Get")
        assert_bits_equal(sh.get(q1), ref.get(q1), "the timed-out Get, again")
