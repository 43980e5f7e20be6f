"""Page-locked host frames (pskv_host_alloc / PSKV_HOST_FRAME).

The mailbox receives each data frame of a message (comm/mailbox.cpp:246-257)
into a frame from the library's pool; HipStorage hands the frames to the C ABI
under PSKV_HOST_FRAME, which reads and writes them in place and lets an Add
return before its kernels run.  These tests hold the frame paths to the same
bar as every other host path: bit-exact against the oracle (assign) and
bit-identical to the staged path (accumulate: the same kernels see the same
batches), with the frames freed -- and their memory handed out again and
overwritten -- while the Adds that read them may still be queued.
"""
import numpy as np
import pytest

from test_gpu_parity import assert_bits_equal

pytestmark = pytest.mark.gpu


def _in_frames(ps, arrays):
    """Copy each array into its own frame; returns (frames, views)."""
    frames, views = [], []
    for a in arrays:
        f = ps.HostFrame(max(1, a.nbytes))
        v = f.array(a.dtype, a.size)
        v[:] = a
        frames.append(f)
        views.append(v)
    return frames, views


def _scribble(ps, nbytes, count=2):
    """Allocate frames of the same size class and overwrite them: a frame whose
    queued reads had not run would be corrupted if the pool handed it out."""
    fs = [ps.HostFrame(nbytes) for _ in range(count)]
    for f in fs:
        f.array(np.uint8, nbytes)[:] = 0xA5
    return fs


def _messages(rng, kb, ke, n, count):
    out = []
    for j in range(count):
        if j % 3 == 0:
            f = int(rng.integers(kb, max(kb + 1, ke - n)))
            k = np.arange(f, f + n, dtype=np.uint32)                              # dense window
        elif j % 3 == 1:
            k = np.sort(rng.integers(kb, ke, size=n)).astype(np.uint32)          # sorted, duplicates
        else:
            k = rng.integers(max(0, kb - 100), ke + 100, size=n).astype(np.uint32)  # unsorted, overflow
            k[0] = 0xFFFFFFFF
        out.append(k)
    return out


@pytest.mark.parametrize("zc", ["default", "dma"])
@pytest.mark.parametrize("n", [300, 5000, 70_000, 400_000])
@pytest.mark.parametrize("mode,dt", [("assign", np.float64), ("assign", np.int32),
                                     ("accumulate", np.float32), ("accumulate", np.int32)])
def test_frame_add_get_parity(cuda, oracle_mod, mode, dt, n, zc):
    import parameter_server_amd as ps

    # zc "dma": every frame call above the inline size DMAs instead of reading in place
    opts = {"FRAME_ZC_MAX_BYTES": 0} if zc == "dma" else None
    rng = np.random.default_rng(n + 7)
    kb, ke = 1000, 1000 + 600_000
    keys = _messages(rng, kb, ke, n, 6)
    vals = [rng.integers(-1000, 1000, size=k.size).astype(dt) for k in keys]
    q = rng.integers(0, ke + 200, size=n + 17).astype(np.uint32)
    q[:2] = [0xFFFFFFFF, kb]
    res = {}
    for path in ("staged", "frames"):
        with ps.Shard(kb, ke, dt, mode=mode, overflow_slots=1 << 12, options=opts) as sh:
            keep = []
            for j, (k, v) in enumerate(zip(keys, vals)):
                if path == "staged":
                    if j == 4:
                        sh.add_grouped([(k, v), (keys[5], vals[5])])
                    elif j != 5:
                        sh.add(k, v)
                    continue
                if j == 5:
                    continue
                if j == 4:  # a grouped Add of two framed batches
                    fr, (fk, fv, gk, gv) = _in_frames(ps, [k, v, keys[5], vals[5]])
                    sh.add_grouped([(fk, fv), (gk, gv)], frame=True)
                else:
                    fr, (fk, fv) = _in_frames(ps, [k, v])
                    sh.add(fk, fv, frame=True)
                for f in fr:  # freed at once: the pool holds them until the Add has run
                    f.free()
                keep += _scribble(ps, max(1, k.nbytes))
            if path == "staged":
                got = sh.get(q)
                parts = np.array_split(q, 3)
                outs = [np.empty(p.size, dt) for p in parts]
                sh.get_grouped(list(zip(parts, outs)))
                grouped = np.concatenate(outs)
            else:
                fr, (fq,) = _in_frames(ps, [q])
                fo = ps.HostFrame(q.size * np.dtype(dt).itemsize)
                got = sh.get(fq, out=fo.array(dt, q.size), frame=True).copy()
                parts = np.array_split(np.arange(q.size), 3)
                fouts = [ps.HostFrame(p.size * np.dtype(dt).itemsize) for p in parts]
                sh.get_grouped([(fq[p[0]:p[-1] + 1], f.array(dt, p.size)) for p, f in zip(parts, fouts)],
                               frame=True)
                grouped = np.concatenate([f.array(dt, p.size) for p, f in zip(parts, fouts)]).copy()
                for f in fr + fouts + [fo]:
                    f.free()
            for f in keep:
                f.free()
            sh.sync()
            res[path] = (got, grouped)
    assert_bits_equal(res["frames"][0], res["staged"][0], "frame get vs staged")
    assert_bits_equal(res["frames"][1], res["staged"][0], "frame grouped get vs staged")
    assert_bits_equal(res["staged"][1], res["staged"][0], "staged grouped vs single")
    if mode == "assign":
        ref = oracle_mod.MapStorageRef(dt)
        for k, v in zip(keys, vals):
            ref.add(k, v)
        assert_bits_equal(res["frames"][0], ref.get(q), "frames vs oracle")


def test_freed_frame_held_until_its_add_has_run(cuda):
    """A frame freed while an Add that reads it is queued is not handed out
    again until that Add has run; afterwards it is reused."""
    import torch

    import parameter_server_amd as ps

    n = 1 << 22
    with ps.Shard(0, 1 << 26, np.float32) as sh:
        big_k = torch.arange(0, 1 << 26, dtype=torch.int32, device=cuda)
        big_v = torch.ones(1 << 26, dtype=torch.float32, device=cuda)
        spare = [ps.HostFrame(4 * n) for _ in range(2)]  # cached frames of the class
        for f in spare:
            f.free()
        fk, fv = ps.HostFrame(4 * n), ps.HostFrame(4 * n)
        fk.array(np.uint32, n)[:] = np.arange(n, dtype=np.uint32)
        fv.array(np.float32, n)[:] = 7.0
        sh.sync()
        for _ in range(32):  # several ms of device work queued ahead of the frame Add
            sh.add(big_k, big_v, sorted_hint=True)
        sh.add(fk.array(np.uint32, n), fv.array(np.float32, n), frame=True)
        pk, pv = fk.ptr, fv.ptr
        fk.free()
        fv.free()
        st = ps.host_pool_stats()
        assert st["held_bytes"] >= 8 * n, st  # the device work ahead is far from done
        again = [ps.HostFrame(4 * n) for _ in range(2)]  # from the cache, not the held frames
        assert not {f.ptr for f in again} & {pk, pv}, "a held frame was handed out"
        for f in again:
            f.array(np.uint8, 4 * n)[:] = 0xFF
        sh.sync()
        assert ps.host_pool_stats()["held_bytes"] == 0
        out = sh.get(np.arange(n, dtype=np.uint32))
        assert np.all(out == 7.0)
        again_ptrs = [f.ptr for f in again]
        for f in again:
            f.free()
        cached = {pk, pv} | set(again_ptrs)
        reused = ps.HostFrame(4 * n)
        assert reused.ptr in cached, "a cached frame of the class comes back"
        reused.free()


def test_frame_flag_outside_frames_and_errors(cuda, oracle_mod):
    """PSKV_HOST_FRAME on pointers that are not (wholly) in frames takes the
    ordinary host paths; freeing twice or freeing a non-frame is EINVAL."""
    import parameter_server_amd as ps

    rng = np.random.default_rng(3)
    k = rng.integers(0, 50_000, size=20_000).astype(np.uint32)
    v = rng.standard_normal(k.size)
    ref = oracle_mod.MapStorageRef(np.float64)
    ref.add(k, v)
    ref.add(k[:10], v[:10])
    with ps.Shard(0, 40_000, np.float64, overflow_slots=1 << 15) as sh:
        f = ps.HostFrame(k.nbytes)
        fk = f.array(np.uint32, k.size)
        fk[:] = k
        sh.add(fk, v, frame=True)            # keys in a frame, values pageable
        sh.add(k[:10], v[:10], frame=True)   # neither in a frame (inline size)
        q = np.arange(0, 50_000, dtype=np.uint32)
        assert_bits_equal(sh.get(q, frame=True), ref.get(q), "mixed frame/pageable")
        f.free()
    from parameter_server_amd import _lib

    f2 = ps.HostFrame(100)
    p = f2.ptr
    f2.free()
    assert _lib.lib.pskv_host_free(p) == _lib.PSKV_EINVAL  # freed twice
    buf = np.zeros(16, np.uint8)
    assert _lib.lib.pskv_host_free(buf.ctypes.data) == _lib.PSKV_EINVAL


def test_frame_pool_reuses_and_trims(cuda):
    import parameter_server_amd as ps

    ps.host_pool_trim()
    a = ps.HostFrame(10_000)
    p = a.ptr
    a.free()
    st = ps.host_pool_stats()
    assert st["cached_bytes"] >= 10_000 and st["held_bytes"] == 0
    b = ps.HostFrame(9_000)  # same 16 KiB class: the cached frame comes back
    assert b.ptr == p
    assert b.ptr % 4096 == 0
    b.free()
    ps.host_pool_trim()
    assert ps.host_pool_stats()["cached_bytes"] == 0


def test_page_locked_memory_has_one_address_on_every_device(cuda):
    """The multi-device assumption behind in-place frame access:
    page-locked host memory is mapped at its host address on every device, so
    one frame pointer serves a kernel on any device (pskv_frames.cpp keeps a
    frame's view only when hipHostGetDevicePointer returns the host address).
    Checked on every visible device through the HIP runtime itself."""
    import ctypes

    import torch

    hip = ctypes.CDLL("libamdhip64.so")
    p = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(1 << 16),
                             ctypes.c_uint(0x1 | 0x2)) == 0  # Portable | Mapped
    try:
        for d in range(torch.cuda.device_count()):
            assert hip.hipSetDevice(d) == 0
            dv = ctypes.c_void_p()
            assert hip.hipHostGetDevicePointer(ctypes.byref(dv), p, ctypes.c_uint(0)) == 0
            assert dv.value == p.value, f"device {d}: view {dv.value:#x} != host {p.value:#x}"
    finally:
        hip.hipSetDevice(0)
        hip.hipHostFree(p)
