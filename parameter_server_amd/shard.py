"""Shard: Python handle on one HBM-resident parameter shard (pskv_shard).

Host inputs are numpy arrays (they stand for the zmq receive buffers the
reference storage sees, comm/mailbox.cpp:246-257); device inputs are torch
tensors on the shard's GPU (PyTorch only supplies memory and streams — every
byte of the Add/Get work is done by the HIP kernels in libpskv.so).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import check, lib

_NP_DTYPE = {_lib.PSKV_I32: np.dtype(np.int32), _lib.PSKV_F32: np.dtype(np.float32),
             _lib.PSKV_F64: np.dtype(np.float64)}
_DTYPE_CODE = {v: k for k, v in _NP_DTYPE.items()}


def dtype_code(dtype) -> int:
    try:
        import torch

        if isinstance(dtype, torch.dtype):
            dtype = {torch.int32: np.int32, torch.float32: np.float32, torch.float64: np.float64}[dtype]
    except ImportError:
        pass
    return _DTYPE_CODE[np.dtype(dtype)]


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def device_count() -> int:
    return int(lib.pskv_device_count())


class Shard:
    """A key range [key_begin, key_end) of uint32 keys held in HBM.

    mode "assign" is the reference semantics (last write wins, missing -> 0);
    "accumulate" is the gradient-reduction mode (param[k] += v)."""

    def __init__(self, key_begin: int = 0, key_end: int = 1 << 32, dtype=np.float32,
                 mode: str = "assign", device: int = 0, overflow_slots: int = 0, options=None):
        self.dtype = np.dtype(dtype) if not _is_torch(dtype) else _NP_DTYPE[dtype_code(dtype)]
        self.code = dtype_code(self.dtype)
        self.mode = {"assign": _lib.PSKV_ASSIGN, "accumulate": _lib.PSKV_ACCUMULATE}[mode]
        self.key_begin, self.key_end, self.device = int(key_begin), int(key_end), int(device)
        h = ctypes.c_void_p()
        check(lib.pskv_shard_create_ex(self.device, self.key_begin, self.key_end, self.code,
                                       self.mode, int(overflow_slots), ctypes.byref(h)))
        self._h = h
        for name, value in (options or {}).items():
            self.set_option(name, value)

    # ------------------------------------------------------------ lifetime
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib.pskv_shard_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self):
        return self._h

    # ------------------------------------------------------------ helpers
    def _host_keys(self, keys):
        return np.ascontiguousarray(keys, dtype=np.uint32)

    def _host_vals(self, vals, n):
        v = np.ascontiguousarray(vals, dtype=self.dtype)
        if v.size != n:
            raise ValueError(f"CHECK_EQ(keys.size(), vals.size()) failed: {n} vs {v.size}")
        return v

    # ------------------------------------------------------------ Add / Get
    def add(self, keys, vals, sorted_hint: bool = False, frame: bool = False):
        """Push one batch.  numpy -> host path; torch CUDA tensors -> device path.
        frame=True: host arrays that live in HostFrames are borrowed until the
        frames are freed (PSKV_HOST_FRAME): read in place, no wait."""
        if _is_torch(keys):
            self._check_dev(keys, vals)
            flags = _lib.PSKV_DEVICE | (_lib.PSKV_SORTED_HINT if sorted_hint else 0)
            if vals.numel() != keys.numel():
                raise ValueError("CHECK_EQ(keys.size(), vals.size()) failed")
            check(lib.pskv_add(self._h, keys.data_ptr(), vals.data_ptr(), keys.numel(), flags))
            return
        k = self._host_keys(keys)
        v = self._host_vals(vals, k.size)
        flags = _lib.PSKV_HOST_FRAME if frame else _lib.PSKV_HOST
        check(lib.pskv_add(self._h, k.ctypes.data, v.ctypes.data, k.size, flags))

    def get(self, keys, out=None, frame: bool = False):
        """Pull one batch.  numpy keys -> returns a numpy array (synchronous);
        torch keys -> fills/returns a torch tensor (stream-ordered)."""
        if _is_torch(keys):
            import torch

            if out is None:
                out = torch.empty(keys.numel(), dtype=_torch_dtype(self.dtype), device=keys.device)
            self._check_dev(keys, out)
            check(lib.pskv_get(self._h, keys.data_ptr(), keys.numel(), out.data_ptr(),
                               _lib.PSKV_DEVICE))
            return out
        k = self._host_keys(keys)
        res = np.empty(k.size, dtype=self.dtype) if out is None else out
        flags = _lib.PSKV_HOST_FRAME if frame else _lib.PSKV_HOST
        check(lib.pskv_get(self._h, k.ctypes.data, k.size, res.ctypes.data, flags))
        return res

    def prepare(self, batches, is_get: bool = False) -> "BatchSet":
        """Validate and pack a batch list once, for repeated grouped calls."""
        arr, keep, flags = self._batch_array(batches, is_get=is_get)
        return BatchSet(arr, len(batches), flags, keep)

    def add_grouped(self, batches, sorted_hint: bool = False, frame: bool = False):
        """batches: list of (keys, vals) (all torch-device or all numpy-host) or a BatchSet."""
        bs = batches if isinstance(batches, BatchSet) else self.prepare(batches)
        flags = bs.flags
        if sorted_hint and flags & _lib.PSKV_DEVICE:
            flags |= _lib.PSKV_SORTED_HINT
        if frame and not flags & _lib.PSKV_DEVICE:
            flags |= _lib.PSKV_HOST_FRAME
        check(lib.pskv_add_grouped(self._h, bs.arr, bs.n, flags))

    def get_grouped(self, batches, frame: bool = False):
        """batches: list of (keys, out) pairs (out filled in place) or a BatchSet."""
        bs = batches if isinstance(batches, BatchSet) else self.prepare(batches, is_get=True)
        flags = bs.flags
        if frame and not flags & _lib.PSKV_DEVICE:
            flags |= _lib.PSKV_HOST_FRAME
        check(lib.pskv_get_grouped(self._h, bs.arr, bs.n, flags))

    def add_get_grouped(self, adds, gets, sorted_hint: bool = False):
        """add_grouped(adds) then get_grouped(gets) in ONE call (pskv_add_get_grouped:
        the BSP model's flush then the Gets it releases, or a worker round's push
        then pull); the hint applies to the Adds.  adds / gets: batch lists or
        BatchSets."""
        ba = adds if isinstance(adds, BatchSet) else self.prepare(adds)
        bg = gets if isinstance(gets, BatchSet) else self.prepare(gets, is_get=True)
        if (ba.flags ^ bg.flags) & _lib.PSKV_DEVICE and ba.n and bg.n:
            raise ValueError("add_get_grouped: adds and gets must both be device or both host batches")
        flags = ba.flags if ba.n else bg.flags
        if sorted_hint and flags & _lib.PSKV_DEVICE:
            flags |= _lib.PSKV_SORTED_HINT
        check(lib.pskv_add_get_grouped(self._h, ba.arr, ba.n, bg.arr, bg.n, flags))

    def _batch_array(self, batches, is_get):
        arr = (_lib.PskvBatch * max(1, len(batches)))()
        keep = []
        dev = None
        for i, (k, v) in enumerate(batches):
            t = _is_torch(k)
            if dev is None:
                dev = t
            if t != dev:
                raise ValueError("mixed host/device batches in one grouped call")
            if t:
                self._check_dev(k, v)
                if v.numel() != k.numel():
                    raise ValueError("CHECK_EQ(keys.size(), vals.size()) failed")
                keep += [k, v]
                arr[i] = _lib.PskvBatch(k.data_ptr(), v.data_ptr(), k.numel())
            else:
                kk = self._host_keys(k)
                if is_get:
                    if not (isinstance(v, np.ndarray) and v.dtype == self.dtype and v.flags.c_contiguous):
                        raise ValueError("get_grouped host outputs must be C-contiguous arrays of the shard dtype")
                    vv = v
                else:
                    vv = self._host_vals(v, kk.size)
                keep += [kk, vv]
                arr[i] = _lib.PskvBatch(kk.ctypes.data, vv.ctypes.data, kk.size)
        return arr, keep, (_lib.PSKV_DEVICE if dev else _lib.PSKV_HOST)

    def _check_dev(self, *ts):
        for t in ts:
            if not t.is_cuda or t.device.index != self.device or not t.is_contiguous():
                raise ValueError("device tensors must be contiguous and on the shard's GPU")

    # ------------------------------------------------------------ control
    _GENERAL = {"stamps": 0, "auto": 1, "radix": 2}

    def set_option(self, name: str, value):
        """pskv_set_option: a tuning / path option of this shard (include/pskv.h).
        GENERAL also takes "stamps" / "auto" / "radix"; booleans as 0 / 1."""
        if name == "GENERAL" and isinstance(value, str):
            value = self._GENERAL[value]
        check(lib.pskv_set_option(self._h, name.encode(), int(value)))

    def get_option(self, name: str) -> int:
        v = ctypes.c_int64()
        check(lib.pskv_get_option(self._h, name.encode(), ctypes.byref(v)))
        return v.value

    def sync(self):
        check(lib.pskv_sync(self._h))

    def clear(self):
        check(lib.pskv_clear(self._h))

    def set_stream(self, stream_handle):
        """stream_handle: int hipStream_t (e.g. torch.cuda.current_stream().cuda_stream) or None."""
        check(lib.pskv_set_stream(self._h, stream_handle))

    def dense_ptr(self) -> int:
        return int(lib.pskv_dense_ptr(self._h) or 0)

    def info(self) -> dict:
        i = _lib.PskvInfo()
        check(lib.pskv_shard_info(self._h, ctypes.byref(i)))
        return {f: getattr(i, f) for f, _ in _lib.PskvInfo._fields_}

    def set_timing(self, on, kernels=None):
        """on: bool; kernels: optional list of kernel ids (_lib.PSKV_K_*) to time."""
        if kernels is None:
            check(lib.pskv_set_timing(self._h, 1 if on else 0))
        else:
            mask = 0
            for k in kernels:
                mask |= 1 << k
            check(lib.pskv_set_timing_mask(self._h, mask if on else 0))

    def reset_timing(self):
        check(lib.pskv_reset_timing(self._h))

    def kernel_time(self, kernel: int):
        n, ms, el = ctypes.c_uint64(), ctypes.c_double(), ctypes.c_uint64()
        check(lib.pskv_kernel_time(self._h, kernel, ctypes.byref(n), ctypes.byref(ms), ctypes.byref(el)))
        return {"launches": n.value, "total_ms": ms.value, "elements": el.value}

    def dense_view(self):
        """A torch tensor aliasing the dense HBM array (tests only; no copy)."""
        import torch

        n = self.key_end - self.key_begin
        ptr = self.dense_ptr()
        return _tensor_from_ptr(ptr, n, _torch_dtype(self.dtype), self.device)


class BatchSet:
    """A packed pskv_batch array (plus references keeping its buffers alive)."""

    def __init__(self, arr, n, flags, keep):
        self.arr, self.n, self.flags, self._keep = arr, n, flags, keep


def _torch_dtype(npdt):
    import torch

    return {np.dtype(np.int32): torch.int32, np.dtype(np.float32): torch.float32,
            np.dtype(np.float64): torch.float64}[np.dtype(npdt)]


def _tensor_from_ptr(ptr, n, tdtype, device):
    """Wrap raw device memory as a torch tensor via __cuda_array_interface__."""
    import torch

    typestr = {torch.int32: "<i4", torch.float32: "<f4", torch.float64: "<f8"}[tdtype]

    class _Holder:
        __cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (ptr, False),
                                    "version": 2, "strides": None}

    with torch.cuda.device(device):
        return torch.as_tensor(_Holder(), device=f"cuda:{device}")


class HostFrame:
    """A page-locked host frame from the library's pool (pskv_host_alloc): the
    buffer a mailbox receives one message payload into (comm/mailbox.cpp:246-257).
    `array(dtype, n, offset)` views it as numpy; `free()` returns it (the pool
    holds it back until queued PSKV_HOST_FRAME reads of it have run)."""

    def __init__(self, nbytes: int):
        p = ctypes.c_void_p()
        check(lib.pskv_host_alloc(int(nbytes), ctypes.byref(p)))
        self.ptr, self.nbytes = p.value, int(nbytes)

    def array(self, dtype, n: int, offset: int = 0) -> np.ndarray:
        dt = np.dtype(dtype)
        if self.ptr is None or offset < 0 or offset + n * dt.itemsize > self.nbytes:
            raise ValueError("view outside the frame")
        buf = (ctypes.c_char * (n * dt.itemsize)).from_address(self.ptr + offset)
        return np.frombuffer(buf, dtype=dt, count=n)

    def free(self):
        if self.ptr is not None:
            p, self.ptr = self.ptr, None
            check(lib.pskv_host_free(p))

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.free()


def host_pool_stats() -> dict:
    v = [ctypes.c_uint64() for _ in range(3)]
    check(lib.pskv_host_pool_stats(*[ctypes.byref(x) for x in v]))
    return {"live_bytes": v[0].value, "cached_bytes": v[1].value, "held_bytes": v[2].value}


def host_pool_trim():
    check(lib.pskv_host_pool_trim())


def range_slice(ranges, keys):
    """Mirror of RangePartitionManager::Slice through the product library
    (pskv_range_slice).  Returns [(range_index, start, length), ...]."""
    k = np.ascontiguousarray(keys, dtype=np.uint32)
    nr = len(ranges)
    rb = np.ascontiguousarray([b for b, _ in ranges], dtype=np.uint64)
    re = np.ascontiguousarray([e for _, e in ranges], dtype=np.uint64)
    sr = np.empty(max(nr, 1), dtype=np.int32)
    ss = np.empty(max(nr, 1), dtype=np.uint64)
    sl = np.empty(max(nr, 1), dtype=np.uint64)
    ns = check(lib.pskv_range_slice(rb.ctypes.data, re.ctypes.data, nr, k.ctypes.data, k.size,
                                    sr.ctypes.data, ss.ctypes.data, sl.ctypes.data))
    return [(int(sr[i]), int(ss[i]), int(sl[i])) for i in range(ns)]


def jump_hash(keys, num_buckets: int) -> np.ndarray:
    """Bucket of every key under the reference's default partitioner
    (ConsistentHashingPartitionManager, base/consistent_hashing_partition_manager.hpp:81-89)
    through the product library (pskv_jump_hash).  int32 array, values in
    [0, num_buckets)."""
    k = np.ascontiguousarray(keys, dtype=np.uint32)
    out = np.empty(k.size, dtype=np.int32)
    check(lib.pskv_jump_hash(k.ctypes.data, k.size, int(num_buckets), out.ctypes.data))
    return out
