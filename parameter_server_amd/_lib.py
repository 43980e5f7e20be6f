"""ctypes binding of libpskv.so (the C ABI in include/pskv.h).

The shared library is built in-tree by __graft_entry__.build() (hipcc,
--offload-arch=gfx950).  There is no fallback: if the library is missing or
fails to load, importing this module raises, so no test or bench can silently
run without the HIP kernels.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# PSKV_LIB_PATH: a diagnostic build of the same library (tools/step_stamps.py);
# never set by tests, smoke() or bench.py
LIB_PATH = os.environ.get("PSKV_LIB_PATH") or os.path.join(_HERE, "libpskv.so")

# keep in sync with include/pskv.h
PSKV_OK = 0
PSKV_EINVAL = -1
PSKV_EHIP = -2
PSKV_ENOMEM = -3
PSKV_ESTATE = -4

PSKV_I32, PSKV_F32, PSKV_F64 = 0, 1, 2
PSKV_ASSIGN, PSKV_ACCUMULATE = 0, 1
PSKV_HOST, PSKV_DEVICE, PSKV_SORTED_HINT, PSKV_HOST_FRAME = 0x0, 0x1, 0x2, 0x4

PSKV_K_GATHER = 0
PSKV_K_ASSIGN_SORTED = 1
PSKV_K_ASSIGN_TILES = 2
PSKV_K_GENERAL_MARK = 3
PSKV_K_GENERAL_COMMIT = 4
PSKV_K_RADIX = 5
PSKV_K_DENSE_CHECK = 6
PSKV_K_ACC_DENSE = 7
PSKV_K_INLINE_ADD = 8
PSKV_K_INLINE_GET = 9
PSKV_K_REPLAY = 10
PSKV_K_COUNT = 11
KERNEL_NAMES = {
    PSKV_K_GATHER: "k_gather",
    PSKV_K_ASSIGN_SORTED: "k_assign_sorted",
    PSKV_K_ASSIGN_TILES: "k_assign_group",
    PSKV_K_GENERAL_MARK: "k_general_mark",
    PSKV_K_GENERAL_COMMIT: "k_general_commit",
    PSKV_K_RADIX: "k_radix_bucket",
    PSKV_K_DENSE_CHECK: "k_dense_check",
    PSKV_K_ACC_DENSE: "k_acc_dense",
    PSKV_K_INLINE_ADD: "k_inline_add",
    PSKV_K_INLINE_GET: "k_inline_get",
    PSKV_K_REPLAY: "k_replay",
}

# Every symbol include/pskv.h declares (checked by tests/test_abi.py).
EXPORTED = [
    "pskv_shard_create", "pskv_shard_create_ex", "pskv_shard_destroy", "pskv_add", "pskv_get",
    "pskv_add_grouped", "pskv_get_grouped", "pskv_add_get_grouped", "pskv_sync", "pskv_clear", "pskv_set_stream",
    "pskv_get_stream", "pskv_dense_ptr", "pskv_shard_info", "pskv_set_timing", "pskv_set_timing_mask",
    "pskv_kernel_time", "pskv_reset_timing", "pskv_range_slice", "pskv_jump_hash", "pskv_last_error",
    "pskv_abi_version", "pskv_device_count", "pskv_host_alloc", "pskv_host_free",
    "pskv_host_pool_stats", "pskv_host_pool_trim", "pskv_set_option", "pskv_get_option",
]


class PskvBatch(ctypes.Structure):
    _fields_ = [("keys", ctypes.c_void_p), ("vals", ctypes.c_void_p), ("n", ctypes.c_uint64)]


class PskvInfo(ctypes.Structure):
    _fields_ = [
        ("device", ctypes.c_int), ("dtype", ctypes.c_int), ("mode", ctypes.c_int),
        ("value_bytes", ctypes.c_int), ("key_begin", ctypes.c_uint32), ("key_end", ctypes.c_uint64),
        ("dense_bytes", ctypes.c_uint64), ("overflow_capacity", ctypes.c_uint64),
        ("overflow_count", ctypes.c_uint64), ("n_add_calls", ctypes.c_uint64),
        ("n_get_calls", ctypes.c_uint64), ("n_sorted_launches", ctypes.c_uint64),
        ("n_general_launches", ctypes.c_uint64),
    ]


class PskvError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"pskv error {code}: {msg}")
        self.code = code


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: the HIP extension has not been built "
            "(run `python -c 'import __graft_entry__ as g; g.build()'`)")
    L = ctypes.CDLL(LIB_PATH)
    vp, u64, i32, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint32
    sig = {
        "pskv_shard_create": ([i32, u32, u64, i32, i32, ctypes.POINTER(vp)], i32),
        "pskv_shard_create_ex": ([i32, u32, u64, i32, i32, u64, ctypes.POINTER(vp)], i32),
        "pskv_shard_destroy": ([vp], i32),
        "pskv_add": ([vp, vp, vp, u64, i32], i32),
        "pskv_get": ([vp, vp, u64, vp, i32], i32),
        "pskv_add_grouped": ([vp, ctypes.POINTER(PskvBatch), u64, i32], i32),
        "pskv_get_grouped": ([vp, ctypes.POINTER(PskvBatch), u64, i32], i32),
        "pskv_add_get_grouped": ([vp, ctypes.POINTER(PskvBatch), u64, ctypes.POINTER(PskvBatch), u64, i32], i32),
        "pskv_sync": ([vp], i32),
        "pskv_clear": ([vp], i32),
        "pskv_set_stream": ([vp, vp], i32),
        "pskv_get_stream": ([vp], vp),
        "pskv_dense_ptr": ([vp], vp),
        "pskv_shard_info": ([vp, ctypes.POINTER(PskvInfo)], i32),
        "pskv_set_timing": ([vp, i32], i32),
        "pskv_set_timing_mask": ([vp, u32], i32),
        "pskv_kernel_time": ([vp, i32, ctypes.POINTER(u64), ctypes.POINTER(ctypes.c_double),
                              ctypes.POINTER(u64)], i32),
        "pskv_reset_timing": ([vp], i32),
        "pskv_range_slice": ([vp, vp, i32, vp, u64, vp, vp, vp], i32),
        "pskv_jump_hash": ([vp, u64, i32, vp], i32),
        "pskv_last_error": ([], ctypes.c_char_p),
        "pskv_abi_version": ([], i32),
        "pskv_device_count": ([], i32),
        "pskv_host_alloc": ([u64, ctypes.POINTER(vp)], i32),
        "pskv_host_free": ([vp], i32),
        "pskv_host_pool_stats": ([ctypes.POINTER(u64)] * 3, i32),
        "pskv_host_pool_trim": ([], i32),
        "pskv_set_option": ([vp, ctypes.c_char_p, ctypes.c_int64], i32),
        "pskv_get_option": ([vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)], i32),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    return L


lib = _load()


def check(rc: int) -> int:
    if rc < 0:
        raise PskvError(rc, lib.pskv_last_error().decode(errors="replace"))
    return rc
