"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the Add/Get hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / CPU baseline.  The product path
(parameter_server_amd, libpskv.so) never touches it.

Contents
  MapStorageRef / VectorStorageRef  ctypes handles on oracle/liboracle.so, the C++
      restatement of server/map_storage.hpp:17-45 and server/vector_storage.hpp:16-49
  dense_last_wins / accumulate_ref   numpy restatements for sizes the tree/scan
      restatements cannot reach in seconds (validated against them at small sizes
      in tests/test_oracle.py)
  range_slice_ref                    pure-Python restatement of
      base/range_partition_manager.hpp:19-46 (small inputs)
  jump_hash_ref / hash_slice_ref     pure-Python restatement of the jump consistent
      hash (Lamping & Veach 2014) and of ConsistentHashingPartitionManager::Slice
      (base/consistent_hashing_partition_manager.hpp:18-42,81-89)

Parity pin: the reference cannot be built here (its storages include
glog/logging.h, absent from the image, and a stand-in header is not allowed), so
these restatements are pinned by the reference's own known-answer tests and the
reference probe outputs recorded in SURVEY.md §0 (tests/golden/*.json).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

DTYPES = {0: np.int32, 1: np.float32, 2: np.float64}
DTYPE_CODE = {np.dtype(np.int32): 0, np.dtype(np.float32): 1, np.dtype(np.float64): 2}


def build(quiet: bool = True) -> str:
    """Compile liboracle.so with the committed Makefile (g++)."""
    import subprocess

    out = subprocess.run(["make", "-C", _HERE], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)
    return os.path.join(_HERE, "liboracle.so")


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.oracle_create.restype = ctypes.c_void_p
        L.oracle_create.argtypes = [ctypes.c_int, ctypes.c_int]
        L.oracle_destroy.argtypes = [ctypes.c_void_p]
        L.oracle_add.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
        L.oracle_get.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_size.restype = ctypes.c_uint64
        L.oracle_size.argtypes = [ctypes.c_void_p]
        L.oracle_range_assign.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        _LIB = L
    return _LIB


class _StorageRef:
    kind = -1

    def __init__(self, dtype=np.float32):
        self.dtype = np.dtype(dtype)
        self._h = lib().oracle_create(self.kind, DTYPE_CODE[self.dtype])
        if not self._h:
            raise ValueError("bad dtype")

    def close(self):
        if self._h:
            lib().oracle_destroy(self._h)
            self._h = None

    __del__ = close

    def add(self, keys, vals):
        k = np.ascontiguousarray(keys, dtype=np.uint32)
        v = np.ascontiguousarray(vals, dtype=self.dtype)
        if k.shape != v.shape:
            raise ValueError("CHECK_EQ(keys.size(), vals.size()) failed")
        lib().oracle_add(self._h, k.ctypes.data, v.ctypes.data, k.size)

    def get(self, keys):
        k = np.ascontiguousarray(keys, dtype=np.uint32)
        out = np.empty(k.size, dtype=self.dtype)
        lib().oracle_get(self._h, k.ctypes.data, k.size, out.ctypes.data)
        return out

    def size(self) -> int:
        return int(lib().oracle_size(self._h))


class MapStorageRef(_StorageRef):
    """server/map_storage.hpp:17-45 — std::map, assign, 0 for absent keys."""
    kind = 0


class VectorStorageRef(_StorageRef):
    """server/vector_storage.hpp:16-49 — append; Get = O(stored x queried) last-match scan."""
    kind = 1


def dense_last_wins(param: np.ndarray, key_begin: int, keys: np.ndarray, vals: np.ndarray) -> None:
    """Apply one assign batch to a dense array in place: the LAST occurrence of a
    key wins (map_storage.hpp:22-23 sequential loop).  Keys must be in range."""
    keys = np.asarray(keys, dtype=np.uint32)
    if keys.size == 0:
        return
    rev = keys[::-1]
    u, first_in_rev = np.unique(rev, return_index=True)
    last = keys.size - 1 - first_in_rev
    param[u.astype(np.int64) - key_begin] = np.asarray(vals)[last]


def accumulate_ref(param64: np.ndarray, abs64: np.ndarray, key_begin: int, keys, vals) -> None:
    """Accumulate-mode reference: exact-ish float64 sums plus the running sum of
    |v| used by the stated tolerance (DESIGN.md §Accumulate tolerance)."""
    idx = np.asarray(keys, dtype=np.int64) - key_begin
    v = np.asarray(vals, dtype=np.float64)
    np.add.at(param64, idx, v)
    np.add.at(abs64, idx, np.abs(v))


def range_slice_ref(ranges, keys):
    """Pure-Python restatement of RangePartitionManager::Slice
    (base/range_partition_manager.hpp:19-46).  ranges: list of (begin, end) in
    server order; returns [(range_index, [keys...]), ...]."""
    out = []
    r, server = 0, -1
    i = 0
    keys = [int(k) for k in keys]
    while i < len(keys):
        k = keys[i]
        b, e = ranges[r]
        if (b <= k < e) or r + 1 >= len(ranges):
            if server < r:
                server = r
                out.append((r, [k]))
            else:
                out[-1][1].append(k)
            i += 1
        else:
            r += 1
    return out


def jump_hash_ref(key: int, num_buckets: int) -> int:
    """Jump consistent hash as published (Lamping & Veach, 2014) and as the
    reference states it (base/consistent_hashing_partition_manager.hpp:81-89):
    64-bit LCG state, next candidate (b + 1) * 2^31 / ((state >> 33) + 1) in
    double precision, truncated."""
    key &= (1 << 64) - 1
    b, j = -1, 0
    while j < num_buckets:
        b = j
        key = (key * 2862933555777941757 + 1) & ((1 << 64) - 1)
        j = int((b + 1) * (float(1 << 31) / float((key >> 33) + 1)))
    return b


def hash_slice_ref(server_ids, keys, vals=None):
    """ConsistentHashingPartitionManager::Slice (base/consistent_hashing_partition_manager.hpp:18-76):
    one slice per receiving server, in order of its first key; keys (and
    values) in input order.  Returns [(server_id, [keys...]) or (server_id,
    [keys...], [vals...]), ...]."""
    out, where = [], {}
    for i, k in enumerate(keys):
        sid = server_ids[jump_hash_ref(int(k), len(server_ids))]
        if sid not in where:
            where[sid] = len(out)
            out.append((sid, [], []) if vals is not None else (sid, []))
        out[where[sid]][1].append(int(k))
        if vals is not None:
            out[where[sid]][2].append(float(vals[i]))
    return out


def range_assign(ranges, keys) -> np.ndarray:
    """C restatement of the same walk (fast): range index for every key."""
    rb = np.ascontiguousarray([b for b, _ in ranges], dtype=np.uint64)
    re = np.ascontiguousarray([e for _, e in ranges], dtype=np.uint64)
    k = np.ascontiguousarray(keys, dtype=np.uint32)
    out = np.empty(k.size, dtype=np.int32)
    if k.size:
        lib().oracle_range_assign(rb.ctypes.data, re.ctypes.data, len(ranges), k.ctypes.data,
                                  k.size, out.ctypes.data)
    return out
