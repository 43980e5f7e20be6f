"""Host-side mirror of the reference storage plugin surface, backed by HBM.

Mirrors, with the same names, argument meaning and error behaviour:
  Flag, Meta, Message           base/message.hpp:14-58 (Message.data = list of byte arrays,
                                 the SArray<char> frames of the reference)
  AbstractStorage               server/abstract_storage.hpp:12-42 (template-method Add/Get;
                                 Get echoes the request keys and swaps sender/recver)
  HipStorage                    drop-in for MapStorage<Val> / VectorStorage<Val>
                                 (server/map_storage.hpp, server/vector_storage.hpp)
  RangePartitionManager         base/range_partition_manager.hpp:14-77 (through pskv_range_slice)
  ConsistentHashingPartitionManager
                                base/consistent_hashing_partition_manager.hpp:9-90 (through pskv_jump_hash)

A reference glog CHECK failure aborts the process; here it raises CheckError.
The C++ adaptor with the same shape is include/ps/hip_storage.hpp.
"""
from __future__ import annotations

import enum
from dataclasses import dataclass, field
from typing import List

import numpy as np

from .shard import Shard, jump_hash, range_slice


class CheckError(AssertionError):
    """A failed reference CHECK (glog would abort)."""


def CHECK(cond, msg=""):
    if not cond:
        raise CheckError(msg or "CHECK failed")


class Flag(enum.IntEnum):  # base/message.hpp:14
    kExit = 0
    kBarrier = 1
    kResetWorkerInModel = 2
    kClock = 3
    kAdd = 4
    kGet = 5


@dataclass
class Meta:  # base/message.hpp:17-37
    flag: Flag = Flag.kExit
    sender: int = -1
    recver: int = -1
    model_id: int = -1


@dataclass
class Message:  # base/message.hpp:39-58
    meta: Meta = field(default_factory=Meta)
    data: List[np.ndarray] = field(default_factory=list)

    def AddData(self, arr) -> None:
        """Append one frame; like SArray<char>(SArray<V>) it is a zero-copy byte view."""
        a = np.ascontiguousarray(arr)
        self.data.append(a.view(np.uint8).reshape(-1))


def typed(frame: np.ndarray, dtype) -> np.ndarray:
    """SArray<W>(SArray<char>) reinterpret (sarray.h:67-82): size = bytes / sizeof(W),
    truncated to whole elements."""
    dt = np.dtype(dtype)
    b = np.ascontiguousarray(frame).view(np.uint8).reshape(-1)
    whole = (b.size // dt.itemsize) * dt.itemsize
    return b[:whole].view(dt)


class AbstractStorage:
    """server/abstract_storage.hpp:12-42."""

    def Add(self, msg: Message) -> None:
        CHECK(len(msg.data) == 2, "CHECK(msg.data.size() == 2)")
        typed_keys = typed(msg.data[0], np.uint32)
        self.SubAdd(typed_keys, msg.data[1])

    def Get(self, msg: Message) -> Message:
        CHECK(len(msg.data) == 1, "CHECK(msg.data.size() == 1)")
        typed_keys = typed(msg.data[0], np.uint32)
        reply = Message()
        reply.meta.recver = msg.meta.sender
        reply.meta.sender = msg.meta.recver
        reply.meta.flag = msg.meta.flag
        reply.meta.model_id = msg.meta.model_id
        reply_keys = typed_keys  # aliases the request keys (abstract_storage.hpp:27)
        reply_vals = self.SubGet(reply_keys)
        reply.AddData(reply_keys)
        reply.AddData(reply_vals)
        return reply

    def SubAdd(self, typed_keys: np.ndarray, vals: np.ndarray) -> None:
        raise NotImplementedError

    def SubGet(self, typed_keys: np.ndarray) -> np.ndarray:
        raise NotImplementedError

    def FinishIter(self) -> None:
        raise NotImplementedError


class HipStorage(AbstractStorage):
    """HBM-resident storage: every SubAdd / SubGet runs the HIP kernels.

    Defaults reproduce the reference's argument-less construction
    (driver/engine.hpp:100-109): the whole uint32 key space, assign semantics."""

    def __init__(self, val_dtype=np.float32, key_begin: int = 0, key_end: int = 1 << 32,
                 device: int = 0, mode: str = "assign", overflow_slots: int = 0):
        self.val_dtype = np.dtype(val_dtype)
        self.shard = Shard(key_begin, key_end, self.val_dtype, mode=mode, device=device,
                           overflow_slots=overflow_slots)

    def SubAdd(self, typed_keys, vals) -> None:
        typed_vals = typed(vals, self.val_dtype)
        CHECK(typed_keys.size == typed_vals.size,
              f"CHECK_EQ(typed_keys.size(), typed_vals.size()) failed: {typed_keys.size} vs {typed_vals.size}")
        self.shard.add(typed_keys, typed_vals)

    def SubGet(self, typed_keys) -> np.ndarray:
        vals = self.shard.get(np.ascontiguousarray(typed_keys, dtype=np.uint32))
        return vals.view(np.uint8)

    def FinishIter(self) -> None:
        self.shard.sync()

    def close(self):
        self.shard.close()


class RangePartitionManager:
    """base/range_partition_manager.hpp:14-77 — contiguous key ranges, one per
    server thread.  Keys are assumed sorted, exactly as the reference assumes:
    out-of-order or out-of-range keys fall through to later / the last server."""

    def __init__(self, server_thread_ids, ranges):
        self.server_thread_ids_ = list(server_thread_ids)
        self.ranges_ = [(int(b), int(e)) for b, e in ranges]

    def GetNumServers(self) -> int:
        return len(self.server_thread_ids_)

    def GetServerThreadIds(self):
        return list(self.server_thread_ids_)

    def Slice(self, keys_or_kvs):
        if isinstance(keys_or_kvs, tuple):
            keys, vals = keys_or_kvs
            keys = np.ascontiguousarray(keys, dtype=np.uint32)
            vals = np.ascontiguousarray(vals, dtype=np.float64)  # KVPairs carry double (abstract_partition_manager.hpp:21-22)
            return [(self.server_thread_ids_[r], (keys[s:s + n], vals[s:s + n]))
                    for r, s, n in range_slice(self.ranges_, keys)]
        keys = np.ascontiguousarray(keys_or_kvs, dtype=np.uint32)
        return [(self.server_thread_ids_[r], keys[s:s + n]) for r, s, n in range_slice(self.ranges_, keys)]


class ConsistentHashingPartitionManager:
    """base/consistent_hashing_partition_manager.hpp:9-90 — the reference
    Engine's default partitioner (driver/engine.hpp:143-150): key -> server
    server_thread_ids[JumpConsistentHash(key, #servers)].  Slices come in order
    of each server's first key, keys (and values, as double) in input order,
    as the reference's own test pins
    (base/consistent_hashing_partition_manager_test.cpp:48-139)."""

    def __init__(self, server_thread_ids):
        self.server_thread_ids_ = list(server_thread_ids)

    def GetNumServers(self) -> int:
        return len(self.server_thread_ids_)

    def GetServerThreadIds(self):
        return list(self.server_thread_ids_)

    def _groups(self, keys):
        b = jump_hash(keys, len(self.server_thread_ids_))
        if b.size == 0:
            return []
        first = np.unique(b, return_index=True)[1]          # first appearance of each bucket
        order = b[np.sort(first)]
        return [(int(x), np.nonzero(b == x)[0]) for x in order]

    def Slice(self, keys_or_kvs):
        if isinstance(keys_or_kvs, tuple):
            keys, vals = keys_or_kvs
            keys = np.ascontiguousarray(keys, dtype=np.uint32)
            vals = np.ascontiguousarray(vals, dtype=np.float64)  # KVPairs carry double
            return [(self.server_thread_ids_[x], (keys[i], vals[i])) for x, i in self._groups(keys)]
        keys = np.ascontiguousarray(keys_or_kvs, dtype=np.uint32)
        return [(self.server_thread_ids_[x], keys[i]) for x, i in self._groups(keys)]
