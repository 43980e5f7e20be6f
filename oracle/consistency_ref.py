"""TEST INFRASTRUCTURE ONLY — an independent restatement of the reference's
consistency models, for checking the cfg-5 replay (tests/cpp/ssp_replay.cpp).

Only tests/ may import this module.  It shares no code with
include/ps/consistency.hpp (the C++ restatement the replay runs): the replay
writes its model traffic with `--trace FILE` -- every message handed to a
server's model, the replies that handling pushed, every shard's final contents
-- and `check_trace` feeds the same arrivals to the models below, over a
dict-backed MapStorage, and compares every reply byte for byte.  A divergence
of consistency.hpp from the reference models, or of the storage behind it (the
HBM shards in the HIP run), shows as the first reply that differs.

Restated from:
  ProgressTracker   server/util/progress_tracker.cpp:7-49
  PendingBuffer     server/util/pending_buffer.cpp:5-28
  SSPModel          server/consistency/ssp_model.cpp:15-57
  BSPModel          server/consistency/bsp_model.cpp:14-86
  ASPModel          server/consistency/asp_model.cpp:14-41
  AbstractStorage   server/abstract_storage.hpp:14-32 (Add / Get template methods)
  MapStorage        server/map_storage.hpp:17-45 (last write wins, 0 if absent)
  ServerThread      server/server_thread.cpp:29-46 (dispatch by flag)

One documented deviation is kept, as consistency.hpp keeps it (DESIGN.md §6,
tests/golden restatement_cases): at a BSP min-clock advance the reference
re-runs each buffered Get through Get() while iterating get_buffer_ and then
clears it (bsp_model.cpp:27-30), so a Get still ahead is pushed onto the vector
being iterated and then dropped; here it stays buffered for the next advance.

Parity pin: the models are checked against the reference's own model tests
(tests/golden/reference_known_answers.json model_cases, run by
tests/test_consistency_ref.py) before they are trusted with a trace.
"""
from __future__ import annotations

import struct
from typing import Dict, List, Optional

import numpy as np

# base/message.hpp:14 Flag (a char enum)
K_EXIT, K_BARRIER, K_RESET, K_CLOCK, K_ADD, K_GET = range(6)


class Msg:
    __slots__ = ("flag", "sender", "recver", "model_id", "data")

    def __init__(self, flag, sender=-1, recver=-1, model_id=-1, data=None):
        self.flag, self.sender, self.recver, self.model_id = flag, sender, recver, model_id
        self.data: List[bytes] = list(data or [])

    def key(self):
        return (self.flag, self.sender, self.recver, self.model_id, tuple(self.data))

    def __repr__(self):
        return (f"Msg(flag={self.flag}, sender={self.sender}, recver={self.recver}, "
                f"model_id={self.model_id}, data=[{', '.join(str(len(d)) + ' B' for d in self.data)}])")


class Tracker:
    """progress_tracker.cpp: per-thread clocks and the min clock."""

    def __init__(self):
        self.prog: Dict[int, int] = {}
        self.min_clock = 0

    def init(self, tids):
        self.min_clock = 0
        for t in tids:  # std::map::insert: an existing entry keeps its clock (:10-11)
            self.prog.setdefault(int(t), 0)

    def progress(self, tid):
        return self.prog[tid]  # .at(): KeyError for an unknown thread (:27)

    def unique_min(self, tid):
        if self.prog[tid] != self.min_clock:
            return False
        return sum(1 for v in self.prog.values() if v == self.min_clock) == 1

    def advance(self, tid):
        was_unique = self.unique_min(tid)
        self.prog[tid] += 1
        if was_unique:
            self.min_clock += 1
            return self.min_clock
        return -1


class MapStore:
    """map_storage.hpp over AbstractStorage's template methods."""

    def __init__(self, dtype):
        self.dtype = np.dtype(dtype)
        self.kv: Dict[int, bytes] = {}
        self.zero = bytes(self.dtype.itemsize)

    def add(self, m: Msg):
        assert len(m.data) == 2  # abstract_storage.hpp:15
        keys = np.frombuffer(m.data[0], dtype=np.uint32)
        w = self.dtype.itemsize
        vals = m.data[1]
        assert len(keys) == len(vals) // w  # map_storage.hpp:20
        for i, k in enumerate(keys.tolist()):
            self.kv[k] = vals[i * w:(i + 1) * w]

    def get(self, m: Msg) -> Msg:
        assert len(m.data) == 1  # abstract_storage.hpp:20
        keys = np.frombuffer(m.data[0], dtype=np.uint32)
        vals = b"".join(self.kv.get(k, self.zero) for k in keys.tolist())
        # reply meta: sender/recver swapped, flag and model_id copied (:23-26)
        return Msg(m.flag, m.recver, m.sender, m.model_id, [m.data[0], vals])


def _reset_reply(m: Msg, model_id: int) -> Msg:
    return Msg(K_RESET, m.recver, m.sender, model_id)


class SSP:
    def __init__(self, model_id, store, staleness, out):
        self.model_id, self.store, self.staleness, self.out = model_id, store, staleness, out
        self.tracker = Tracker()
        self.pending: Dict[int, List[Msg]] = {}

    def clock(self, m):
        new_min = self.tracker.advance(m.sender)
        if new_min != -1:
            # the buffered REQUESTS go to the reply queue (ssp_model.cpp:20-21)
            self.out.extend(self.pending.pop(new_min, []))

    def add(self, m):
        self.store.add(m)

    def get(self, m):
        c = self.tracker.progress(m.sender)
        if c > self.tracker.min_clock + self.staleness:
            self.pending.setdefault(c - self.staleness, []).append(m)
        else:
            self.out.append(self.store.get(m))

    def reset(self, m):
        self.tracker.init(np.frombuffer(m.data[0], dtype=np.uint32).tolist())
        self.out.append(_reset_reply(m, -1))  # model_id left unset (ssp_model.cpp:51-55)


class BSP:
    def __init__(self, model_id, store, out):
        self.model_id, self.store, self.out = model_id, store, out
        self.tracker = Tracker()
        self.adds: List[Msg] = []
        self.gets: List[Msg] = []

    def clock(self, m):
        if self.tracker.advance(m.sender) != -1:
            for a in self.adds:  # arrival order (bsp_model.cpp:20-25)
                self.store.add(a)
            self.adds = []
            gets, self.gets = self.gets, []  # re-buffered Gets survive (deviation above)
            for g in gets:
                self.get(g)

    def add(self, m):
        self.adds.append(m)

    def get(self, m):
        if self.tracker.progress(m.sender) > self.tracker.min_clock:
            self.gets.append(m)
        else:
            self.out.append(self.store.get(m))

    def reset(self, m):
        self.tracker.init(np.frombuffer(m.data[0], dtype=np.uint32).tolist())
        self.out.append(_reset_reply(m, self.model_id))


class ASP:
    def __init__(self, model_id, store, out):
        self.model_id, self.store, self.out = model_id, store, out
        self.tracker = Tracker()

    def clock(self, m):
        pass

    def add(self, m):
        self.store.add(m)

    def get(self, m):
        self.out.append(self.store.get(m))

    def reset(self, m):
        self.tracker.init(np.frombuffer(m.data[0], dtype=np.uint32).tolist())
        self.out.append(_reset_reply(m, self.model_id))


def make_model(kind: str, store: MapStore, out: list, staleness: int = 0, model_id: int = 0):
    if kind == "ssp":
        return SSP(model_id, store, staleness, out)
    if kind == "bsp":
        return BSP(model_id, store, out)
    if kind == "asp":
        return ASP(model_id, store, out)
    raise ValueError(kind)


def dispatch(model, m: Msg):
    """server_thread.cpp:29-46: one model call per message, by flag."""
    if m.flag == K_CLOCK:
        model.clock(m)
    elif m.flag == K_ADD:
        model.add(m)
    elif m.flag == K_GET:
        model.get(m)
    elif m.flag == K_RESET:
        model.reset(m)


# --------------------------------------------------------------------- traces
_HDR = struct.Struct("<ibiiiI")


def read_trace(path: str):
    """Yield ('I'|'O', server, Msg) and ('F', server, np.ndarray[f64])."""
    with open(path, "rb") as f:
        buf = f.read()
    p, n = 0, len(buf)
    while p < n:
        kind = chr(buf[p])
        p += 1
        if kind == "F":
            s, cnt = struct.unpack_from("<iQ", buf, p)
            p += 12
            v = np.frombuffer(buf, dtype=np.float64, count=cnt, offset=p)
            p += 8 * cnt
            yield kind, s, v
            continue
        if kind not in "IO":
            raise ValueError(f"bad trace record kind {kind!r} at byte {p - 1}")
        s, flag, snd, rcv, mid, nd = _HDR.unpack_from(buf, p)
        p += _HDR.size
        data = []
        for _ in range(nd):
            (ln,) = struct.unpack_from("<Q", buf, p)
            p += 8
            data.append(bytes(buf[p:p + ln]))
            p += ln
        yield kind, s, Msg(flag, snd, rcv, mid, data)


def check_trace(path: str, kind: str, staleness: int, ranges, dtype=np.float64) -> dict:
    """Replay the trace's arrivals through the models above; every reply the
    trace records must equal the one produced here, and every shard's final
    contents the dict store's.  Returns counts; raises AssertionError at the
    first difference."""
    n_srv = len(ranges)
    outs = [[] for _ in range(n_srv)]
    stores = [MapStore(dtype) for _ in range(n_srv)]
    models = [make_model(kind, stores[s], outs[s], staleness) for s in range(n_srv)]
    pending: Optional[List[Msg]] = None
    pending_srv = -1
    n_in = n_out = n_final = n_echo = 0

    def drain():
        assert not pending, f"server {pending_srv}: {len(pending)} expected replies not in the trace: {pending[:2]}"

    for rec_kind, s, x in read_trace(path):
        if rec_kind == "I":
            drain()
            outs[s].clear()
            dispatch(models[s], x)
            pending, pending_srv = list(outs[s]), s
            n_in += 1
        elif rec_kind == "O":
            assert s == pending_srv and pending, f"trace reply #{n_out} (server {s}) was not produced: {x}"
            want = pending.pop(0)
            assert x.key() == want.key(), f"reply #{n_out} from server {s} differs: trace {x} vs restatement {want}"
            if x.flag == K_GET and len(x.data) == 1:
                n_echo += 1
            n_out += 1
        else:
            drain()
            pending = None
            lo, hi = ranges[s]
            st = stores[s]
            ref = np.array([np.frombuffer(st.kv.get(k, st.zero), dtype=dtype)[0] for k in range(lo, hi)],
                           dtype=dtype) if hi - lo <= 4096 else _dense(st, lo, hi, dtype)
            assert x.shape == ref.shape and x.tobytes() == ref.tobytes(), f"final contents of server {s} differ"
            n_final += 1
    drain()
    assert n_final == n_srv, f"{n_final} final records for {n_srv} servers"
    return {"inputs": n_in, "replies": n_out, "echoes": n_echo, "servers": n_final}


def _dense(st: MapStore, lo: int, hi: int, dtype) -> np.ndarray:
    out = np.zeros(hi - lo, dtype=dtype)
    for k, v in st.kv.items():
        if lo <= k < hi:
            out[k - lo] = np.frombuffer(v, dtype=dtype)[0]
    return out
