"""bench.py — device-resident KV Add+Get throughput (BASELINE.json metric).

One step = one pass of the hot path over one push set and one pull set: a
grouped Add of the step's push batches, then a grouped Get of windows the push
did NOT touch (zero push/pull overlap, config.push_pull_overlap_keys = 0;
round 4).  Consecutive steps rotate over R window sets (--sets, default 16 at
N = 1 and 64 at N > 1; set r drawn with seed set_seed(r), set 0 being the
config's own seed).  The
round-2 form (the Get pulls the windows it just pushed, Infinity-Cache warm)
is kept as extra.cache_warm_step.  Inputs are resident in HBM before timing.

  N = 1: configs[1] (cfg 2) — 1e8-key float shard, J x 1M contiguous-key
         windows at uniform 1M-aligned bases (seed 42 for set 0), vals U(-1,1),
         assign mode; the pull is every window slot of the shard's 100 that the
         push set left free (~52), in a seeded order.  The 1e8-key shard is
         400 MB against the 256 MB Infinity Cache, so part of the array stays
         cached across steps whatever the step does: roofline.cold runs the same
         step on a 1e9-key shard (4 GB, cfg 4's whole key space; a window
         recurs every ~8 steps), where HBM serves every byte.
  N > 1: configs[3] (cfg 4) — 1e9 keys range-partitioned over N GPUs (one
         shard per rank, base/range_partition_manager.hpp's map).  J = 64
         producer streams; stream s pushes a contiguous 1M window at a uniformly
         random base in [0, 1e9 - 1M] (seed 1000 + s for set 0), which the range
         map slices — a window straddling a boundary splits in two.  The pull
         is J windows at random bases meeting no pushed window and no other
         pulled one, sliced the same way.  Each rank applies the slices routed
         to it, in producer order, as one grouped Add (the server's grouped
         flush), and pulls likewise.  The total work per step is fixed:
         "scaling": "strong".  The weak-scaled form (64 windows inside every
         rank's own range) is extra.weak_scaled.  No collective on the data
         path; torch.distributed (RCCL) only for the barrier and the max-time /
         sum-bytes reductions.

Bytes per step (counting what the step must move):
  Add (assign)  n*4 keys + u*V values + u*V parameter writes, u = distinct keys
                pushed (only the last push of a key needs its value read: a
                window shadowed by a later one in the step costs its keys only)
  Get           q*(4+2V) (key read + parameter read + value write)

Prints ONE JSON line on rank 0 with roofline (per-kernel rates from HIP events
on the launch stream, the dominant kernel's as `frac`, and the cold form's) and
cpu_baseline (the oracle restatement of the reference storages timed on this
host by rank 0: one thread with one storage at N = 1, beside 8 server threads
with 8 storages; at N > 1 the 8-thread sample is the value).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident KV Add+Get GB/s (grad+param bytes) at 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: HBM3E 8.0 TB/s spec
V = 4  # f32 values


def step_bytes(n_push, u_push, n_pull, vb=V):
    """Algorithmic bytes of one step's Add and Get (module docstring)."""
    add = n_push * 4 + 2 * u_push * vb
    get = n_pull * (4 + 2 * vb)
    return add, get


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batches", type=int, default=64, help="push batches (N=1) / producer streams (N>1) per step")
    p.add_argument("--batch-keys", type=int, default=1_000_000)
    p.add_argument("--sets", type=int, default=None,
                   help="window sets rotated over the steps (producers push new windows every step); default 16 "
                        "at N = 1, 64 at N > 1, where each set is a fresh random draw of the 64 producer windows "
                        "and more draws bring the ranks' totals over the timed steps to what an endless stream "
                        "of draws gives them (the largest rank share over the mean at N = 8: 1.078 with 16 sets, "
                        "1.027 with 64)"),
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-extra", action="store_true", help="skip the side measurements (e2e, f64, accumulate)")
    p.add_argument("--no-zipf", action="store_true", help="skip the cfg-3 sparse (Zipf) measurement")
    p.add_argument("--no-cold", action="store_true", help="skip the cold (HBM-served) form on a 1e9-key shard")
    p.add_argument("--cold-only", action="store_true",
                   help="run only the cold form (N = 1) and print its record (rocprof summaries of that form)")
    p.add_argument("--cold-keys", type=float, default=1e9, help="shard size of the cold form")
    p.add_argument("--cpu-batches", type=int, default=64,
                   help="1M-key windows in the 1-thread CPU baseline sample (~10 s)")
    p.add_argument("--vector-sizes", default="100000,200000,300000",
                   help="VectorStorage restatement sample sizes (a*n^2 fit to 1e6)")
    p.add_argument("--vector-only", action="store_true",
                   help="time only the VectorStorage restatement at --vector-sizes (no GPU; e.g. the one "
                        "measured 1e6-key run of config 1) and print its JSON")
    return p.parse_args(argv)


def default_sets(sets, world):
    """Window sets rotated over the steps: --sets, or 16 at N = 1 and 64 at
    N > 1 (each a fresh cfg-4 draw; with 64 the largest of 8 ranks' totals is
    1.027 of the mean, with 16 1.078); at least 2."""
    return max(2, sets if sets is not None else (16 if world == 1 else 64))


def dist_init(args):
    """One process per GPU (torchrun).  RCCL ("nccl") carries only the barrier and
    the scalar reductions.  Rehearsal knobs for a 1-GPU box (never used by the
    driver): PSKV_BENCH_BACKEND=gloo and PSKV_BENCH_SHARE_GPU=1 put every rank on
    cuda:0 and synchronise over gloo (tests/test_dist_gpu.py)."""
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("PSKV_BENCH_SHARE_GPU") == "1":
        local = 0
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        backend = os.environ.get("PSKV_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    return rank, world, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def in_turns(world, fn):
    """Run fn() on every rank; in the shared-device rehearsal
    (PSKV_BENCH_SHARE_GPU=1, several ranks on ONE GPU, never the driver's
    run) one rank at a time.  Heavy torch setup (the cfg-3 Zipf draw over a
    1e8-key CDF, torch.unique) issued by several processes at once on one
    device was measured to stall for minutes, pskv code or not (DESIGN.md §8,
    tools/proc_share_probe.py); one at a time it takes ~0.2 s a rank."""
    if world == 1 or os.environ.get("PSKV_BENCH_SHARE_GPU") != "1":
        return fn()
    import torch
    import torch.distributed as dist

    out = None
    for r in range(world):
        if r == dist.get_rank():
            out = fn()
            torch.cuda.synchronize()
        dist.barrier()
    return out


def _reduce_device(dev):
    import torch.distributed as dist

    return dev if dist.get_backend() == "nccl" else "cpu"


def max_over_ranks(x, world, dev):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64, device=_reduce_device(dev))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, world, dev):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64, device=_reduce_device(dev))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


# ------------------------------------------------------------------ planning


def plan_rank(rank, world, J, B, r=0, weak=False, bases=None, space=None):
    """Key range and push slices (window set r) of one rank — pure host logic,
    tested on CPU (tests/test_oracle.py, tests/test_dist.py with gloo).

    Returns (key_space, lo, hi, slices, bases): slices = [(window w, first key,
    length)] routed to this rank, in producer order; bases = the set's window
    bases (every rank's).  N = 1: cfg 2 (or, with `space`, the same draw on a
    shard of `space` keys: the cold form).  N > 1: cfg 4 (global producer
    windows through the range map), or with weak=True the weak-scaled form (J
    aligned windows inside this rank's range).  `bases` (N > 1) replaces the
    drawn producer windows (tests)."""
    from parameter_server_amd import workload

    seed = workload.set_seed(r, world)
    if world == 1:
        key_space = space or 100_000_000
        lo, hi = 0, key_space
        bases = workload.dense_bases(J, key_space, B, seed=seed)
        slices = [(j, int(b), B) for j, b in enumerate(bases)]
        return key_space, lo, hi, slices, bases
    key_space = 1_000_000_000
    ranges = workload.rank_ranges(key_space, world)
    lo, hi = ranges[rank]
    if weak:
        bases = workload.rank_windows(rank, world, key_space, J, B, seed=seed)
        routed = workload.route_windows(bases, B, ranges)
        # every window of this rank's producers lands on this rank, whole
        assert all(len(routed[q]) == 0 for q in range(world) if q != rank)
        assert len(routed[rank]) == J and all(n == B for _, _, n in routed[rank])
    else:
        if bases is None:
            bases = workload.global_windows(J, key_space, B, seed=seed)
        routed = workload.route_windows(bases, B, ranges)
    slices = [(w, int(bases[w]) + off, n) for w, off, n in routed[rank]]
    return key_space, lo, hi, slices, bases


def plan_pull(rank, world, J, B, r, push_bases, weak=False, space=None, n_pull=None):
    """Pull slices of window set r's step: windows DISJOINT from the step's push
    set (zero push/pull overlap), each pulled once.  N = 1 and the weak-scaled
    form: every aligned window slot the push set left free (cfg 2: ~52 of the
    shard's 100), in a seeded order, at most n_pull of them.  N > 1 (cfg 4): J
    windows at uniformly random bases that meet no pushed window and no other
    pulled one, sliced by the range map like the pushes.  Returns (slices,
    bases) as plan_rank."""
    from parameter_server_amd import workload

    seed = workload.set_seed(r, world) + 7
    if world == 1:
        key_space = space or 100_000_000
        bases = workload.complement_windows(push_bases, 0, key_space, B, seed=seed, n_max=n_pull)
        return [(j, int(b), B) for j, b in enumerate(bases)], bases
    key_space = 1_000_000_000
    ranges = workload.rank_ranges(key_space, world)
    if weak:
        lo, hi = ranges[rank]
        bases = workload.complement_windows(push_bases, lo, hi, B, seed=seed + 1000 * rank, n_max=J)
        return [(j, int(b), B) for j, b in enumerate(bases)], bases
    bases = workload.disjoint_windows(push_bases, J, key_space, B, seed=seed * 100)
    routed = workload.route_windows(bases, B, ranges)
    return [(w, int(bases[w]) + off, n) for w, off, n in routed[rank]], bases


def window_vals(w, r, B, dev, rank=0, weak=False, dtype=None):
    """The value stream of producer w in window set r: U(-1, 1), seed
    42 + w + 100000 r (+ 1000 rank in the weak-scaled form, whose producers
    are per rank).  Every rank draws a window's values alike, so a straddling
    window's two slices carry its values."""
    import torch

    g = torch.Generator(device=dev)
    g.manual_seed(42 + w + 100_000 * r + (1000 * rank if weak else 0))
    return torch.rand(B, generator=g, device=dev, dtype=dtype or torch.float32) * 2 - 1


def make_set(rank, world, J, B, dev, r=0, weak=False, dtype=None, bases=None, space=None, n_pull=None):
    """Window set r of this rank in HBM: the push slices with their (keys, vals)
    batches and distinct-key count, and the step's pull slices with their keys."""
    import torch

    from parameter_server_amd import workload

    _, lo, hi, slices, bases = plan_rank(rank, world, J, B, r, weak, bases, space)
    batches = []
    for w, first, n in slices:
        keys = torch.arange(first, first + n, dtype=torch.int64, device=dev).to(torch.int32)
        off = first - int(bases[w])
        vals = window_vals(w, r, B, dev, rank, weak, dtype)[off:off + n].clone()  # own, aligned buffer
        batches.append((keys, vals))
    pull, pull_bases = plan_pull(rank, world, J, B, r, bases, weak, space, n_pull)
    pull_keys = [torch.arange(first, first + n, dtype=torch.int64, device=dev).to(torch.int32)
                 for _, first, n in pull]
    u = workload.interval_union([(f, n) for _, f, n in slices])
    return {"slices": slices, "batches": batches, "u": u, "r": r, "bases": bases,
            "pull": pull, "pull_keys": pull_keys, "pull_bases": pull_bases}


def overlap_keys(s):
    """Keys a set's pull shares with its own push (0 by construction)."""
    from parameter_server_amd import workload

    push = workload.interval_union([(f, n) for _, f, n in s["slices"]])
    pull = workload.interval_union([(f, n) for _, f, n in s["pull"]])
    both = workload.interval_union([(f, n) for _, f, n in s["slices"] + s["pull"]])
    return push + pull - both


class Form:
    """One way of running the step over R window sets on a shard: step i pushes
    set i % R, then pulls set i % R's pull windows (pull="disjoint": the
    headline, no pulled key pushed in the step) or the windows it just pushed
    (pull="same": the cache-warm round-2 form)."""

    def __init__(self, shard, sets, dev, vb=V, sorted_hint=True, pull="disjoint"):
        import torch

        self.shard, self.sets, self.R, self.vb = shard, sets, len(sets), vb
        self.hint, self.mode = sorted_hint, pull
        tdt = {4: torch.float32, 8: torch.float64}[vb]
        self.pull_slices = [s["pull"] if pull == "disjoint" else s["slices"] for s in sets]
        pull_keys = [s["pull_keys"] if pull == "disjoint" else [k for k, _ in s["batches"]] for s in sets]
        self.outs = [[torch.empty(k.numel(), dtype=tdt, device=dev) for k in pk] for pk in pull_keys]
        self.adds = [shard.prepare(s["batches"]) for s in sets]
        self.gets = [shard.prepare(list(zip(pk, outs)), is_get=True) for pk, outs in zip(pull_keys, self.outs)]
        self.add_b = [step_bytes(sum(n for _, _, n in s["slices"]), s["u"], 0, vb)[0] for s in sets]
        self.get_b = [step_bytes(0, 0, sum(n for _, _, n in p), vb)[1] for p in self.pull_slices]

    def step(self, i):
        # the grouped Add then the grouped Get, in one call
        # (pskv_add_get_grouped: the K2g launch, then K1 carrying its conditional replay -- K1r)
        self.shard.add_get_grouped(self.adds[i % self.R], self.gets[i % self.R], sorted_hint=self.hint)

    def bytes(self, steps):
        """(add bytes, get bytes) of steps 0..steps-1."""
        a = sum(self.add_b[i % self.R] for i in range(steps))
        g = sum(self.get_b[i % self.R] for i in range(steps))
        return a, g

    def touched(self, i):
        """Distinct parameter bytes step i reads or writes (push set ∪ pull set)."""
        from parameter_server_amd import workload

        iv = [(f, n) for _, f, n in self.sets[i % self.R]["slices"] + self.pull_slices[i % self.R]]
        return workload.interval_union(iv) * self.vb

    def self_check(self, lo, hi, dev, rotations=1):
        """From a cleared shard, run `rotations` rotations and compare every pull
        with a torch model of the shard (sequential last-write-wins slice
        assigns, map_storage.hpp:22-23; never-written keys read 0,
        map_storage.hpp:33-37) — the benchmarked state is the reference's."""
        import torch

        self.shard.clear()
        ref = torch.zeros(hi - lo, dtype={4: torch.float32, 8: torch.float64}[self.vb], device=dev)
        for i in range(self.R * rotations):
            t = i % self.R
            for (_, first, n), (_, v) in zip(self.sets[t]["slices"], self.sets[t]["batches"]):
                ref[first - lo:first - lo + n] = v
            self.step(i)
            torch.cuda.synchronize()
            for (_, first, n), o in zip(self.pull_slices[t], self.outs[t]):
                if not torch.equal(o, ref[first - lo:first - lo + n]):
                    raise AssertionError(f"bench self-check failed: step {i}, pull of set {t}, key {first}")
        del ref


def timed(form, steps, world, dev):
    """Exactly `steps` steps bracketed by barrier + synchronize on both sides.
    Returns (max over ranks of this rank's elapsed time, own elapsed)."""
    import torch

    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        form.step(i)
    torch.cuda.synchronize()
    own = time.perf_counter() - t0
    barrier(world)
    return max_over_ranks(own, world, dev), own


def evented(form, steps, world, dev):
    """The same steps again with HIP events around the streaming kernels on
    their launch stream: per-kernel launches and average duration, and the
    algorithmic bytes per launch (this rank's)."""
    import torch

    from parameter_server_amd import _lib

    sh = form.shard
    sh.reset_timing()
    sh.set_timing(True, kernels=[_lib.PSKV_K_GATHER, _lib.PSKV_K_ASSIGN_TILES])
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    for i in range(steps):
        form.step(i)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    sh.set_timing(False)
    add_b, get_b = form.bytes(steps)
    ktimes = {}
    for k, name in _lib.KERNEL_NAMES.items():
        t = sh.kernel_time(k)
        if t["launches"]:
            b = get_b if k == _lib.PSKV_K_GATHER else add_b
            rec = {"launches": t["launches"], "avg_ms": t["total_ms"] / t["launches"],
                   "keys_per_launch": t["elements"] / t["launches"],
                   "algorithmic_bytes": b / t["launches"]}
            rec["GB/s"] = rec["algorithmic_bytes"] / (rec["avg_ms"] / 1e3) / 1e9
            ktimes[name] = rec
    sh.sync()
    return ktimes, max_over_ranks(t3 - t2, world, dev)


def run_form(form, steps, warmup, world, dev):
    """Warm up, time, and sum the bytes over ranks: the aggregate GB/s of a form."""
    import torch

    for i in range(warmup):
        form.step(i)
    torch.cuda.synchronize()
    elapsed, own = timed(form, steps, world, dev)
    a, g = form.bytes(steps)
    total = sum_over_ranks(float(a + g), world, dev)
    return {"GB/s": total / elapsed / 1e9, "ms_per_step": elapsed / steps * 1e3, "elapsed": elapsed,
            "own_GB/s": (a + g) / own / 1e9, "bytes": total}


# ------------------------------------------------------------ CPU baseline


def cpu_baseline(bases, B, n_batches, vector_sizes, servers=1):
    """The oracle (C++ restatement of server/map_storage.hpp) on a bounded
    sample of the same workload: one thread with one storage, and 8 server
    threads with one storage each (the reference runs one storage
    per server thread); VectorStorage (cfg 1) at several sizes with the a*n^2
    fit extrapolated to config 1's 1e6 keys (skipped with no sizes).
    servers = 8 (the N > 1 line) reports the 8-thread sample as the baseline
    value, the 1-thread one beside it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg

    oracle.build()
    rng = np.random.default_rng(42)
    m = oracle.MapStorageRef(np.float32)
    ks = [np.arange(int(b), int(b) + B, dtype=np.uint32) for b in bases[:n_batches]]
    vs = [(rng.random(B, dtype=np.float32) * 2 - 1) for _ in ks]
    t0 = time.perf_counter()
    for k, v in zip(ks, vs):
        m.add(k, v)
    for k in ks:
        m.get(k)
    t_map = time.perf_counter() - t0
    m.close()
    vector = vector_storage_fit(oracle, vector_sizes) if vector_sizes else None
    # 8 server threads with 8 storages (the reference runs one
    # storage per server thread); ctypes drops the GIL inside the oracle calls
    import threading

    T, mt_batches = 8, min(12, len(ks))  # 8 threads x 12 windows each (~3 s)
    shards = [oracle.MapStorageRef(np.float32) for _ in range(T)]
    work = [[(k, v) for k, v in zip(ks[:mt_batches], vs[:mt_batches])] for _ in range(T)]
    barrier_t = threading.Barrier(T + 1)

    def serve(t):
        barrier_t.wait()
        for k, v in work[t]:
            shards[t].add(k, v)
        for k, _ in work[t]:
            shards[t].get(k)

    th = [threading.Thread(target=serve, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    barrier_t.wait()
    t0 = time.perf_counter()
    for x in th:
        x.join()
    t_mt = time.perf_counter() - t0
    # same byte accounting as the GPU value (u = distinct keys pushed; the Get
    # of the same windows)
    u = B * len(set(int(b) for b in bases[:n_batches]))
    add_b, get_b = step_bytes(B * len(ks), u, B * len(ks))
    u_mt = B * len(set(int(b) for b in bases[:mt_batches]))
    for sh in shards:
        sh.close()
    one = {
        "value": (add_b + get_b) / t_map / 1e9,
        "unit": "GB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"MapStorage restatement (std::map, 1 thread), {len(ks)} x {B} contiguous float keys of the "
                  f"same workload (window set 0), Add then Get, {t_map:.2f} s",
    }
    eight = {
        "value": sum(step_bytes(B * mt_batches, u_mt, B * mt_batches)) * T / t_mt / 1e9, "unit": "GB/s",
        "cores": T, "kind": "port", "seconds": t_mt,
        "sample": f"{T} server threads x one MapStorage restatement each (the reference's one storage per server "
                  f"thread), {mt_batches} x {B} contiguous float keys of window set 0 per thread, Add then Get, "
                  f"{t_mt:.2f} s"}
    if servers == 1:
        rec = dict(one, eight_threads=eight)
    else:
        rec = dict(eight, one_thread=one)
    if vector is not None:
        rec["vector_storage"] = vector
    rec["host_cpu"] = _cpu_model()
    return rec


def vector_storage_fit(oracle, sizes):
    """Config 1 (VectorStorage Add+Get of n contiguous float keys,
    server/vector_storage_test.cpp's shape) timed at several n; Get is the
    O(stored x queried) scan of vector_storage.hpp:34-43, so t(n) = a * n^2
    (least squares, no lower-order terms: a quadratic scan has no intercept and
    no negative linear part -- round 4's full quadratic fit had both and
    extrapolated 288 s where the measured run took 215 s) is extrapolated to
    the config's 1e6 keys.  The one measured 1e6 run is carried beside it."""
    import threading

    pts = []
    for n in sizes:
        done = threading.Event()
        t_start = time.perf_counter()

        def beat(n=n, done=done, t_start=t_start):  # a long scan still shows progress
            while not done.wait(30.0):
                print(f"vector_storage n={n}: {time.perf_counter() - t_start:.0f} s", file=sys.stderr, flush=True)

        hb = threading.Thread(target=beat, daemon=True)
        hb.start()
        vec = oracle.VectorStorageRef(np.float32)
        k = np.arange(n, dtype=np.uint32)
        v = (0.5 * k).astype(np.float32)
        t0 = time.perf_counter()
        vec.add(k, v)
        got = vec.get(k)
        t = time.perf_counter() - t0
        done.set()
        hb.join()
        assert np.array_equal(got, v)
        pts.append((n, t))
        vec.close()
    ns = np.array([p[0] for p in pts], dtype=np.float64)
    ts = np.array([p[1] for p in pts], dtype=np.float64)
    a = float(np.sum(ts * ns ** 2) / np.sum(ns ** 4))
    t1e6 = a * 1e12
    return {"samples": [{"n": int(n), "seconds": t, "GB/s": 24.0 * n / t / 1e9} for n, t in pts],
            "fit_seconds": {"a_n2": a, "form": "t = a * n^2, least squares"},
            "extrapolated_1e6_seconds": t1e6,
            "value": 24.0 * 1e6 / t1e6 / 1e9, "unit": "GB/s",
            "sample": "VectorStorage restatement (append + O(stored x queried) last-match scan), config 1's "
                      "contiguous float keys at the sizes listed, 1 thread; value = the a*n^2 fit at 1e6 keys"}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_pmc(kernel_substr, config, name="pmc_latest.json"):
    """HBM traffic per dispatch from the committed rocprofv3 --pmc summary, if it
    was collected on this same bench configuration (profiles/pmc_latest.json:
    the headline; pmc_cold_latest.json: the cold form)."""
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    if d.get("config") != config:
        return None, None
    for name, rec in d.get("kernels", {}).items():
        if kernel_substr in name and rec.get("hbm_bytes_per_dispatch"):
            return rec["hbm_bytes_per_dispatch"], d.get("source", path)
    return None, None


def _zipf_cpu_sample(zb, B):
    """The oracle's MapStorage restatement (1 thread) on the first cfg-3 Zipf
    batches, same byte accounting as the GPU number (the baseline for cfg 3)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU baseline leg

    ks = [k.cpu().numpy().view(np.uint32) for k, _ in zb]
    vs = [v.cpu().numpy() for _, v in zb]
    m = oracle.MapStorageRef(np.float32)
    t0 = time.perf_counter()
    for k, v in zip(ks, vs):
        m.add(k, v)
    for k in ks:
        m.get(k)
    t = time.perf_counter() - t0
    u = int(np.unique(np.concatenate(ks)).size)
    add_b, get_b = step_bytes(len(ks) * B, u, len(ks) * B)
    return {"GB/s": (add_b + get_b) / t / 1e9, "seconds": t, "cores": 1, "kind": "port",
            "sample": f"{len(ks)} x {B} Zipf keys of the same workload, Add then Get"}


# --------------------------------------------------------- side measurements


def side_measurements(dev, B):
    """Secondary numbers (same JSON line, under "extra"): cfg 3 Zipf in
    accumulate mode, cfg-2 windows in accumulate mode (Add only), and the
    end-to-end rate from host buffers."""
    import torch

    import parameter_server_amd as ps
    from parameter_server_amd import _lib, workload

    out = {}
    stream = torch.cuda.current_stream()
    # cfg 3 pushes: Zipf(0.99) over 1e8 keys, unsorted, 8 x 1M
    space, J = 100_000_000, 8
    zb = workload.zipf_batches(J, space, batch=B, device=dev)
    u_all = int(torch.unique(torch.cat([k for k, _ in zb])).numel())
    reps = 5
    # cfg 3 in accumulate mode (the north star's LDS segmented-sum path): K5,
    # per-super-chunk LDS sums, key buckets, one owner workgroup per bucket
    with ps.Shard(0, space, np.float32, mode="accumulate") as sh:
        sh.set_stream(stream.cuda_stream)
        for _ in range(2):
            sh.add_grouped(zb)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            sh.add_grouped(zb)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        sh.set_stream(None)
    acc_b = J * B * (4 + V) + 2 * u_all * V
    out["zipf_accumulate_add"] = {"workload": "cfg 3 pushes (8 x 1M Zipf(0.99), unsorted), accumulate mode "
                                              "(K5: LDS super-chunk sums + key buckets, no global atomics)",
                                  "GB/s": acc_b * reps / dt / 1e9, "ms_per_call": dt / reps * 1e3}
    del zb
    # cfg 2 windows in accumulate mode (the north star's scatter-accumulate):
    # sorted hint -> K6 density proof + K7 one RMW per key (sums in call order)
    J = 64
    db = workload.dense_batches(J, space, batch=B, device=dev)
    with ps.Shard(0, space, np.float32, mode="accumulate") as sh:
        sh.set_stream(stream.cuda_stream)
        adds = sh.prepare(db)
        for _ in range(2):
            sh.add_grouped(adds, sorted_hint=True)
        torch.cuda.synchronize()
        reps = 10
        t0 = time.perf_counter()
        for _ in range(reps):
            sh.add_grouped(adds, sorted_hint=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        sh.set_timing(True, kernels=[_lib.PSKV_K_DENSE_CHECK, _lib.PSKV_K_ACC_DENSE])
        for _ in range(reps):
            sh.add_grouped(adds, sorted_hint=True)
        torch.cuda.synchronize()
        kt = {_lib.KERNEL_NAMES[k]: sh.kernel_time(k) for k in (_lib.PSKV_K_DENSE_CHECK, _lib.PSKV_K_ACC_DENSE)}
        sh.set_timing(False)
        sh.set_stream(None)
    # accumulate Add bytes: n*(4+V) input (every value is summed) + 2*u*V
    # parameter read-modify-write
    u_acc = len(set(int(b) for b in workload.dense_bases(J, space, B))) * B
    acc_b = J * B * (4 + V) + 2 * u_acc * V
    k_ms = {n: t["total_ms"] / max(1, t["launches"]) for n, t in kt.items()}
    out["accumulate_dense_add"] = {
        "workload": f"cfg 2 windows, {J} x 1M contiguous float pushes, accumulate mode "
                    "(sorted hint -> K6 density proof + K7 one RMW per key, no atomics)",
        "GB/s": acc_b * reps / dt / 1e9, "ms_per_call": dt / reps * 1e3,
        "kernels_avg_ms": k_ms,
        "k_acc_dense_GB/s": (J * B * V + 2 * u_acc * V) / (k_ms["k_acc_dense"] * 1e-3) / 1e9,
        "k_dense_check_GB/s": (J * B * 4) / (k_ms["k_dense_check"] * 1e-3) / 1e9}
    del db
    out.update(e2e_measurements(B, space))
    return out


def e2e_measurements(B, space):
    """End to end: keys/vals start in host memory (the zmq frames), outputs
    return to host.  Algorithmic GB/s as the device figure, and the PCIe bytes
    per second the same calls moved (Add: keys + values H2D; Get: keys H2D,
    values D2H)."""
    import torch

    import parameter_server_amd as ps
    from parameter_server_amd import workload

    out = {}
    rng = np.random.default_rng(0)
    J = 8
    hk = [np.arange(b, b + B, dtype=np.uint32) for b in workload.dense_bases(J, space, B)]
    hv = [rng.random(B, dtype=np.float32) for _ in hk]
    ho = [np.empty(B, np.float32) for _ in hk]
    last = {int(k[0]): j for j, k in enumerate(hk)}  # repeated windows: the later push wins
    u = len(last) * B
    add_b, get_b = step_bytes(J * B, u, J * B)
    pcie = J * B * (4 + V) + J * B * (4 + V)  # Add H2D keys+vals, Get H2D keys + D2H values

    def measure(name, what, k, v, o, frame=False):
        reps = 3
        with ps.Shard(0, space, np.float32) as sh:
            sh.add_grouped(list(zip(k, v)), frame=frame)
            sh.get_grouped(list(zip(k, o)), frame=frame)
            t0 = time.perf_counter()
            for _ in range(reps):
                sh.add_grouped(list(zip(k, v)), frame=frame)
                sh.get_grouped(list(zip(k, o)), frame=frame)
            sh.sync()
            dt = time.perf_counter() - t0
        assert all(np.array_equal(x, hv[last[int(kk[0])]]) for x, kk in zip(o, k))
        out[name] = {"workload": what, "GB/s": (add_b + get_b) * reps / dt / 1e9,
                     "pcie_GB/s": pcie * reps / dt / 1e9, "ms_per_step": dt / reps * 1e3}

    measure("e2e_host_buffers", "8 x 1M contiguous float keys from pageable host memory, Add then Get "
                                "(H2D + kernels + D2H, host sortedness check included)", hk, hv, ho)

    def pin(a):
        t = torch.from_numpy(a.view(np.int32) if a.dtype == np.uint32 else a).pin_memory()
        return t.numpy().view(a.dtype)

    measure("e2e_pinned_buffers", "as e2e_host_buffers, from page-locked host memory (direct DMA)",
            [pin(k) for k in hk], [pin(v) for v in hv], [pin(o) for o in ho])
    frames = [ps.HostFrame(B * 4) for _ in range(3 * J)]
    fk = [f.array(np.uint32, B) for f in frames[:J]]
    fv = [f.array(np.float32, B) for f in frames[J:2 * J]]
    fo = [f.array(np.float32, B) for f in frames[2 * J:]]
    for a, b in zip(fk + fv, hk + hv):
        a[:] = b
    measure("e2e_frame_buffers", "as e2e_host_buffers, from pskv_host_alloc frames under PSKV_HOST_FRAME "
                                 "(borrowed: Adds return once queued)", fk, fv, fo, frame=True)
    for f in frames:
        f.free()
    return out


def zipf_sparse(rank, world, dev, lo, hi, B, steps, J=8):
    """cfg 3 on every rank: J x 1M unsorted Zipf(0.99) pushes then the same
    pulls per step, assign mode, over this rank's range shard (N = 1: the 1e8-key
    cfg-3 shard; N > 1: the rank's 1e9/N range, its own key permutation, so the
    sparse path is weak-scaled like the dense one).  Barrier + synchronize around
    exactly `steps` steps, max over ranks; bytes as SURVEY §8d with u = distinct
    keys pushed in the step.  The K5 (Add) and K1 (Get) durations come from an
    evented second pass."""
    import torch

    import parameter_server_amd as ps
    from parameter_server_amd import _lib, workload

    space = hi - lo

    def draw():
        zb_ = workload.zipf_batches(J, space, batch=B, device=dev, perm_seed=7 + rank, seed=42 + 1000 * rank,
                                    lo=lo)
        return zb_, int(torch.unique(zb_[0][0]).numel()), int(torch.unique(torch.cat([k for k, _ in zb_])).numel())

    zb, uniq, u_all = in_turns(world, draw)
    zo = [torch.empty_like(v) for _, v in zb]
    progress("cfg 3: batches built, distinct keys counted")
    with ps.Shard(lo, hi, np.float32, device=dev.index) as sh:
        progress("cfg 3: shard created")
        sh.set_stream(torch.cuda.current_stream().cuda_stream)
        adds = sh.prepare(zb)
        gets = sh.prepare([(k, o) for (k, _), o in zip(zb, zo)], is_get=True)
        for i in range(2):
            sh.add_grouped(adds)
            sh.sync()  # bounded (SYNC_TIMEOUT_MS): a K5 that never completes is reported, not waited on
            if i == 0:
                progress("cfg 3: first Add (K5) complete")
            sh.get_grouped(gets)
            sh.sync()
            if i == 0:
                progress("cfg 3: first Get (K1) complete")
        # self-check: every key in the tail of the LAST batch was last written
        # there (a later write would be later in that tail), so it reads its
        # last occurrence's value
        last = {}
        kk, vv = zb[-1][0].cpu().numpy(), zb[-1][1].cpu().numpy()
        last.update(zip(kk[-4096:].tolist(), vv[-4096:].tolist()))
        probe = torch.tensor(list(last), dtype=torch.int32, device=dev)
        progress("cfg 3: probe keys resident")
        got_t = sh.get(probe)
        sh.sync()
        got = got_t.cpu().numpy()
        assert np.array_equal(got, np.array([last[int(x)] for x in probe.cpu().numpy()], np.float32)), \
            "zipf self-check failed"
        progress("cfg 3: self-check done")
        barrier(world)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            sh.add_grouped(adds)
            sh.get_grouped(gets)
        torch.cuda.synchronize()
        t_own = time.perf_counter() - t0
        barrier(world)
        elapsed = max_over_ranks(t_own, world, dev)
        sh.set_timing(True, kernels=[_lib.PSKV_K_RADIX, _lib.PSKV_K_GATHER])
        for _ in range(steps):
            sh.add_grouped(adds)
            sh.get_grouped(gets)
        torch.cuda.synchronize()
        kt = {n: sh.kernel_time(k) for k, n in ((_lib.PSKV_K_RADIX, "k_rb_bin+k_rb_resolve (K5 Add)"),
                                                 (_lib.PSKV_K_GATHER, "k_gather (K1 Get)"))}
        sh.set_timing(False)
        sh.set_stream(None)
    add_b, get_b = step_bytes(J * B, u_all, J * B)
    own = (add_b + get_b) * steps
    total = sum_over_ranks(float(own), world, dev)
    value = total / elapsed / 1e9
    kernels = {}
    for n, t in kt.items():
        ms = t["total_ms"] / max(1, t["launches"])
        b = add_b if n.startswith("k_rb") else get_b
        kernels[n] = {"avg_ms": ms, "algorithmic_bytes": b, "GB/s": b / (ms * 1e-3) / 1e9,
                      "frac": b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
    progress("cfg 3: timed; random-access floor")
    floor = in_turns(world, lambda: random_access_floor(zb, lo, space, dev))
    if floor is not None:
        k5_ms = kernels["k_rb_bin+k_rb_resolve (K5 Add)"]["avg_ms"]
        k1_ms = kernels["k_gather (K1 Get)"]["avg_ms"]
        # the floor of each kernel: one random access per distinct key (the
        # same keys, each touched once, caches flushed) plus its streaming
        # bytes at the dense kernels' measured rate
        stream_gbs = 6500.0
        floor["K5_floor_ms"] = floor["scatter_ms"] + J * B * (4 + V) / stream_gbs / 1e6
        floor["K1_floor_ms"] = floor["gather_ms"] + J * B * (4 + V) / stream_gbs / 1e6
        floor["K5_frac_of_floor"] = floor["K5_floor_ms"] / k5_ms
        floor["K1_frac_of_floor"] = floor["K1_floor_ms"] / k1_ms
    return {
        "workload": f"cfg 3 sparse: {J} x {B} unsorted Zipf(0.99) pushes then the same pulls per step per GPU "
                    f"over a {space:.3g}-key range shard, assign mode (K5 key buckets + K1 gather)",
        "value": value, "unit": "GB/s", "n_gpus": world, "steps": steps, "ms_per_step": elapsed / steps * 1e3,
        "per_gpu": {"mean_GB/s": value / world, "min_GB/s": -max_over_ranks(-own / t_own / 1e9, world, dev),
                    "max_GB/s": max_over_ranks(own / t_own / 1e9, world, dev)},
        "roofline": {"bound": "hbm", "achieved": value / world, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": value / world / HBM_PEAK_GBS,
                     "note": "algorithmic bytes (SURVEY §8d, u = distinct keys) per GPU per second; "
                             "random single-value accesses fetch whole lines, so the line traffic is higher"},
        "kernels": kernels,
        "random_access_floor": floor,
        "unique_keys_per_batch": uniq, "distinct_keys_per_step": u_all,
        "bytes_per_step_per_gpu": add_b + get_b}, zb


def random_access_floor(zb, lo, space, dev, reps=5):
    """The random-access ceiling the cfg-3 kernels work against, measured on
    this box: the step's distinct keys, each touched ONCE in random order, by
    the gather / scatter kernels of tools/micro/random_access.hip (16 offsets
    per lane in flight) on a fresh float array of the shard's size, with L2
    and the 256 MB Infinity Cache flushed by a read of 1 GiB before every
    timed op.  A random single-value access costs a DRAM row activation and a
    64-byte sector (stores: a partial-line merge), so this rate -- not 8 TB/s
    -- bounds a key-at-a-time kernel; the K5 / K1 floors add their streaming
    bytes.  Measurement infrastructure, not the product (libpskv never calls
    it)."""
    import ctypes

    import torch

    path = os.path.join(ROOT, "tools", "micro", "librandom_access.so")
    if not os.path.exists(path):  # built by __graft_entry__.build(); a side figure, not the metric
        print(f"bench: {path} not built; zipf_sparse.random_access_floor skipped", file=sys.stderr)
        return None
    lib = ctypes.CDLL(path)
    keys = torch.unique(torch.cat([k for k, _ in zb]).to(torch.int64) - lo)
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    idx = keys[torch.randperm(keys.numel(), device=dev, generator=g)].to(torch.int32)
    u = idx.numel()
    assert int(idx.min()) >= 0 and int(idx.max()) < space
    arr = torch.zeros(space, dtype=torch.float32, device=dev)
    vals = torch.rand(u, device=dev, generator=g)
    out = torch.empty(u, dtype=torch.float32, device=dev)
    # a read-only sweep of 1 GiB evicts L2 and the Infinity Cache without
    # leaving dirty lines for the timed kernel to write back (a fill would)
    flush = torch.ones(1 << 28, dtype=torch.float32, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    res = {"gather_ms": [], "scatter_ms": []}
    for r in range(reps + 1):
        for name in ("gather_ms", "scatter_ms"):
            flush.sum()
            ev[0].record()
            if name == "gather_ms":
                rc = lib.ra_gather(ctypes.c_void_p(idx.data_ptr()), ctypes.c_uint32(u),
                                   ctypes.c_void_p(arr.data_ptr()), ctypes.c_void_p(out.data_ptr()), st)
            else:
                rc = lib.ra_scatter(ctypes.c_void_p(idx.data_ptr()), ctypes.c_uint32(u),
                                    ctypes.c_void_p(vals.data_ptr()), ctypes.c_void_p(arr.data_ptr()), st)
            ev[1].record()
            torch.cuda.synchronize()
            assert rc == 0, f"random_access {name}: hip error {rc}"
            if r:
                res[name].append(ev[0].elapsed_time(ev[1]))
    assert torch.equal(out, arr.index_select(0, idx.long())), "random_access gather check"
    del out, flush, arr
    rec = {"distinct_keys": u, "how": "tools/micro/random_access.hip gather / scatter of the step's distinct "
                                      "keys, each once, random order, caches flushed; median of %d" % reps}
    for name in ("gather_ms", "scatter_ms"):
        ms = float(np.median(res[name]))
        rec[name] = ms
        rec[name.replace("_ms", "_G_accesses/s")] = u / (ms * 1e-3) / 1e9
    return rec


def variant_f64(rank, world, J, B, dev, R, steps, lo, hi):
    """The headline step with 8-byte values (the reference apps' Val = double,
    app/logistic_regression.cpp): same windows, f64 shard, V = 8 bytes."""
    import torch

    import parameter_server_amd as ps

    sets = [make_set(rank, world, J, B, dev, r, dtype=torch.float64) for r in range(R)]
    with ps.Shard(lo, hi, np.float64, device=dev.index) as sh:
        sh.set_stream(torch.cuda.current_stream().cuda_stream)
        f = Form(sh, sets, dev, vb=8)
        f.self_check(lo, hi, dev)
        res = run_form(f, steps, 2, world, dev)
        sh.set_stream(None)
    return {"workload": f"the headline step with float64 values ({J} x {B} windows pushed, the free window slots "
                        "pulled, assign)",
            "GB/s": res["GB/s"], "ms_per_step": res["ms_per_step"]}


def variant_accumulate(rank, world, J, B, dev, sets, steps, lo, hi):
    """The headline step in ACCUMULATE mode (the north star's gradient push:
    param[k] += v, then the pull): K6 density proof + K7 one read-modify-write
    per key (sums in call order) + K1.  Bytes: Add n*(4+V) + 2*u*V (every value
    is summed, and the RMW), Get q*(4+2V).  A self-check compares one rotation
    with a torch model of the sequential sums first."""
    import torch

    import parameter_server_amd as ps

    with ps.Shard(lo, hi, np.float32, mode="accumulate", device=dev.index) as sh:
        sh.set_stream(torch.cuda.current_stream().cuda_stream)
        f = Form(sh, sets, dev)
        # accumulate bytes: every pushed value is read
        f.add_b = [sum(n for _, _, n in s["slices"]) * (4 + V) + 2 * s["u"] * V for s in sets]
        ref = torch.zeros(hi - lo, dtype=torch.float32, device=dev)
        for i in range(f.R):
            for (_, first, n), (_, v) in zip(sets[i]["slices"], sets[i]["batches"]):
                ref[first - lo:first - lo + n] += v
            f.step(i)
            torch.cuda.synchronize()
            for (_, first, n), o in zip(f.pull_slices[i], f.outs[i]):
                assert torch.equal(o, ref[first - lo:first - lo + n]), "accumulate self-check failed"
        del ref
        res = run_form(f, steps, 2, world, dev)
        sh.set_stream(None)
    return {"workload": f"the headline step in accumulate mode (gradient push +=, then pull of the free window "
                        f"slots), "
                        f"{J} x {B} windows (K6 + K7 + K1)",
            "GB/s": res["GB/s"], "ms_per_step": res["ms_per_step"]}


def kernel_fracs(ktimes):
    """Per-kernel fraction of the HBM peak (algorithmic bytes / avg duration)."""
    return {n: dict(k, frac=k["GB/s"] / HBM_PEAK_GBS) for n, k in ktimes.items()}


def cold_form(dev, J, B, R, steps, warmup, space, n_pulls):
    """The headline step on a shard of `space` keys (default 1e9 = cfg 4's whole
    key space: 4 GB of parameters against the 256 MB Infinity Cache): push set r
    = J windows at uniform 1M-aligned bases (seed set_seed(r)), pull = n_pulls[r]
    free window slots (as many as cfg 2's set r pulls).  With 1000 window slots
    a window recurs only every ~8 steps, after ~4 GB of other traffic, so both
    kernels are served by HBM — the rate a cold rank sees, and the roofline's
    cold figure.  N = 1 only (one process; the 1e9-key shard alone)."""
    import torch

    import parameter_server_amd as ps

    sets = []
    for r in range(R):
        sets.append(make_set(0, 1, J, B, dev, r, space=space, n_pull=n_pulls[r % len(n_pulls)]))
        progress(f"cold form: set {r + 1} of {R} built")
    assert all(overlap_keys(s) == 0 for s in sets)
    torch.cuda.synchronize()
    progress("cold form: sets resident; creating the shard")
    with ps.Shard(0, space, np.float32, device=dev.index) as sh:
        progress("cold form: shard created")
        sh.set_stream(torch.cuda.current_stream().cuda_stream)
        f = Form(sh, sets, dev)
        f.self_check(0, space, dev)
        progress("cold form: self-check done")
        res = run_form(f, steps, max(warmup, R), 1, dev)
        progress("cold form: timed steps done")
        kt, ev_s = evented(f, steps, 1, dev)
        sh.set_stream(None)
    a, g = f.bytes(steps)
    del f, sets
    torch.cuda.empty_cache()
    dom = max(kt.items(), key=lambda kv: kv[1]["avg_ms"] * kv[1]["launches"])
    traffic, src = load_pmc(dom[0], {"n_gpus": 1, "batches": J, "batch_keys": B, "sets": R, "form": "cold",
                                     "shard_keys": int(space)}, "pmc_cold_latest.json")
    return {"workload": f"the headline step on a {space:.3g}-key float shard ({space * 4 / 1e9:.0f} GB of parameters): "
                        f"{J} x {B} windows at 1M-aligned bases pushed, then free window slots pulled (as many as "
                        "cfg 2 pulls), zero push/pull overlap, a window recurring only every ~8 steps: every "
                        "parameter read and write is served by HBM",
            "shard_keys": int(space), "GB/s": res["GB/s"], "ms_per_step": res["ms_per_step"],
            "bytes_per_step": (a + g) / steps, "ms_per_step_evented": ev_s / steps * 1e3,
            "kernels": kernel_fracs(kt),
            "kernel": dom[0], "frac": dom[1]["GB/s"] / HBM_PEAK_GBS, "traffic": traffic,
            "traffic_over_algorithmic": traffic / dom[1]["algorithmic_bytes"] if traffic else None,
            "traffic_source": src}


_T0 = time.perf_counter()


_RANK_TAG = f" r{os.environ['RANK']}" if int(os.environ.get("WORLD_SIZE", "1")) > 1 else ""


def progress(what):
    """One line per phase on stderr (a long run shows where it is; rank-tagged
    at N > 1)."""
    print(f"bench{_RANK_TAG} [{time.perf_counter() - _T0:7.1f} s] {what}", file=sys.stderr, flush=True)


def watchdog():
    """PSKV_BENCH_WATCHDOG=<s> (diagnostics, never set by the driver): every s
    seconds dump every thread's Python stack to stderr, so a run that stops
    making progress shows where each rank waits."""
    s = float(os.environ.get("PSKV_BENCH_WATCHDOG", "0") or 0)
    if s > 0:
        import faulthandler

        faulthandler.dump_traceback_later(s, repeat=True, file=sys.stderr)


def main(argv=None):
    args = parse(argv)
    watchdog()
    if args.vector_only:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle  # test infrastructure: the CPU baseline leg (VectorStorage restatement)

        oracle.build()
        sizes = [int(x) for x in args.vector_sizes.split(",") if x]
        res = vector_storage_fit(oracle, sizes)
        res["host_cpu"] = _cpu_model()
        print(json.dumps(res), flush=True)
        return
    # the JSON line is the only thing on stdout: everything else the run prints
    # (torch.distributed / gloo / RCCL banners, library notices) goes to stderr
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch

    import parameter_server_amd as ps
    from parameter_server_amd import workload

    rank, world, local = dist_init(args)
    dev = torch.device(f"cuda:{local}")
    J, B = args.batches, args.batch_keys
    # planning rank / world: the process's own, or (probe knob, one process,
    # never used by the driver) PSKV_BENCH_EMULATE="r/N" = rank r's share of
    # the N-GPU cfg-4 workload alone on this GPU
    prank, pworld = rank, world
    if os.environ.get("PSKV_BENCH_EMULATE") and world == 1:
        prank, pworld = (int(x) for x in os.environ["PSKV_BENCH_EMULATE"].split("/"))
    R = default_sets(args.sets, pworld)
    if args.cold_only:
        # the cold form pulls as many windows as cfg 2's set r: host planning only
        progress("cold form only")
        n_pulls = [len(plan_pull(0, 1, J, B, r, plan_rank(0, 1, J, B, r)[4])[0]) for r in range(R)]
        rec = cold_form(dev, J, B, R, args.steps, args.warmup, int(args.cold_keys), n_pulls)
        json_out.write(json.dumps({"cold": rec}) + "\n")
        json_out.flush()
        return
    sets = [make_set(prank, pworld, J, B, dev, r) for r in range(R)]
    assert all(overlap_keys(s) == 0 for s in sets), "a pull set overlaps its push set"
    n_pulls = [len(s["pull"]) for s in sets]
    key_space, lo, hi = plan_rank(prank, pworld, J, B)[:3]
    stream = torch.cuda.current_stream()
    shard = ps.Shard(lo, hi, np.float32, device=local)
    shard.set_stream(stream.cuda_stream)  # torch events and the kernels share one stream
    form = Form(shard, sets, dev)
    # correctness guard on the benchmarked state: one rotation from a cleared
    # shard, every pull against a model of the shard
    progress("headline: self-check")
    form.self_check(lo, hi, dev)
    progress("headline: timed steps")
    head = run_form(form, args.steps, max(args.warmup, R), world, dev)
    ktimes, evented_s = evented(form, args.steps, world, dev)
    touched = min(form.touched(i) for i in range(R))
    a_b, g_b = form.bytes(args.steps)
    own_bytes = a_b + g_b
    n_push = sum(n for s in sets for _, _, n in s["slices"]) / R  # keys this rank receives per step
    per_gpu = {"mean_GB/s": head["GB/s"] / world,
               "min_GB/s": -max_over_ranks(-head["own_GB/s"], world, dev),
               "max_GB/s": max_over_ranks(head["own_GB/s"], world, dev),
               "min_keys_pushed_per_step": -max_over_ranks(-n_push, world, dev),
               "max_keys_pushed_per_step": max_over_ranks(n_push, world, dev)}

    zipf_res = None
    if not args.no_zipf:
        progress("cfg 3 (Zipf)")
        zipf_res, zb = zipf_sparse(prank, world, dev, lo, hi, B, args.steps)
    cold = None
    if pworld == 1 and not args.no_cold:
        shard.set_stream(None)  # the cold shard takes the stream meanwhile
        progress("cold form")
        cold = cold_form(dev, J, B, R, args.steps, args.warmup, int(args.cold_keys), n_pulls)
        shard.set_stream(stream.cuda_stream)

    # dominant kernel: the one with the most time in the evented pass
    dom = max(ktimes.items(), key=lambda kv: kv[1]["avg_ms"] * kv[1]["launches"])
    achieved = dom[1]["GB/s"]
    cfg_key = {"n_gpus": world, "batches": J, "batch_keys": B, "sets": R, "form": "pull-free-slots"}
    traffic, traffic_src = load_pmc(dom[0], cfg_key)
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": dom[0],
            "algorithmic_bytes_per_launch": dom[1]["algorithmic_bytes"],
            "bytes_per_unit": "Add n*4 + 2*u*V (keys, last values, parameter writes), Get q*(4+2V); V=4, "
                              "u = distinct pushed keys",
            "timing": "HIP events on the launch stream around each launch of the two streaming "
                      "kernels, over a second pass of the same K steps run right after the "
                      "event-free timed region",
            "ms_per_step_evented": evented_s / args.steps * 1e3,
            "kernels": kernel_fracs(ktimes)}
    if cold is not None:
        roof["cold"] = cold
    if traffic_src:
        roof["traffic_source"] = traffic_src
        roof["traffic_over_algorithmic"] = traffic / dom[1]["algorithmic_bytes"]

    result = {
        "metric": METRIC,
        "value": head["GB/s"],
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": head["ms_per_step"],
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": (f"cfg 2 dense: 1e8-key float shard, {J} x {B} contiguous-key windows at 1M-aligned bases "
                         if pworld == 1 else
                         f"cfg 4 ranges: 1e9 keys over {pworld} range shards, {J} producer streams each pushing one "
                         f"{B}-key contiguous window at a uniformly random base, sliced by the range map ") +
                        "pushed, then windows the push did not touch pulled (zero push/pull overlap), per step; "
                        f"assign (last-write-wins) mode, grouped launches, {R} window sets rotated over the steps",
            "key_space": key_space,
            "shard_keys_per_gpu": hi - lo,
            "windows_per_step": J,
            "batch_keys": B,
            "window_sets": R,
            "window_set_seeds": [workload.set_seed(r, pworld) for r in range(R)],
            "keys_pushed_per_step_per_gpu": n_push,
            "keys_pulled_per_step_per_gpu": sum(n for s in sets for _, _, n in s["pull"]) / R,
            "push_pull_overlap_keys": max(overlap_keys(s) for s in sets),
            "distinct_pushed_keys_per_step_per_gpu": sum(s["u"] for s in sets) / R,
            "bytes_per_step_per_gpu": own_bytes / args.steps,
            "param_bytes_touched_per_step_per_gpu": touched,
            "parallelism": f"range-sharded x{pworld} (no collective)",
        },
        "roofline": roof,
        # cfg 4 reports per-GPU next to aggregate: each rank's own
        # bytes over its own time, min / max over ranks
        "per_gpu": per_gpu,
    }
    if (prank, pworld) != (rank, world):
        result["config"]["emulated_rank"] = f"{prank}/{pworld} (probe: one rank's share alone on one GPU)"
    if zipf_res is not None:
        result["zipf_sparse"] = zipf_res
    extra = {}
    if not args.no_extra:
        warm = Form(shard, sets, dev, pull="same")
        w = run_form(warm, args.steps, 2, world, dev)
        extra["cache_warm_step"] = {
            "workload": "the round-2 headline form: the Get pulls the windows the step just pushed (their "
                        "parameters are still in the 256 MB Infinity Cache)", "GB/s": w["GB/s"],
            "ms_per_step": w["ms_per_step"]}
        del warm
        if pworld > 1:
            wsets = [make_set(prank, pworld, J, B, dev, r, weak=True) for r in range(R)]
            wf = Form(shard, wsets, dev)
            wf.self_check(lo, hi, dev)
            wr = run_form(wf, args.steps, 2, world, dev)
            extra["weak_scaled"] = {
                "workload": f"weak scaling: every rank's own {J} producers push 1M-aligned windows inside its "
                            "range (per-GPU work fixed), pull of free window slots of the range", "GB/s": wr["GB/s"],
                "ms_per_step": wr["ms_per_step"],
                "per_gpu_min_GB/s": -max_over_ranks(-wr["own_GB/s"], world, dev)}
            del wf, wsets
    shard.set_stream(None)
    shard.close()
    if rank == 0 and not args.no_cpu_baseline:
        progress("cpu baseline")
        if pworld == 1:
            sizes = [int(x) for x in args.vector_sizes.split(",") if x]
            result["cpu_baseline"] = cpu_baseline([f for _, f, _ in sets[0]["slices"]], B, args.cpu_batches, sizes)
            if zipf_res is not None:  # cfg 3's own CPU baseline: the same Zipf batches
                result["cpu_baseline"]["zipf"] = _zipf_cpu_sample(zb[:2], B)
        else:
            # cfg 4's baseline: 8 server threads with 8 storages on
            # this host, over the producers' windows of set 0, after every timed
            # region (the other ranks wait at the closing barrier meanwhile)
            result["cpu_baseline"] = cpu_baseline(list(sets[0]["bases"]), B, 16, [], servers=8)
    if zipf_res is not None:
        del zb
    if pworld == 1 and not args.no_extra:
        progress("side measurements")
        extra["dense_f64_step"] = variant_f64(rank, world, J, B, dev, R, args.steps, lo, hi)
        extra["dense_accumulate_step"] = variant_accumulate(rank, world, J, B, dev, sets, args.steps, lo, hi)
        extra.update(side_measurements(dev, B))
    if extra:
        result["extra"] = extra
    if rank == 0:
        json_out.write(json.dumps(result) + "\n")
        json_out.flush()
    if world > 1:
        import torch.distributed as dist

        barrier(world)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
