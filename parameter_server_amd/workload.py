"""Synthetic push/pull workloads of BASELINE.json's configs.

  cfg 2  dense:  shard [0, 1e8) float; batches of 1M contiguous keys at base
                 b_j = seed-42 uniform multiple of 1M; vals U(-1, 1), seed 42+j
  cfg 3  zipf:   key space 1e8; 1M keys per batch, Zipf(s=0.99) over ranks
                 1..1e8, rank -> key by a seed-7 random permutation, unsorted
  cfg 4  ranges: 1e9 keys over G range shards (rank r owns [r*K/G, (r+1)*K/G),
                 base/range_partition_manager.hpp's map); 64 producer streams,
                 stream s pushes a contiguous 1M window at a uniformly random
                 base in [0, K - 1M] (seed 1000 + s), sliced by the range map —
                 a window straddling a boundary splits in two (global_windows,
                 route_windows).  The weak-scaled form (every rank's producers
                 push 1M-aligned windows inside its own range) is rank_windows.

Generation uses torch on the target device (outside any timed region).
"""
from __future__ import annotations

import numpy as np

MILLION = 1_000_000


def dense_bases(n_batches: int, key_space: int, batch: int = MILLION, seed: int = 42,
                lo: int = 0) -> np.ndarray:
    """Uniform multiples of `batch` in [lo, lo+key_space) (cfg 2 / cfg 4 windows)."""
    rng = np.random.default_rng(seed)
    slots = key_space // batch
    return lo + rng.integers(0, slots, size=n_batches, dtype=np.int64) * batch


def dense_batches(n_batches, key_space, batch=MILLION, device="cuda:0", dtype=None, seed=42,
                  lo=0):
    """[(keys u32 tensor, vals tensor)] for cfg 2 (keys sorted, contiguous)."""
    import torch

    dtype = dtype or torch.float32
    out = []
    for j, b in enumerate(dense_bases(n_batches, key_space, batch, seed, lo)):
        keys = torch.arange(int(b), int(b) + batch, dtype=torch.int64, device=device).to(torch.int32)
        g = torch.Generator(device=device)
        g.manual_seed(seed + j)
        if dtype in (torch.float32, torch.float64):
            vals = torch.rand(batch, generator=g, device=device, dtype=dtype) * 2 - 1
        else:
            vals = torch.randint(-2**31, 2**31 - 1, (batch,), generator=g, device=device, dtype=dtype)
        out.append((keys, vals))
    return out


def zipf_batches(n_batches, key_space, batch=MILLION, s=0.99, device="cuda:0", dtype=None,
                 perm_seed=7, seed=42, lo=0):
    """cfg 3: exact discrete Zipf(s) ranks via an inverse CDF, mapped to keys
    lo + perm[rank] by a seeded permutation of [0, key_space); order unsorted."""
    import torch

    dtype = dtype or torch.float32
    w = torch.arange(1, key_space + 1, dtype=torch.float64, device=device).pow_(-s)
    cdf = torch.cumsum(w, 0)
    cdf /= cdf[-1].clone()
    del w
    gp = torch.Generator(device=device)
    gp.manual_seed(perm_seed)
    perm = torch.randperm(key_space, generator=gp, device=device)
    out = []
    for j in range(n_batches):
        g = torch.Generator(device=device)
        g.manual_seed(seed + j)
        u = torch.rand(batch, generator=g, device=device, dtype=torch.float64)
        ranks = torch.searchsorted(cdf, u).clamp_(max=key_space - 1)
        keys = (perm[ranks] + lo).to(torch.int32)
        if dtype in (torch.float32, torch.float64):
            vals = torch.rand(batch, generator=g, device=device, dtype=dtype) * 2 - 1
        else:
            vals = torch.randint(-2**31, 2**31 - 1, (batch,), generator=g, device=device, dtype=dtype)
        out.append((keys, vals))
    del cdf, perm
    return out


def rank_ranges(key_space: int, world: int):
    """Equal contiguous key ranges, one per GPU (range_partition_manager.hpp's map)."""
    step = key_space // world
    return [(r * step, (r + 1) * step if r + 1 < world else key_space) for r in range(world)]


def rank_windows(rank: int, world: int, key_space: int, n_windows: int, batch: int = MILLION,
                 seed: int = 1000):
    """cfg 4 producer windows for one rank: stream s of rank r draws its base with
    seed `seed` + (r * n_windows + s) (default 1000), a uniform multiple of `batch`
    inside the rank's range.  Returns base offsets (int64)."""
    lo, hi = rank_ranges(key_space, world)[rank]
    slots = (hi - lo) // batch
    bases = []
    for s in range(n_windows):
        rng = np.random.default_rng(seed + rank * n_windows + s)
        bases.append(lo + int(rng.integers(0, slots)) * batch)
    return np.asarray(bases, dtype=np.int64)


def global_windows(n_producers: int, key_space: int, batch: int = MILLION, seed: int = 1000):
    """cfg 4: producer stream s pushes the window [b_s, b_s + batch)
    with b_s uniform over [0, key_space - batch], drawn with seed `seed` + s
    (default 1000 + s).  Any alignment: windows straddle range boundaries."""
    return np.asarray([int(np.random.default_rng(seed + s).integers(0, key_space - batch + 1))
                       for s in range(n_producers)], dtype=np.int64)


def complement_windows(push_bases, lo: int, hi: int, batch: int = MILLION, seed: int = 0,
                       n_max: int | None = None) -> np.ndarray:
    """The pull windows of a step on an aligned shard (cfg 2; the cold form; the
    weak-scaled cfg 4): every `batch`-aligned window slot of [lo, hi) that the
    step's push set does not touch, in a seeded random order, at most n_max of
    them.  The pull then reads only parameters the step did not write, and reads
    each once (no repeated window inside one Get).  A push window that starts
    off the slot grid covers two slots; both count as touched."""
    slots = (hi - lo) // batch
    pushed = set()
    for b in push_bases:
        first, last = (int(b) - lo) // batch, (int(b) + batch - 1 - lo) // batch
        pushed.update(range(first, last + 1))
    free = np.array([s for s in range(slots) if s not in pushed], dtype=np.int64)
    free = free[np.random.default_rng(seed).permutation(free.size)]
    if n_max is not None:
        free = free[:n_max]
    return lo + free * batch


def disjoint_windows(push_bases, n: int, key_space: int, batch: int = MILLION, seed: int = 0,
                     max_draws: int = 100_000) -> np.ndarray:
    """The pull windows of a cfg-4 step: n windows at uniformly random bases in
    [0, key_space - batch] (any alignment), drawn in turn with seed `seed` + s and
    redrawn until the window meets neither a pushed window nor an earlier pull
    window — zero push/pull overlap, no key pulled twice.  A window that finds
    no free place within `max_draws` draws (the push and pull windows cannot
    fit the key space: too many or too large batches) raises ValueError instead
    of drawing for ever."""
    taken = sorted((int(b), int(b) + batch) for b in push_bases)
    out = []
    for s in range(n):
        rng = np.random.default_rng(seed + s)
        for _ in range(max_draws):
            b = int(rng.integers(0, key_space - batch + 1))
            if all(e <= b or b + batch <= a for a, e in taken):
                break
        else:
            raise ValueError(f"disjoint_windows: pull window {s} of {n} ({batch} keys) found no place free of "
                             f"{len(push_bases)} push and {s} pull windows in a {key_space}-key space after "
                             f"{max_draws} draws")
        taken.append((b, b + batch))
        out.append(b)
    return np.asarray(out, dtype=np.int64)


def interval_union(intervals) -> int:
    """Number of distinct keys covered by half-open [a, a + n) intervals."""
    tot, end = 0, -1
    for a, n in sorted((int(a), int(n)) for a, n in intervals if n > 0):
        b = a + n
        if b <= end:
            continue
        tot += b - max(a, end)
        end = b
    return tot


def set_seed(r: int, world: int) -> int:
    """Base seed of window set r (the bench rotates R sets of windows over its
    steps, so no step re-pushes the windows the step before it touched).  Set 0
    is the config's own seed: 42 (cfg 2) / 1000 (cfg 4)."""
    return (42 if world == 1 else 1000) + 100_000 * r


def route_windows(bases, batch, ranges):
    """Slice every window [b, b+batch) with the range shard map (mirror of
    RangePartitionManager::Slice over a sorted window).  Returns, per range,
    a list of (window index, start offset, length).  A window that straddles a
    boundary splits into two slices."""
    per = [[] for _ in ranges]
    for w, b in enumerate(bases):
        b = int(b)
        e = b + batch
        r = 0
        pos = b
        while pos < e:
            while r + 1 < len(ranges) and not (ranges[r][0] <= pos < ranges[r][1]):
                r += 1
            end = e if r + 1 == len(ranges) else min(e, ranges[r][1])
            per[r].append((w, pos - b, end - pos))
            pos = end
    return per
