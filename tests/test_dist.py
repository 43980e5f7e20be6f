"""Multi-rank path of bench.py on CPU (gloo, world_size 2 and 4): the range
shard map, per-rank windows, and the max/sum reductions the bench uses.  The
shards are independent (no data-path collective), so this is all the N>1
path adds on top of the single-GPU kernels."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import oracle

        J, B = 64, 1_000_000
        for r in (0, 1, 3):
            key_space, lo, hi, slices, bases = bench.plan_rank(rank, world, J, B, r)
            assert key_space == 1_000_000_000
            # gather every rank's range and slices of the 64 global producer windows
            rr = [None] * world
            dist.all_gather_object(rr, (lo, hi, slices, [int(b) for b in bases]))
            ranges = [(a, b) for a, b, _, _ in rr]
            assert ranges[0][0] == 0 and ranges[-1][1] == key_space
            assert all(ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
            assert all(x[3] == rr[0][3] for x in rr)  # every rank draws the same windows
            pieces = {}
            for q_, (a, b, sl, _) in enumerate(rr):
                for w, first, n in sl:
                    assert a <= first and first + n <= b  # a slice lies in its rank's range
                    pieces.setdefault(w, []).append((first, n, q_))
            # every window is covered exactly, in range order: whole, or split at a
            # range boundary where it straddles one
            assert sorted(pieces) == list(range(J))
            for w, ps_ in pieces.items():
                ps_.sort()
                b0 = int(bases[w])
                assert ps_[0][0] == b0 and sum(n for _, n, _ in ps_) == B
                assert all(ps_[i][0] + ps_[i][1] == ps_[i + 1][0] for i in range(len(ps_) - 1))
                # the reference slicer (range_partition_manager.hpp:19-46) routes
                # the window's keys the same way: its slice boundaries and owners
                keys = sorted({b0, b0 + B - 1} | {f for f, _, _ in ps_} | {f + n - 1 for f, n, _ in ps_})
                ref = oracle.range_slice_ref(ranges, np.array(keys, dtype=np.uint32))
                want = [(q_, [k for k in keys if f <= k < f + n]) for f, n, q_ in ps_]
                assert ref == want, (w, ref, want)
            # the step's pull: J windows meeting no pushed window and no other
            # pull, routed by the same map; every rank draws the same ones
            pull, pbases = bench.plan_pull(rank, world, J, B, r, bases)
            pp = [None] * world
            dist.all_gather_object(pp, (pull, [int(b) for b in pbases]))
            assert all(x[1] == pp[0][1] for x in pp)
            assert sum(n for sl, _ in pp for _, _, n in sl) == J * B
            for q_, (sl, _) in enumerate(pp):
                a, b, _, _ = rr[q_]
                assert all(a <= f and f + n <= b for _, f, n in sl)
            assert bench.overlap_keys({"slices": slices, "pull": pull}) == 0
            # weak-scaled form: this rank's windows stay inside its range, whole
            _, lo_w, hi_w, sl_w, _ = bench.plan_rank(rank, world, J, B, r, weak=True)
            assert (lo_w, hi_w) == (lo, hi) and len(sl_w) == J
            assert all(lo <= f and f + n <= hi and n == B for _, f, n in sl_w)
            _, b_w = bench.plan_rank(rank, world, J, B, r, weak=True)[3:]
            pw, _ = bench.plan_pull(rank, world, J, B, r, b_w, weak=True)
            assert pw and all(lo <= f and f + n <= hi for _, f, n in pw)
            assert bench.overlap_keys({"slices": sl_w, "pull": pw}) == 0
        # reductions as bench.py does them (device = cpu under gloo)
        t = bench.max_over_ranks(float(rank + 1), world, torch.device("cpu"))
        u = bench.sum_over_ranks(10.0, world, torch.device("cpu"))
        q.put((rank, t, u, len(slices)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_bench_multirank_plan_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get() for _ in range(world))
    for rank, mx, sm, nb in res:
        assert mx == float(world) and sm == 10.0 * world and nb >= 0
    assert sum(nb for *_, nb in res) >= 64  # the last set's windows, split ones counted per slice
