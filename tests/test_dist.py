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

        J, B = 16, 1_000_000
        key_space, lo, hi, bases = bench.plan_rank(rank, world, J, B)
        # gather every rank's range and windows
        rr = [None] * world
        dist.all_gather_object(rr, (lo, hi, [int(b) for b in bases]))
        ranges = [(a, b) for a, b, _ in rr]
        assert ranges[0][0] == 0 and ranges[-1][1] == key_space
        assert all(ranges[i][1] == ranges[i + 1][0] for i in range(world - 1))
        # the reference slicer routes a sample of every window's keys to its owner
        for r, (_, _, bs) in enumerate(rr):
            for b in bs:
                sample = np.array([b, b + 1, b + B // 2, b + B - 1], dtype=np.uint32)
                sl = oracle.range_slice_ref(ranges, sample)
                assert [s for s, _ in sl] == [r], (r, b, sl)
        # every window set the bench rotates over routes to its rank too, and
        # the sets differ (distinct seeds)
        for r in (1, 3):
            _, lo_r, hi_r, bases_r = bench.plan_rank(rank, world, J, B, r)
            assert (lo_r, hi_r) == (lo, hi)
            assert all(lo <= int(b) and int(b) + B <= hi for b in bases_r)
            assert list(bases_r) != list(bases)
        # reductions as bench.py does them (device = cpu under gloo)
        t = bench.max_over_ranks(float(rank + 1), world, torch.device("cpu"))
        u = bench.sum_over_ranks(10.0, world, torch.device("cpu"))
        q.put((rank, t, u, len(set(bases))))
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
        assert mx == float(world) and sm == 10.0 * world and nb >= 1
