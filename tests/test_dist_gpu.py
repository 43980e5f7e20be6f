"""cfg 4's multi-rank path on the GPU: two or four rank processes (gloo, all on
cuda:0, bench.py's PSKV_BENCH_SHARE_GPU rehearsal setup) each own one range
shard of the 1e9-key space (5e8 / 2.5e8 keys) (base/range_partition_manager.hpp's map) and run
bench.py's own step — 64 producer windows at uniformly random bases, sliced by
the range map (straddling windows split), pushed as one grouped Add per rank,
then windows no push of the step touched pulled — through the timed region (barrier,
synchronize, max over ranks).  Every pull, and at the end every rank's WHOLE
dense array, is compared bit for bit with the oracle's sequential
last-write-wins restatement (map_storage.hpp:17-27) of the slices that rank
received, in the order it applied them."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    import sys

    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), PSKV_BENCH_BACKEND="gloo", PSKV_BENCH_SHARE_GPU="1")
    try:
        import torch

        import bench
        import oracle

        oracle.build()
        r_, w_, local = bench.dist_init(bench.parse([]))
        assert (r_, w_, local) == (rank, world, 0)
        dev = torch.device("cuda:0")
        n_slices, split, keys, nz = _run_share(rank, world, world, dev)
        total = bench.sum_over_ranks(float(keys), world, dev)
        q.put((rank, "ok", n_slices, split, total, nz))
        bench.barrier(world)
        import torch.distributed as dist

        dist.destroy_process_group()
    except BaseException as e:  # report, never hang the parent
        import traceback

        q.put((rank, "error", traceback.format_exc(), 0, 0, 0))
        raise


def _run_share(rank, world, sync_world, dev):
    """Rank `rank`'s share of the `world`-GPU cfg-4 plan on `dev`: two drawn
    window sets of 64 producers plus one whose windows straddle every range
    boundary, 2 x 3 steps through bench.Form.step checked pull by pull against
    the oracle, then the same steps through bench.timed, then the WHOLE dense
    array against the oracle.  `sync_world` is the process group's size (1: the
    share runs alone, no collective).  Returns (slices, split slices, keys
    routed here, nonzero keys of the final state)."""
    import torch

    import bench
    import oracle
    import parameter_server_amd as ps

    J, B, R = 64, 1_000_000, 3
    sets = [bench.make_set(rank, world, J, B, dev, r) for r in range(2)]
    # a third set whose windows surely straddle every range boundary (and
    # overlap each other across it): the range map splits each in two
    bases = straddle_bases(world)
    sets.append(bench.make_set(rank, world, len(bases), B, dev, 2, bases=bases))
    own_edges = sum(1 for m in edges(world) if m in (rank * (10 ** 9 // world), (rank + 1) * (10 ** 9 // world)))
    assert len(sets[2]["slices"]) == 4 * own_edges and all(n < B for _, _, n in sets[2]["slices"])
    _, lo, hi, _, _ = bench.plan_rank(rank, world, J, B)
    assert hi - lo == 1_000_000_000 // world
    ref = np.zeros(hi - lo, np.float32)
    host = [[(f, v.cpu().numpy()) for (_, f, _), (_, v) in zip(s["slices"], s["batches"])] for s in sets]
    with ps.Shard(lo, hi, np.float32, device=dev.index or 0) as sh:
        sh.set_stream(torch.cuda.current_stream().cuda_stream)
        form = bench.Form(sh, sets, dev)
        steps = 2 * R
        # stepwise: every pull against the oracle state after the step's Add
        for i in range(steps):
            for f, v in host[i % R]:
                oracle.dense_last_wins(ref, lo, np.arange(f, f + v.size, dtype=np.uint32), v)
            form.step(i)
            torch.cuda.synchronize()
            t = i % R
            assert bench.overlap_keys(sets[t]) == 0
            for (_, f, n), o in zip(form.pull_slices[t], form.outs[t]):
                got = o.cpu().numpy()
                if not np.array_equal(got.view(np.uint32), ref[f - lo:f - lo + n].view(np.uint32)):
                    raise AssertionError(f"rank {rank}/{world} step {i}: pull of key {f} differs from the oracle")
        # the timed region as bench.py runs it, then the oracle catches up
        elapsed, own = bench.timed(form, steps, sync_world, dev)
        assert elapsed >= own > 0
        for i in range(steps):
            for f, v in host[i % R]:
                oracle.dense_last_wins(ref, lo, np.arange(f, f + v.size, dtype=np.uint32), v)
        dense = sh.dense_view().cpu().numpy()
        sh.set_stream(None)
        sh.sync()
        del form
    if not np.array_equal(dense.view(np.uint32), ref.view(np.uint32)):
        bad = np.nonzero(dense.view(np.uint32) != ref.view(np.uint32))[0]
        raise AssertionError(f"rank {rank}/{world}: {bad.size} keys differ, first at {lo + bad[:4]}")
    n_slices = sum(len(s["slices"]) for s in sets)
    split = sum(1 for s in sets for _, _, n in s["slices"] if n < B)
    keys = sum(n for s in sets for _, _, n in s["slices"])
    nz = int(np.count_nonzero(ref))
    del sets, ref, dense
    torch.cuda.empty_cache()
    return n_slices, split, keys, nz


@pytest.mark.parametrize("world", [8])
def test_cfg4_rank_shares_bit_exact(cuda, oracle_mod, world):
    """The N = 8 cfg-4 plan the driver's 8-GPU run executes, one rank's share at
    a time on cuda:0 in this process (eight processes on one GPU is the
    shared-device rehearsal DESIGN.md §8 records as stalling in torch's
    device-wide sorts): every rank's 1.25e8-key range shard, its slices of the
    64-producer window sets, the straddling windows at all 7 boundaries, every
    pull and the whole final array bit-exact against the oracle
    (base/range_partition_manager.hpp:19-46, server/map_storage.hpp:17-27)."""
    res = []
    for r in range(world):
        res.append(_run_share(r, world, 1, cuda))
        print(f"cfg4 N={world} rank {r}: {res[-1][0]} slices, {res[-1][2]} keys, bit-exact", flush=True)
    # every set's windows arrived whole over the ranks (straddling ones in two)
    assert sum(r[2] for r in res) == (2 * 64 + len(straddle_bases(world))) * 1_000_000
    assert all(r[0] > 0 and r[3] > 0 for r in res)
    # split slices: the outer ranks hold one boundary (4 straddling windows),
    # the inner ranks two
    assert res[0][1] >= 4 and res[-1][1] >= 4 and all(r[1] >= 8 for r in res[1:-1])


def edges(world):
    """The inner range boundaries of the 1e9-key space over `world` shards."""
    return [r * (10 ** 9 // world) for r in range(1, world)]


def straddle_bases(world):
    """Four windows across every boundary m: m - 300001, m - 999999, m - 1 and
    m - 300001 again (a repeated, overlapping window)."""
    return np.array([b for m in edges(world) for b in (m - 300_001, m - 999_999, m - 1, m - 300_001)])


@pytest.mark.parametrize("world", [2, 4])
def test_cfg4_ranks_bit_exact(world):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = []
    for _ in range(world):
        res.append(q.get(timeout=300))
    for p in ps:
        p.join(60)
    errs = [r for r in res if r[1] != "ok"]
    assert not errs, "\n".join(str(e[2]) for e in errs)
    assert all(p.exitcode == 0 for p in ps)
    res.sort()
    # every set's windows arrived whole over the ranks (split ones in two)
    assert res[0][4] == (2 * 64 + len(straddle_bases(world))) * 1_000_000
    assert all(r[2] > 0 and r[3] >= 4 and r[5] > 0 for r in res)


_RCCL_PROBE = r"""
import sys
sys.path.insert(0, sys.argv[1])
import torch
import torch.distributed as dist

import bench

dev = torch.device("cuda:0")
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=dev)
assert dist.get_backend() == "nccl"


class Form:  # a step with real device work on torch's stream
    def __init__(self):
        self.x = torch.zeros(1 << 20, device=dev)

    def step(self, i):
        self.x.add_(1.0)


f = Form()
elapsed, own = bench.timed(f, 5, 2, dev)  # world 2: the collective path, on one rank
assert elapsed == own > 0, (elapsed, own)
assert float(f.x[0]) == 5.0
assert bench.max_over_ranks(3.5, 2, dev) == 3.5
assert bench.sum_over_ranks(2.25, 2, dev) == 2.25
bench.barrier(2)
dist.destroy_process_group()
print("rccl ok")
"""


def test_rccl_synchronisation_one_rank(cuda):
    """bench.py's N > 1 synchronisation over RCCL ("nccl" -- the backend of the
    driver's multi-GPU run, which the gloo rehearsals above do not touch),
    exercised on the one GPU a box has: a world-1 process group bound to
    cuda:0 as dist_init binds it, the barrier-bracketed timed region, and the
    float64 MAX / SUM all-reduces the ranks' timings and byte counts go
    through (world passed as 2 so the collective path runs)."""
    import subprocess
    import sys

    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    r = subprocess.run(["timeout", "-k", "10", "120", sys.executable, "-c", _RCCL_PROBE, ROOT], capture_output=True,
                       text=True, cwd=ROOT, env=env)
    assert r.returncode == 0 and "rccl ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
