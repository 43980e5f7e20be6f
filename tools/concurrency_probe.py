"""Upper bound of running a step's Get concurrently with its Add.

bench.py's step pushes window set r (K2g, K4r) and then pulls windows the push
did not touch (K1); the two kernels run back to back on the shard's stream.
This probe asks what the hardware would give if the Get's chunks ran beside
the Add instead: two shards X and Y over the same key range, X takes the
step's Add and Y the step's Get (the same access shapes on different memory,
so the kernels do not depend on each other), and per step
  seq   X.add_grouped, Y.get_grouped on ONE stream (what the ordering costs)
  conc  X.add_grouped on stream A, Y.get_grouped on stream B, B waiting for
        the step's start on A and A for the Get's end on B (a step's Add
        waits for the previous step's Get: the write-after-read order a real
        concurrent Get needs)
  free  as conc without the two cross-stream waits (no ordering at all: the
        streams run free until the end; the hardware's concurrency alone)
  ref   the real pskv_add_get_grouped on X alone (K2g, K4r, K1)
measured interleaved, `rounds` x `steps` steps each, for N = 1 (cfg 2) and a
rank of N = 8 (cfg 4, rank 0).

  python tools/concurrency_probe.py [steps] [rounds]
"""
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import bench
    import parameter_server_amd as ps

    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    for rank, world, R in ((0, 1, 8), (0, 8, 16)):
        J, B = 64, 1_000_000
        _, lo, hi, _, _ = bench.plan_rank(rank, world, J, B)
        sets = [bench.make_set(rank, world, J, B, dev, r) for r in range(R)]
        sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
        with ps.Shard(lo, hi, np.float32) as X, ps.Shard(lo, hi, np.float32) as Y:
            outs = [[torch.empty(k.numel(), dtype=torch.float32, device=dev) for k in s["pull_keys"]] for s in sets]
            adds = [X.prepare(s["batches"]) for s in sets]
            gets_y = [Y.prepare(list(zip(s["pull_keys"], o)), is_get=True) for s, o in zip(sets, outs)]
            gets_x = [X.prepare(list(zip(s["pull_keys"], o)), is_get=True) for s, o in zip(sets, outs)]
            keys = sum(sum(n for _, _, n in s["slices"]) for s in sets) / R
            pulls = sum(sum(n for _, _, n in s["pull"]) for s in sets) / R

            e0, e1 = torch.cuda.Event(), torch.cuda.Event()  # reused: a wait captures the record before it

            def run(mode):
                if mode == "seq":
                    X.set_stream(sa.cuda_stream)
                    Y.set_stream(sa.cuda_stream)
                elif mode in ("conc", "free"):
                    X.set_stream(sa.cuda_stream)
                    Y.set_stream(sb.cuda_stream)
                else:
                    X.set_stream(sa.cuda_stream)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(steps):
                    t = i % R
                    if mode == "ref":
                        X.add_get_grouped(adds[t], gets_x[t], sorted_hint=True)
                    elif mode == "seq":
                        X.add_grouped(adds[t], sorted_hint=True)
                        Y.get_grouped(gets_y[t])
                    elif mode == "free":
                        X.add_grouped(adds[t], sorted_hint=True)
                        Y.get_grouped(gets_y[t])
                    else:
                        e0.record(sa)
                        sb.wait_event(e0)
                        X.add_grouped(adds[t], sorted_hint=True)
                        Y.get_grouped(gets_y[t])
                        e1.record(sb)
                        sa.wait_event(e1)
                torch.cuda.synchronize()
                return (time.perf_counter() - t0) / steps * 1e6

            for m in ("ref", "seq", "conc", "free"):
                run(m)  # warm-up
            res = {m: [] for m in ("ref", "seq", "conc", "free")}
            for _ in range(rounds):
                for m in res:
                    res[m].append(run(m))
            X.set_stream(None)
            Y.set_stream(None)
            print(f"N={world} rank {rank}: {keys / 1e6:.2f} M keys pushed, {pulls / 1e6:.2f} M pulled per step; "
                  f"us/step median over {rounds} x {steps}: " +
                  ", ".join(f"{m} {statistics.median(v):.1f} (min {min(v):.1f})" for m, v in res.items()),
                  flush=True)
        del sets


if __name__ == "__main__":
    main()
