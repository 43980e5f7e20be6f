"""Where a timed region's fixed cost goes (rank 0 of N = 8 by default).

bench.py times exactly K steps between two synchronize calls, so each region
pays once for the first step's host path (Python, the library's host work,
the launch) before the GPU starts, and for the wake-up after the last kernel.
At a rank's ~38 us step and the driver's K = 20 that is several percent.
Measured here, on bench.py's own Form and window sets:
  host_call_us   host time of one step call while the GPU is busy (it runs ahead)
  one_step_us    synchronize, t0, one step, synchronize: the whole exposed path
  k_steps_us     the same for K steps, per step, K in 1, 2, 5, 10, 20, 50, 200
  sync_idle_us   synchronize on an idle device

  PSKV_BENCH_EMULATE=0/8 python tools/timed_region_probe.py
"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    import bench
    import parameter_server_amd as ps

    emu = os.environ.get("PSKV_BENCH_EMULATE", "0/8")
    rank, world = (int(x) for x in emu.split("/"))
    J, B = 64, 1_000_000
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    _, lo, hi, _, _ = bench.plan_rank(rank, world, J, B)
    R = 16
    sets = [bench.make_set(rank, world, J, B, dev, r) for r in range(R)]
    with ps.Shard(lo, hi, np.float32) as sh:
        sh.set_stream(torch.cuda.current_stream().cuda_stream)
        form = bench.Form(sh, sets, dev)
        for i in range(3 * R):
            form.step(i)
        torch.cuda.synchronize()

        def region(k, start=0):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(k):
                form.step(start + i)
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) * 1e6

        # host cost per call with the GPU busy (queue well below its depth)
        torch.cuda._sleep(20_000_000)
        t0 = time.perf_counter()
        for i in range(20):
            form.step(i)
        host = (time.perf_counter() - t0) / 20 * 1e6
        torch.cuda.synchronize()
        # the call's host path in parts: the Add alone, the Get alone, one-batch forms
        parts = {}
        one_add = sh.prepare(sets[0]["batches"][:1])
        one_get = sh.prepare([(sets[0]["pull_keys"][0], form.outs[0][0])], is_get=True)
        for name, fn in (("add_grouped (all batches)", lambda i: sh.add_grouped(form.adds[i % R], sorted_hint=True)),
                         ("get_grouped (all batches)", lambda i: sh.get_grouped(form.gets[i % R])),
                         ("add_grouped (1 batch)", lambda i: sh.add_grouped(one_add, sorted_hint=True)),
                         ("get_grouped (1 batch)", lambda i: sh.get_grouped(one_get)),
                         ("a library call that queues nothing (pskv_get_option)", lambda i: sh.get_option("NT")),
                         ("nothing", lambda i: None)):
            torch.cuda._sleep(20_000_000)
            t0 = time.perf_counter()
            for i in range(20):
                fn(i)
            parts[name] = (time.perf_counter() - t0) / 20 * 1e6
            torch.cuda.synchronize()
        idle = []
        for _ in range(50):
            t0 = time.perf_counter()
            torch.cuda.synchronize()
            idle.append((time.perf_counter() - t0) * 1e6)
        res = {}
        for k in (1, 2, 5, 10, 20, 50, 200):
            res[k] = statistics.median(region(k, 7 * j) / k for j in range(7))
        print(f"{emu}: host_call_us {host:.1f}, sync_idle_us {statistics.median(idle):.1f}")
        for n, v in parts.items():
            print(f"  host us per call, {n}: {v:.1f}")
        for k, v in res.items():
            print(f"  K = {k:3d}: {v:7.2f} us per step (fixed cost if the step is the K = 200 figure: "
                  f"{(v - res[200]) * k:6.1f} us per region)", flush=True)
        sh.set_stream(None)


if __name__ == "__main__":
    main()
