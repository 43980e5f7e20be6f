"""Does the cfg-2 step get faster as a fresh box warms up?  Runs bench.py's
step (same window sets, same calls) in back-to-back timed blocks of 100 steps
for SECONDS and prints each block's ms/step, so a clock or memory warm-up
shows as a trend over the first blocks.

  python tools/warm_probe.py [SECONDS]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    import parameter_server_amd as ps

    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
    dev = torch.device("cuda:0")
    J, B, R = 64, 1_000_000, 4
    sets = [bench.make_workload(0, 1, J, B, dev, r) for r in range(R)]
    _, lo, hi = sets[0][:3]
    outs = [torch.empty(B, dtype=torch.float32, device=dev) for _ in range(J)]
    shard = ps.Shard(lo, hi, np.float32)
    shard.set_stream(torch.cuda.current_stream().cuda_stream)
    plans = [(shard.prepare(b), shard.prepare([(k, o) for (k, _), o in zip(b, outs)], is_get=True))
             for *_, b in sets]

    def step(i):
        a, g = plans[i % R]
        shard.add_grouped(a, sorted_hint=True)
        shard.get_grouped(g)

    t_start = time.perf_counter()
    blk = 0
    while time.perf_counter() - t_start < secs:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(100):
            step(i)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 10.0
        print(f"t={time.perf_counter() - t_start:6.2f}s block {blk:4d}: {ms:.4f} ms/step", flush=True)
        blk += 1


if __name__ == "__main__":
    main()
