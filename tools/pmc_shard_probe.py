"""Where a rocprofv3 --pmc pass over bench.py's cold form stops: shard creation,
one grouped Add and one grouped Get at growing shard sizes, a line per stage.
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -- python3 tools/pmc_shard_probe.py
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import parameter_server_amd as ps

    t0 = time.perf_counter()
    dev = torch.device("cuda:0")

    def say(what):
        print(f"[{time.perf_counter() - t0:6.1f} s] {what}", flush=True)

    for size in (100_000_000, 250_000_000, 500_000_000, 1_000_000_000):
        say(f"{size:.0e}: create")
        with ps.Shard(0, size, np.float32) as sh:
            sh.sync()
            say(f"{size:.0e}: created")
            k = torch.arange(size - 1_000_000, size, dtype=torch.int32, device=dev)
            v = torch.ones(1_000_000, dtype=torch.float32, device=dev)
            sh.add_grouped([(k, v), (k, v)], sorted_hint=True)
            sh.sync()
            say(f"{size:.0e}: add")
            o = torch.empty_like(v)
            sh.get_grouped([(k, o)])
            sh.sync()
            assert torch.equal(o, v)
            say(f"{size:.0e}: get")
        torch.cuda.synchronize()
        say(f"{size:.0e}: destroyed")


if __name__ == "__main__":
    main()
