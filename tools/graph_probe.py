"""Does a HIP graph of the benchmarked steps beat launching them one by one?
bench.py's cfg-2 form (or, with PSKV_BENCH_EMULATE=r/N, rank r's cfg-4 share),
R window sets: one rotation of R steps is captured once into a torch CUDA graph
(the library launches on torch's current stream) and replayed; the same steps
are also launched eagerly.  Interleaved rounds, µs per step, median.

  python tools/graph_probe.py [rounds]
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

    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    J, B, R = 64, 1_000_000, 16
    prank, pworld = 0, 1
    if os.environ.get("PSKV_BENCH_EMULATE"):
        prank, pworld = (int(x) for x in os.environ["PSKV_BENCH_EMULATE"].split("/"))
    sets = [bench.make_set(prank, pworld, J, B, dev, r) for r in range(R)]
    _, lo, hi = bench.plan_rank(prank, pworld, J, B)[:3]
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        sh = ps.Shard(lo, hi, np.float32)
        sh.set_stream(side.cuda_stream)
        form = bench.Form(sh, sets, dev)
        form.self_check(lo, hi, dev)
        for i in range(2 * R):
            form.step(i)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=side):
            for i in range(R):
                form.step(i)
        torch.cuda.synchronize()
        eager, graph = [], []
        for _ in range(rounds):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(4 * R):
                form.step(i)
            torch.cuda.synchronize()
            eager.append((time.perf_counter() - t0) / (4 * R) * 1e6)
            t0 = time.perf_counter()
            for _ in range(4):
                g.replay()
            torch.cuda.synchronize()
            graph.append((time.perf_counter() - t0) / (4 * R) * 1e6)
        # the graph's steps are the benchmarked steps: the shard after them matches
        form.self_check(lo, hi, dev)
        print(f"rank {prank}/{pworld}: eager {statistics.median(eager):7.2f} us/step, "
              f"graph {statistics.median(graph):7.2f} us/step (median of {rounds})", flush=True)
        sh.set_stream(None)
        sh.close()


if __name__ == "__main__":
    main()
