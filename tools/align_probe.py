"""How much does a window's alignment cost the streaming kernels?  bench.py's
cfg-2 step (64 x 1M windows pushed over a 1e8-key float shard, the free window
slots pulled) with every pushed and pulled window shifted by `delta` keys (0:
16-byte aligned parameter accesses; 1-3: every 4-key group straddles two
16-byte parameter slots), in one process, per-kernel HIP-event times.  cfg 4's
producer windows start at any key.

  python tools/align_probe.py [deltas, default 0,1,2,3] [steps]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import bench
    import parameter_server_amd as ps

    deltas = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,1,2,3").split(",")]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda:0")
    J, B, R = 64, 1_000_000, 4
    base_sets = [bench.make_set(0, 1, J, B, dev, r) for r in range(R)]
    for rep in range(2):
        for d in deltas:
            sets = []
            for s in base_sets:
                # every window moved up by d keys; the last slot's loses its
                # top d keys (the shard ends at 1e8), so none meets another
                sl = [(w, f + d, min(n, 100_000_000 - f - d)) for w, f, n in s["slices"]]
                bt = [(torch.arange(f, f + n, dtype=torch.int64, device=dev).to(torch.int32), v[:n])
                      for (_, f, n), (_, v) in zip(sl, s["batches"])]
                pl = [(w, f + d, min(n, 100_000_000 - f - d)) for w, f, n in s["pull"]]
                pk = [torch.arange(f, f + n, dtype=torch.int64, device=dev).to(torch.int32) for _, f, n in pl]
                from parameter_server_amd import workload
                sets.append({"slices": sl, "batches": bt, "u": workload.interval_union([(f, n) for _, f, n in sl]),
                             "r": s["r"], "pull": pl, "pull_keys": pk})
                assert bench.overlap_keys(sets[-1]) == 0
            with ps.Shard(0, 100_000_000, np.float32) as sh:
                sh.set_stream(torch.cuda.current_stream().cuda_stream)
                f = bench.Form(sh, sets, dev)
                if rep == 0:
                    f.self_check(0, 100_000_000, dev)
                res = bench.run_form(f, steps, 4, 1, dev)
                kt, _ = bench.evented(f, steps, 1, dev)
                sh.set_stream(None)
            print(f"rep {rep} delta {d}: step {res['ms_per_step']*1e3:.1f} us {res['GB/s']:.0f} GB/s  " +
                  "  ".join(f"{k} {v['avg_ms']*1e3:.1f} us ({v['GB/s']:.0f} GB/s)" for k, v in kt.items()),
                  flush=True)


if __name__ == "__main__":
    main()
