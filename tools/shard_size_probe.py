"""Does the shard's size change the streaming kernels' rate?  The same step —
grouped Add of 32 distinct 1M-key windows, then grouped Get of the next set's
32 windows, 16 sets rotated, every window 1M-aligned (phase 0) and no window
of a set repeated in the next — on shards of 1e8, 5e8 and 1e9 float keys (the
N = 1, N = 2 and whole-cfg-4 sizes).  HIP-event time per kernel.  FLUSH=1 evicts L2 and
the Infinity Cache (a 1 GiB read sweep) before every step, outside the kernels.

  python tools/shard_size_probe.py [spaces, default 1e8,5e8,1e9]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import parameter_server_amd as ps
    from parameter_server_amd import _lib

    spaces = [int(float(x)) for x in (sys.argv[1] if len(sys.argv) > 1 else "1e8,5e8,1e9").split(",")]
    dev = torch.device("cuda:0")
    B, J, R, steps = 1_000_000, 32, 16, 40
    for space in spaces:
        rng = np.random.default_rng(3)
        slots = space // B
        perm = rng.permutation(slots)
        sets = []
        for r in range(R):  # consecutive sets share no window (slots permits it at these sizes)
            w = perm[(r * J) % (slots - J + 1):][:J] if slots >= 2 * J else rng.choice(slots, J, replace=False)
            bt = [(torch.arange(int(b) * B, int(b) * B + B, dtype=torch.int64, device=dev).to(torch.int32),
                   torch.rand(B, device=dev)) for b in w]
            outs = [torch.empty(B, device=dev) for _ in w]
            sets.append((bt, outs))
        with ps.Shard(0, space, np.float32) as sh:
            sh.set_stream(torch.cuda.current_stream().cuda_stream)
            adds = [sh.prepare(bt) for bt, _ in sets]
            gets = [sh.prepare([(k, o) for (k, _), o in zip(bt, outs)], is_get=True) for bt, outs in sets]
            for i in range(R):
                sh.add_grouped(adds[i], sorted_hint=True)
                sh.get_grouped(gets[(i + 1) % R])
            torch.cuda.synchronize()
            sh.reset_timing()
            sh.set_timing(True, kernels=[_lib.PSKV_K_GATHER, _lib.PSKV_K_ASSIGN_TILES])
            flush = torch.ones(1 << 28, device=dev) if os.environ.get("FLUSH") == "1" else None
            for i in range(steps):
                if flush is not None:  # L2 and Infinity Cache evicted (read-only sweep) before each step
                    flush.sum()
                sh.add_grouped(adds[i % R], sorted_hint=True)
                sh.get_grouped(gets[(i + 1) % R])
            torch.cuda.synchronize()
            sh.set_timing(False)
            kt = {n: sh.kernel_time(k) for k, n in ((_lib.PSKV_K_ASSIGN_TILES, "K2g"), (_lib.PSKV_K_GATHER, "K1"))}
            sh.set_stream(None)
        line = [f"space {space:.0e}:"]
        for n, t in kt.items():
            ms = t["total_ms"] / max(1, t["launches"])
            keys = t["elements"] / max(1, t["launches"])
            line.append(f"{n} {ms * 1e3:7.1f} us ({keys * 12 / ms / 1e6:5.0f} GB/s)")
        print("  ".join(line), flush=True)
        del sets, adds, gets
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
