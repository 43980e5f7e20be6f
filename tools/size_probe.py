"""Fixed cost per launch of the streaming kernels: K2g (grouped sorted Add)
and K1 (grouped Get) over J = 2..64 contiguous 1M-key windows of a 1e8-key
float shard (distinct, non-overlapping windows, 1M-aligned; every call pulls
/ pushes windows the previous call did not touch), HIP-event time per kernel
and wall time per Add+Get pair, then the least-squares fit t = t0 + bytes / BW
per kernel.  A rank's cfg-4 share at N = 8 is ~8 windows: what t0 costs there.

  python tools/size_probe.py [J list, default 2,4,8,16,32,64] [reps]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import parameter_server_amd as ps
    from parameter_server_amd import _lib

    js = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,4,8,16,32,64").split(",")]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    dev = torch.device("cuda:0")
    space, B, V = 100_000_000, 1_000_000, 4
    rng = np.random.default_rng(5)
    nwin = space // B
    res = {}
    with ps.Shard(0, space, np.float32) as sh:
        sh.set_stream(torch.cuda.current_stream().cuda_stream)
        for J in js:
            # R sets of J distinct windows each, sets disjoint where possible
            R = max(2, min(8, nwin // J))
            sets = []
            for r in range(R):
                w = rng.choice(nwin, size=J, replace=False)
                bt = [(torch.arange(int(b) * B, int(b) * B + B, dtype=torch.int64, device=dev).to(torch.int32),
                       torch.rand(B, device=dev)) for b in w]
                outs = [torch.empty(B, device=dev) for _ in w]
                sets.append((sh.prepare(bt), sh.prepare([(k, o) for (k, _), o in zip(bt, outs)], is_get=True)))
            for i in range(4):
                sh.add_grouped(sets[i % R][0], sorted_hint=True)
                sh.get_grouped(sets[(i + 1) % R][1])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(reps):
                sh.add_grouped(sets[i % R][0], sorted_hint=True)
                sh.get_grouped(sets[(i + 1) % R][1])
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / reps
            sh.reset_timing()
            sh.set_timing(True, kernels=[_lib.PSKV_K_GATHER, _lib.PSKV_K_ASSIGN_TILES])
            for i in range(reps):
                sh.add_grouped(sets[i % R][0], sorted_hint=True)
                sh.get_grouped(sets[(i + 1) % R][1])
            torch.cuda.synchronize()
            sh.set_timing(False)
            kt = {n: sh.kernel_time(k) for k, n in ((_lib.PSKV_K_ASSIGN_TILES, "K2g"), (_lib.PSKV_K_GATHER, "K1"))}
            ms = {n: t["total_ms"] / max(1, t["launches"]) for n, t in kt.items()}
            add_b = J * B * (4 + 2 * V)
            get_b = J * B * (4 + 2 * V)
            res[J] = (wall * 1e3, ms["K2g"], ms["K1"], add_b, get_b)
            print(f"J={J:3d}  step {wall * 1e6:8.1f} us ({(add_b + get_b) / wall / 1e9:6.0f} GB/s)  "
                  f"K2g {ms['K2g'] * 1e3:7.1f} us ({add_b / ms['K2g'] / 1e6:6.0f} GB/s)  "
                  f"K1 {ms['K1'] * 1e3:7.1f} us ({get_b / ms['K1'] / 1e6:6.0f} GB/s)", flush=True)
            del sets
        sh.set_stream(None)
    for name, col, bcol in (("step", 0, None), ("K2g", 1, 3), ("K1", 2, 4)):
        x = np.array([res[J][3] + res[J][4] if bcol is None else res[J][bcol] for J in js], dtype=np.float64)
        y = np.array([res[J][col] * 1e-3 for J in js])
        A = np.stack([np.ones_like(x), x], 1)
        (c0, c1), *_ = np.linalg.lstsq(A, y, rcond=None)
        print(f"fit {name:4s}: t0 = {c0 * 1e6:6.2f} us, BW = {1 / c1 / 1e9:7.0f} GB/s")


if __name__ == "__main__":
    main()
