"""Where a rank-sized step's time goes: the K2g (dense Add) and K1 (Get)
launches of bench.py's step, every workgroup's phase stamps from a diagnostic
build (-DPSKV_STEP_STAMPS, ab/stamps/libpskv.so; the real-time clock, 100 MHz,
shared by every XCD), relative to the first K2g workgroup's entry.

  PSKV_LIB_PATH=ab/stamps/libpskv.so python tools/step_stamps.py [rank/N] [steps]

Prints, per kernel, the spread of workgroup entry times, the phase durations
(median / p90) and the last workgroup's end, and the gap between K2g's last
store and K1's first entry; with HIP-event durations of the same launches.
"""
import ctypes
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
    from parameter_server_amd import _lib

    spec = sys.argv[1] if len(sys.argv) > 1 else "0/8"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    r, n = (int(x) for x in spec.split("/"))
    J, B = 64, 1_000_000
    dev = torch.device("cuda:0")
    R = bench.default_sets(None, n)
    sets = [bench.make_set(r, n, J, B, dev, i) for i in range(R)]
    _, lo, hi = bench.plan_rank(r, n, J, B)[:3]
    lib = ctypes.CDLL(_lib.LIB_PATH)
    lib.pskv_diag_step_stamps.argtypes = [ctypes.c_void_p]
    buf = np.zeros((2, 8192, 4), dtype=np.uint64)
    with ps.Shard(lo, hi, np.float32) as sh:
        sh.set_stream(torch.cuda.current_stream().cuda_stream)
        f = bench.Form(sh, sets, dev)
        for i in range(2 * R):
            f.step(i)
        torch.cuda.synchronize()
        # the HIP-event durations of the same steps, in a pass of their own:
        # an event record between the kernels moves their gaps
        sh.reset_timing()
        sh.set_timing(True, kernels=[_lib.PSKV_K_GATHER, _lib.PSKV_K_ASSIGN_TILES])
        for i in range(steps):
            f.step(i)
        torch.cuda.synchronize()
        sh.set_timing(False)
        ev = {k: sh.kernel_time(k)["total_ms"] * 1e3 / max(1, sh.kernel_time(k)["launches"])
              for k in (_lib.PSKV_K_ASSIGN_TILES, _lib.PSKV_K_GATHER)}
        # the step's wall time without events (the previous step drained first)
        walls = []
        for i in range(steps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            f.step(i)
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e6)
        rows = []
        for i in range(steps):
            lib.pskv_diag_step_stamps(buf.ctypes.data)  # clear
            f.step(i)
            torch.cuda.synchronize()
            assert lib.pskv_diag_step_stamps(buf.ctypes.data) == 0
            a, g = buf[0].astype(np.int64), buf[1].astype(np.int64)
            na = int((a[:, 0] > 0).sum())
            ng = int((g[:, 0] > 0).sum())
            a, g = a[:na], g[:ng]
            t0 = a[:, 0].min()
            us = lambda x: (x - t0) / 100.0  # 100 MHz ticks -> us
            rec = {
                "k2g_wgs": na, "k1_wgs": ng,
                "k2g_entry_last": us(a[:, 0].max()),
                "k2g_prologue_med": float(np.median(a[:, 1] - a[:, 0]) / 100.0),
                "k2g_first_chunk_med": float(np.median(a[a[:, 2] > 0, 2] - a[a[:, 2] > 0, 1]) / 100.0) if (a[:, 2] > 0).any() else 0.0,
                "k2g_wg_life_med": float(np.median(a[:, 3] - a[:, 0]) / 100.0),
                "k2g_last_store": us(a[:, 3].max()),
                "k1_entry_first": us(g[:, 0].min()), "k1_entry_last": us(g[:, 0].max()),
                "k1_keys_med": float(np.median(g[g[:, 1] > 0, 1] - g[g[:, 1] > 0, 0]) / 100.0) if (g[:, 1] > 0).any() else 0.0,
                "k1_wg_life_med": float(np.median(g[g[:, 2] > 0, 2] - g[g[:, 2] > 0, 0]) / 100.0) if (g[:, 2] > 0).any() else 0.0,
                "k1_last_store": us(g[:, 2].max()),
                "ev_k2g": ev[_lib.PSKV_K_ASSIGN_TILES], "ev_k1": ev[_lib.PSKV_K_GATHER],
            }
            # K2g workgroups that started after the first round had ended
            rec["k2g_wgs_started_late"] = int((a[:, 0] > np.median(a[:, 3])).sum())
            rows.append(rec)
        sh.set_stream(None)
    print(f"rank {spec}: {steps} steps; times in us from the first K2g workgroup's entry; "
          f"step wall (synchronize on both sides, no events) median {np.median(walls):.1f} us")
    for key in rows[0]:
        vals = np.array([r_[key] for r_ in rows], dtype=np.float64)
        print(f"  {key:24s} median {np.median(vals):8.2f}   min {vals.min():8.2f}   max {vals.max():8.2f}")


if __name__ == "__main__":
    main()
