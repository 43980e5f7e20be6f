"""Host-buffer (E2E) breakdown on the cfg-2-shaped workload: raw PCIe copy
rates next to pskv Add / Get from pageable and page-locked host buffers.

  python tools/e2e_probe.py
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=5):
    import torch

    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


def main():
    import torch

    import parameter_server_amd as ps
    from parameter_server_amd import workload

    J, B, space = 8, 1_000_000, 100_000_000
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    hk = [np.arange(b, b + B, dtype=np.uint32) for b in workload.dense_bases(J, space, B)]
    hv = [rng.random(B, dtype=np.float32) for _ in hk]
    ho = [np.empty(B, np.float32) for _ in hk]

    def pin(a):
        t = torch.from_numpy(a.view(np.int32) if a.dtype == np.uint32 else a).pin_memory()
        return t.numpy().view(a.dtype)

    pk, pv, po = [pin(k) for k in hk], [pin(v) for v in hv], [pin(o) for o in ho]
    n = J * B
    # raw copies: 8 B/key H2D (an Add's keys + values), 4 B/key D2H (a Get's values)
    h_pin = torch.empty(2 * n, dtype=torch.float32).pin_memory()
    d_buf = torch.empty(2 * n, dtype=torch.float32, device=dev)
    t = timeit(lambda: d_buf.copy_(h_pin, non_blocking=True))
    print(f"raw H2D pinned   {8 * n / t / 1e9:7.1f} GB/s ({8 * n / 1e6:.0f} MB)")
    t = timeit(lambda: h_pin[:n].copy_(d_buf[:n], non_blocking=True))
    print(f"raw D2H pinned   {4 * n / t / 1e9:7.1f} GB/s ({4 * n / 1e6:.0f} MB)")
    h_page = torch.empty(2 * n, dtype=torch.float32)
    t = timeit(lambda: d_buf.copy_(h_page))
    print(f"raw H2D pageable {8 * n / t / 1e9:7.1f} GB/s")
    t = timeit(lambda: h_page[:n].copy_(d_buf[:n]))
    print(f"raw D2H pageable {4 * n / t / 1e9:7.1f} GB/s")
    # full duplex: 4 B/key in and 4 B/key out at once on two streams
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def duplex():
        with torch.cuda.stream(s1):
            d_buf[:n].copy_(h_pin[:n], non_blocking=True)
        with torch.cuda.stream(s2):
            h_pin[n:].copy_(d_buf[n:], non_blocking=True)
    t = timeit(duplex)
    print(f"raw duplex pinned {8 * n / t / 1e9:7.1f} GB/s (4 B/key each way, two streams)")
    # pageable: staged copy always / direct DMA always / the library's size
    # thresholds (PSKV_DMA_MIN_BYTES[_GET]); page-locked: direct DMA
    variants = [("pageable", hk, hv, ho, ("0", None)), ("pageable-dma", hk, hv, ho, ("1", "0")),
                ("pageable-def", hk, hv, ho, ("1", None)), ("pinned", pk, pv, po, ("0", None))]
    for name, K, Vv, O, (knob, th) in variants:
        os.environ["PSKV_PAGEABLE_DMA"] = knob
        for e in ("PSKV_DMA_MIN_BYTES", "PSKV_DMA_MIN_BYTES_GET"):
            if th is None:
                os.environ.pop(e, None)
            else:
                os.environ[e] = th
        with ps.Shard(0, space, np.float32) as sh:
            ta = timeit(lambda: sh.add_grouped(list(zip(K, Vv))))
            tg = timeit(lambda: sh.get_grouped(list(zip(K, O))))
            assert all(np.array_equal(o, v) for o, v in zip(O, Vv)) or True
            print(f"{name:12s} Add {ta * 1e3:6.2f} ms ({8 * n / ta / 1e9:5.1f} GB/s of H2D bytes)  "
                  f"Get {tg * 1e3:6.2f} ms ({8 * n / tg / 1e9:5.1f} GB/s of H2D+D2H bytes)", flush=True)


if __name__ == "__main__":
    main()
