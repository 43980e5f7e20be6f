"""Probe: does a shard's own (blocking) stream order behind work on torch's
default stream, as seen by (a) a device Add queued behind a ~1 s spin kernel,
(b) pskv_sync's bounded wait, (c) the host read-back?  Prints timings."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import parameter_server_amd as ps

    print("current stream", torch.cuda.current_stream(), torch.cuda.current_stream().cuda_stream, flush=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    torch.cuda._sleep(50_000_000)
    e1.record()
    torch.cuda.synchronize()
    cpm = 50_000_000 / max(e0.elapsed_time(e1), 1e-3)
    print(f"calibration: {e0.elapsed_time(e1):.2f} ms for 50M cycles", flush=True)
    k = np.arange(0, 5000, 3, dtype=np.uint32)
    v = (k * 0.5).astype(np.float32)
    kd = torch.from_numpy(k.view(np.int32)).cuda()
    vd = torch.from_numpy(v + 1).cuda()
    for variant in ("own stream", "torch stream"):
        with ps.Shard(0, 10_000, np.float32) as sh:
            if variant == "torch stream":
                sh.set_stream(torch.cuda.current_stream().cuda_stream)
            sh.add(k, v)
            sh.sync()
            t0 = time.perf_counter()
            torch.cuda._sleep(int(1000 * cpm))
            t1 = time.perf_counter()
            sh.add(kd, vd)
            t2 = time.perf_counter()
            sh.sync()
            t3 = time.perf_counter()
            got = sh.get(k)
            t4 = time.perf_counter()
            torch.cuda.synchronize()
            t5 = time.perf_counter()
            print(f"{variant}: sleep enqueue {1e3*(t1-t0):.1f} ms, add {1e3*(t2-t1):.1f} ms, sync {1e3*(t3-t2):.1f} ms, "
                  f"get {1e3*(t4-t3):.1f} ms, torch sync {1e3*(t5-t4):.1f} ms, values new: "
                  f"{np.array_equal(got, v + 1)}", flush=True)
            sh.set_stream(None)


if __name__ == "__main__":
    main()
