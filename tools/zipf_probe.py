"""Per-kernel breakdown of the general (unsorted) path on cfg 3 Zipf batches,
assign and accumulate, plus the same keys through the Get alone (the random
read floor).  Interleaved variants in one process (env knobs per shard).

  python tools/zipf_probe.py ["KNOB=V,..."] ...
  (PROBE_DTYPE=f64: 8-byte values; PROBE_J, PROBE_ROUNDS, PROBE_SPACE,
  PROBE_WORKLOAD=dense)
"""
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import parameter_server_amd as ps
    from parameter_server_amd import _lib, workload

    variants = sys.argv[1:] or [""]
    J = int(os.environ.get("PROBE_J", "8"))
    rounds = int(os.environ.get("PROBE_ROUNDS", "5"))
    space, B = int(float(os.environ.get("PROBE_SPACE", "1e8"))), 1_000_000
    dev = torch.device("cuda:0")
    f64 = os.environ.get("PROBE_DTYPE", "f32") == "f64"  # 8-byte values
    ndt, tdt = (np.float64, torch.float64) if f64 else (np.float32, torch.float32)
    if os.environ.get("PROBE_WORKLOAD", "zipf") == "dense":
        zb = workload.dense_batches(J, space, batch=B, device=dev, dtype=tdt)
    else:
        zb = workload.zipf_batches(J, space, batch=B, device=dev, dtype=tdt)
    zo = [torch.empty_like(v) for _, v in zb]
    u_all = int(torch.unique(torch.cat([k for k, _ in zb])).numel())
    print(f"{os.environ.get('PROBE_WORKLOAD', 'zipf')}: {J} x {B} keys, distinct per step {u_all}, per batch {int(torch.unique(zb[0][0]).numel())}")
    shards = []
    for v in variants:
        for mode in ("assign", "accumulate"):
            env = dict(kv.split("=") for kv in v.split(",") if kv)
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            sh = ps.Shard(0, space, ndt, mode=mode)
            for k, o in old.items():
                os.environ.pop(k) if o is None else os.environ.__setitem__(k, o)
            adds = sh.prepare(zb)
            gets = sh.prepare([(k, o) for (k, _), o in zip(zb, zo)], is_get=True)
            shards.append((f"{v or 'default'}/{mode}", sh, adds, gets, env))
    res = {n: {} for n, *_ in shards}
    for r in range(rounds + 1):
        for name, sh, adds, gets, env in shards:
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)  # launch-time knobs (read per launch) see the variant too
            sh.reset_timing()
            sh.set_timing(r > 0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            sh.add_grouped(adds)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            sh.get_grouped(gets)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            sh.set_timing(False)
            for k, o in old.items():
                os.environ.pop(k) if o is None else os.environ.__setitem__(k, o)
            if r == 0:
                continue
            res[name].setdefault("add_wall", []).append((t1 - t0) * 1e3)
            res[name].setdefault("get_wall", []).append((t2 - t1) * 1e3)
            for k, kn in _lib.KERNEL_NAMES.items():
                t = sh.kernel_time(k)
                if t["launches"]:
                    res[name].setdefault(kn, []).append(t["total_ms"] / t["launches"])
    n = J * B
    for name, d in res.items():
        parts = [f"{name:32s}"]
        for k, v in d.items():
            parts.append(f"{k}={statistics.median(v):.4f}ms")
        g = statistics.median(d["k_gather"])
        parts.append(f"gather={n * 12 / g / 1e6:.0f}GB/s ({n / g / 1e6:.1f} Gkeys/s)")
        print("  ".join(parts), flush=True)


if __name__ == "__main__":
    main()
