"""Interleaved A/B of tuning variants in ONE process (cdna_hip_programming.md §5.4
rule 24).  Each variant is a shard created under its own environment knobs; the
cfg 2 step (grouped sorted Add + grouped Get of J x 1M windows) runs round-robin
over the variants and per-kernel HIP-event times are reported (median of rounds).

  python tools/tune.py "PSKV_TILE_SHIFT=14" "PSKV_TILE_SHIFT=16" ...
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
    rounds = int(os.environ.get("TUNE_ROUNDS", "8"))
    J = int(os.environ.get("TUNE_J", "64"))
    f64 = os.environ.get("TUNE_DTYPE", "f32") == "f64"  # TUNE_DTYPE=f64: 8-byte values
    V = 8 if f64 else 4
    space = 100_000_000
    dev = torch.device("cuda:0")
    B = int(os.environ.get("TUNE_BATCH", "1000000"))  # TUNE_BATCH: keys per window
    batches = workload.dense_batches(J, space, batch=B, device=dev,
                                     dtype=torch.float64 if f64 else torch.float32)
    outs = [torch.empty_like(v) for _, v in batches]
    shards = []
    for v in variants:
        env = dict(kv.split("=") for kv in v.split(",") if kv)
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        sh = ps.Shard(0, space, np.float64 if f64 else np.float32,
                      mode=os.environ.get("TUNE_MODE", "assign"))  # TUNE_MODE=accumulate: K6 + K7
        for k, o in old.items():
            if o is None:
                os.environ.pop(k)
            else:
                os.environ[k] = o
        adds = sh.prepare(batches)
        gets = sh.prepare([(k, o) for (k, _), o in zip(batches, outs)], is_get=True)
        shards.append((v or "default", sh, adds, gets))
    res = {name: {"step": [], "host": []} for name, *_ in shards}
    for r in range(rounds + 1):
        for name, sh, adds, gets in shards:
            sh.reset_timing()
            sh.set_timing(r > 0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                sh.add_grouped(adds, sorted_hint=True)
                sh.get_grouped(gets)
            th = time.perf_counter()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            sh.set_timing(False)
            if r == 0:
                continue
            res[name]["step"].append((t1 - t0) / 5 * 1e3)
            res[name]["host"].append((th - t0) / 5 * 1e3)
            # the same steps without event timing
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            for _ in range(5):
                sh.add_grouped(adds, sorted_hint=True)
                sh.get_grouped(gets)
            torch.cuda.synchronize()
            res[name].setdefault("step_untimed", []).append((time.perf_counter() - t2) / 5 * 1e3)
            for k, kn in _lib.KERNEL_NAMES.items():
                t = sh.kernel_time(k)
                if t["launches"]:
                    res[name].setdefault(kn, []).append(t["total_ms"] / t["launches"])
    # reference point on the same box: torch's copy kernel moving the same vals (8 B/key)
    ct = []
    for r in range(rounds):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for (_, v), o in zip(batches, outs):
            o.copy_(v)
        torch.cuda.synchronize()
        ct.append((time.perf_counter() - t0) * 1e3)
    med = statistics.median(ct)
    print(f"{f'torch copy_ ({2 * V} B/key)':40s}  {med:.4f}ms ({J * B * 2 * V / (med / 1e3) / 1e9:.0f} GB/s)")
    for name, d in res.items():
        line = [f"{name:40s}"]
        for k, v in d.items():
            med = statistics.median(v)
            extra = ""
            if k in ("k_gather", "k_assign_group"):
                extra = f" ({J * B * (4 + 2 * V) / (med / 1e3) / 1e9:.0f} GB/s)"
            if k in ("step", "step_untimed"):
                extra = f" ({J * B * (8 + 4 * V) / (med / 1e3) / 1e9:.0f} GB/s)"
            line.append(f"{k}={med:.4f}ms{extra}")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
