import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import parameter_server_amd as ps
dev = torch.device("cuda:0")
M = 1 << 20
n = (1 << 32) + M
keys = torch.arange(n, dtype=torch.int64, device=dev).to(torch.int32)
vals = torch.ones(n, dtype=torch.int32, device=dev)
vals[1 << 32:] = 2
torch.cuda.synchronize()
print("vals tail", vals[(1 << 32):(1 << 32) + 4].tolist(), "keys tail", keys[(1 << 32):(1 << 32) + 4].tolist(), flush=True)
with ps.Shard(0, 1 << 32, np.int32) as sh:
    sh.set_timing(True)
    sh.add(keys, vals)
    sh.sync()
    dv = sh.dense_view()
    print("dense[0:4]", dv[:4].tolist(), "dense[M-2:M+2]", dv[M - 2:M + 2].tolist(),
          "bad low", int(torch.count_nonzero(dv[:M] != 2)), "bad mid", int(torch.count_nonzero(dv[M:] != 1)), flush=True)
    from parameter_server_amd import _lib
    for k, nm in _lib.KERNEL_NAMES.items():
        t = sh.kernel_time(k)
        if t["launches"]:
            print(nm, t, flush=True)
    # grouped pieces given explicitly
    sh.clear()
    sh.add_grouped([(keys[: 1 << 31], vals[: 1 << 31]), (keys[1 << 31: 1 << 32], vals[1 << 31: 1 << 32]),
                    (keys[1 << 32:], vals[1 << 32:])])
    sh.sync()
    print("grouped: bad low", int(torch.count_nonzero(dv[:M] != 2)), "bad mid", int(torch.count_nonzero(dv[M:] != 1)), flush=True)
    sh.clear()
    sh.add(keys[1 << 31: 1 << 32], vals[1 << 31: 1 << 32])
    sh.add(keys[1 << 32:], vals[1 << 32:])
    sh.sync()
    print("two calls (2^31 high, then 1M low): bad low", int(torch.count_nonzero(dv[:M] != 2)), flush=True)
    sh.clear()
    sh.add_grouped([(keys[1 << 31: 1 << 32], vals[1 << 31: 1 << 32]), (keys[1 << 32:], vals[1 << 32:])])
    sh.sync()
    print("grouped (2^31 high, 1M low): bad low", int(torch.count_nonzero(dv[:M] != 2)), flush=True)
