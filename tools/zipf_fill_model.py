"""Fill model of K1 (and K5b's stores) on cfg 3's Zipf keys, CPU only: how many
distinct 32/64/128-byte granules the keys touch over the whole chip and summed
over the 8 XCDs when K1's chunks are dealt round-robin to XCDs.

  python tools/zipf_fill_model.py [key_space] [chunk_keys]
"""
import sys

import numpy as np


def main():
    import torch

    sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
    from parameter_server_amd import workload

    space = int(float(sys.argv[1])) if len(sys.argv) > 1 else 100_000_000
    chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 8192  # keys per K1 workgroup chunk
    B, J = 1_000_000, 8
    zb = workload.zipf_batches(J, space, batch=B, device="cpu")
    keys = torch.cat([k for k, _ in zb]).numpy().astype(np.int64)
    per_batch = (B + chunk - 1) // chunk
    wg = np.concatenate([np.arange(B) // chunk + j * per_batch for j in range(J)])
    xcd = wg % 8
    uk = np.unique(keys)
    print(f"{J} x {B} Zipf keys over {space}: {len(uk)} distinct keys")
    for g in (32, 64, 128):
        per = g // 4
        chip = len(np.unique(uk // per))
        xs = sum(len(np.unique(keys[xcd == x] // per)) for x in range(8))
        print(f"{g:4d}-B granules: {chip:9d} distinct on the chip ({chip * g / 1e6:6.1f} MB), "
              f"{xs:9d} summed over XCDs ({xs * g / 1e6:6.1f} MB)")


if __name__ == "__main__":
    main()
