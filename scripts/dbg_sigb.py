"""Timing of the batched signature call alone (C4 shape)."""
import time

import torch

import bench
import sy_amd.device as dev

torch.cuda.set_device(0)
basis, new, files = bench.c4_files(dev, 1 << 20, 10000, 0)
boff, blen, soff, slen = files
torch.cuda.synchronize()
for it in range(6):
    t = time.perf_counter()
    w, s = dev.signature_batch(basis, boff, blen, 4096)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"call {1e3 * (t1 - t):.2f} ms, sync {1e3 * (t2 - t1):.2f} ms", flush=True)
