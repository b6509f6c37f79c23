"""Timing probe for the whole-file XXH3 kernels (single large file, batch of files)."""
import time

import numpy as np
import torch

import sy_amd.device as dev

n = 4 << 30
buf = torch.empty(n, dtype=torch.uint8, device="cuda")
dev.synth_fill(buf, 7)
dev.set_profiling(True)
for name, fn in [("single 4 GiB", lambda: dev.xxh3(buf)),
                 ("4096 x 1 MiB", lambda: dev.xxh3_batch(buf, np.arange(4096, dtype=np.uint64) << 20,
                                                          np.full(4096, 1 << 20, dtype=np.uint64))),
                 ("64 x 64 MiB", lambda: dev.xxh3_batch(buf, np.arange(64, dtype=np.uint64) << 26,
                                                        np.full(64, 1 << 26, dtype=np.uint64)))]:
    fn()
    torch.cuda.synchronize()
    dev.profile(reset=True)
    t = time.perf_counter()
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 3
    prof = dev.profile(reset=True)
    print(name, f"{dt * 1e3:.2f} ms/call {n / dt / 2**30:.1f} GiB/s",
          {k: round(v["ms"] / v["count"], 3) for k, v in prof.items()}, flush=True)
