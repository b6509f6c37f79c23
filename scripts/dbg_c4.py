"""Per-call timing of one C4 step (bench.py --workload c4) to find host overhead."""
import time

import numpy as np
import torch

import bench
import sy_amd.device as dev

torch.cuda.set_device(0)
basis, new, files = bench.c4_files(dev, 1 << 20, 10000, 0)
boff, blen, soff, slen = files
bs = 4096
torch.cuda.synchronize()


def step(T):
    t = time.perf_counter()
    w, s = dev.signature_batch(basis, boff, blen, bs)
    torch.cuda.synchronize(); T["sig"] += time.perf_counter() - t; t = time.perf_counter()
    nblk = (blen + bs - 1) // bs
    last = blen - (nblk - 1) * bs
    idx = dev.BatchIndex(w, s, nblk, last, bs)
    torch.cuda.synchronize(); T["index"] += time.perf_counter() - t; t = time.perf_counter()
    res = dev.match_batch_handle(idx, new, soff, slen)
    dt = time.perf_counter() - t; T["match"] += dt; T["match_last"] = dt; t = time.perf_counter()
    import sys
    print(f"  python match {1e3 * T['match_last']:.2f}" if 'match_last' in T else "", file=sys.stderr)
    idx.close()
    res.close()
    T["free"] += time.perf_counter() - t


T = dict(sig=0.0, index=0.0, match=0.0, free=0.0, match_last=0.0)
step(T)
dev.set_profiling(True)
dev.profile(reset=True)
T = dict(sig=0.0, index=0.0, match=0.0, free=0.0, match_last=0.0)
for _ in range(3):
    step(T)
prof = dev.profile(reset=True)
print({k: round(v / 3 * 1e3, 2) for k, v in T.items()}, flush=True)
print({k: round(v["ms"] / v["count"], 3) for k, v in prof.items()}, flush=True)
