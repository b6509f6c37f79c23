"""Timing of the batched signature call in a C4 step sequence."""
import time

import numpy as np
import torch

import bench
import sy_amd.device as dev
from sy_amd import _lib
from sy_amd._lib import check, lib

torch.cuda.set_device(0)
basis, new, files = bench.c4_files(dev, 1 << 20, 10000, 0)
boff, blen, soff, slen = files
bs = 4096
torch.cuda.synchronize()
import os
if os.environ.get("PROF"):
    dev.set_profiling(True)
for it in range(5):
    t = time.perf_counter()
    offs = np.ascontiguousarray(boff, dtype=np.uint64)
    lens = np.ascontiguousarray(blen, dtype=np.uint64)
    total = int(((lens + np.uint64(bs - 1)) // np.uint64(bs)).sum())
    weak = torch.empty(max(total, 1), dtype=torch.int32, device="cuda")
    strong = torch.empty(max(total, 1), dtype=torch.int64, device="cuda")
    t1 = time.perf_counter()
    check(lib.sydelta_signature_batch_device(0, basis.data_ptr(), offs.ctypes.data, lens.ctypes.data, len(lens), bs,
                                             weak.data_ptr(), strong.data_ptr(), None))
    t2 = time.perf_counter()
    nblk = (blen + bs - 1) // bs
    idx = dev.BatchIndex(weak, strong, nblk, blen - (nblk - 1) * bs, bs)
    t3 = time.perf_counter()
    res = dev.match_batch_handle(idx, new, soff, slen)
    t4 = time.perf_counter()
    idx.close()
    res.close()
    t5 = time.perf_counter()
    print(f"alloc {1e3 * (t1 - t):.2f} sig {1e3 * (t2 - t1):.2f} index {1e3 * (t3 - t2):.2f} match {1e3 * (t4 - t3):.2f}"
          f" free {1e3 * (t5 - t4):.2f}", flush=True)
