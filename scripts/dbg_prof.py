"""Profiling overhead probe: batched signature calls with profiling off/on."""
import time

import numpy as np
import torch

import bench
import sy_amd.device as dev
from sy_amd._lib import check, lib

torch.cuda.set_device(0)
basis, new, files = bench.c4_files(dev, 1 << 20, 10000, 0)
boff, blen, soff, slen = files
bs = 4096
offs = np.ascontiguousarray(boff, dtype=np.uint64)
lens = np.ascontiguousarray(blen, dtype=np.uint64)
total = int(((lens + np.uint64(bs - 1)) // np.uint64(bs)).sum())
weak = torch.empty(total, dtype=torch.int32, device="cuda")
strong = torch.empty(total, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
for prof in (False, True, False, True):
    dev.set_profiling(prof)
    ts = []
    for it in range(8):
        t = time.perf_counter()
        check(lib.sydelta_signature_batch_device(0, basis.data_ptr(), offs.ctypes.data, lens.ctypes.data, len(lens),
                                                 bs, weak.data_ptr(), strong.data_ptr(), None))
        ts.append(1e3 * (time.perf_counter() - t))
    print("prof" if prof else "noprof", " ".join(f"{x:.2f}" for x in ts), flush=True)
