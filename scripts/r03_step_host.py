"""Round 3: host-side pieces of one C3 step (not product code): wall time of each call of
bench.py's C3 step with a device synchronize around it, and the library's own host
breakdown (SYDELTA_HOST_TIMING=1, stderr)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.getcwd()))
import sy_amd.device as dev  # noqa: E402

n, bs = 4 << 30, 4096
basis = torch.empty(n, dtype=torch.uint8, device="cuda")
new = torch.empty(n, dtype=torch.uint8, device="cuda")
dev.synth_fill(basis, 0x5E1D0002)
dev.synth_mutate(new, basis, 0x5E1D0003, 50000)
stream = torch.cuda.current_stream()
for rep in range(4):
    t = {}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    w, s = dev.signature(basis, bs, stream=stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    idx = dev.Index(w, s, bs, bs, device=0, stream=stream)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    d = dev.match(idx, new, stream=stream)
    torch.cuda.synchronize()
    t3 = time.perf_counter()
    del d
    t3a = time.perf_counter()
    idx.close()
    t3b = time.perf_counter()
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    print(f"rep {rep}: signature {1e3*(t1-t0):.3f} ms, index {1e3*(t2-t1):.3f} ms, match {1e3*(t3-t2):.3f} ms, "
          f"del delta {1e3*(t3a-t3):.3f} ms, index free {1e3*(t3b-t3a):.3f} ms, sync {1e3*(t4-t3b):.3f} ms, "
          f"total {1e3*(t4-t0):.3f} ms", flush=True)
