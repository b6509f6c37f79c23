"""Round 3: host-side pieces of one C3 (or, with argument c3b, C3b) step (not product code): wall time of each call of
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
if len(sys.argv) > 1 and sys.argv[1] == "c3b":  # bench.py's C3b source (same seeds as its default)
    import numpy as np

    seed_base = 0x5E1D0002
    dev.synth_mutate_blocks(new, basis, 0, 4096, seed_base + 1, 50000)
    rng = np.random.default_rng(seed_base + 2)
    nblk4 = n // 4096
    ins = np.sort(rng.choice(nblk4, nblk4 // 100, replace=False)) * 4096 + rng.integers(0, 4096, nblk4 // 100)
    extra = torch.from_numpy(rng.integers(0, 256, ins.size, dtype=np.uint8)).cuda()
    cuts = np.concatenate([[0], ins, [n]])
    parts = []
    for i in range(ins.size + 1):
        parts.append(new[int(cuts[i]):int(cuts[i + 1])])
        if i < ins.size:
            parts.append(extra[i:i + 1])
    new = torch.cat(parts)
    del parts
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
