"""Phase timing of the C5 step on one GPU (host overhead hunt)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import sy_amd.device as dev
from sy_amd import shard
gib = float(sys.argv[1]) if len(sys.argv) > 1 else 8
bs = 8192
n = int(gib * (1 << 30))
basis = torch.empty(n, dtype=torch.uint8, device="cuda")
dev.synth_fill_range(basis, 0, 0x5E1D0005)
new = torch.empty(n, dtype=torch.uint8, device="cuda")
dev.synth_fill_range(new, 0, 0x5E1D0005)
dev.synth_mutate_blocks(new, new, 0, bs, 0x5E1D0006, 10000)
torch.cuda.synchronize()
for it in range(4):
    T = [time.perf_counter()]
    w, s = dev.signature(basis, bs); torch.cuda.synchronize(); T.append(time.perf_counter())
    idx = dev.Index(w, s, bs, bs); torch.cuda.synchronize(); T.append(time.perf_counter())
    ch = dev.Chunk(idx, new, 0, n, 0, n - bs + 1); torch.cuda.synchronize(); T.append(time.perf_counter())
    d, ex = ch.walk(0); T.append(time.perf_counter())
    ch.close(); idx.close(); torch.cuda.synchronize(); T.append(time.perf_counter())
    names = ["sig", "index", "classify", "walk", "close"]
    print(" ".join(f"{k}={1e3*(b-a):.2f}ms" for k, a, b in zip(names, T, T[1:])), len(d.kind), flush=True)
