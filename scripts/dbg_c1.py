import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import sy_amd.device as gpu
from oracle import oracle as O
n = 52_428_800
old = O.synth_bytes(n, 0x5E1D0001)
new = old.copy()
new[1 << 20:(1 << 20) + 18] = np.frombuffer(b"MODIFIED DATA HERE", np.uint8)
new[0:20] = np.frombuffer(b"HEADER DATA AT START", np.uint8)
def dev(a):
    t = torch.zeros(len(a) + 16, dtype=torch.uint8, device="cuda")
    t[:len(a)] = torch.from_numpy(a).cuda()
    return t
b = dev(old)
w, s = gpu.signature(b[:n], 4096)
for mode in [None, "1", "0", None, None, "1"]:
    if mode is None: os.environ.pop("SYDELTA_PROBE", None)
    else: os.environ["SYDELTA_PROBE"] = mode
    idx = gpu.Index(w, s, 4096, 4096)
    d = gpu.match(idx, dev(new), length=n)
    idx.close()
    print(mode, len(d.tuples()), d.stats, flush=True)
