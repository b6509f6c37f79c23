"""Compare signature variants against the oracle on a few sizes (GPU)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import oracle as O
C = O.C()
v = os.environ.get("SYDELTA_SIG_VARIANT", "0")
import sy_amd.device as dev
for bs in (256, 1024, 2048, 3072, 4096, 5120, 8192, 64 * 33, 1 << 16):
    n = bs * 37
    h = O.synth_bytes(n, bs)
    t = torch.from_numpy(h).cuda()
    w, s = dev.signature(t, bs)
    ew, es, _ = C.compute_checksums(h, bs, threads=4)
    ok = np.array_equal(w.cpu().numpy().view(np.uint32), ew) and np.array_equal(s.cpu().numpy().view(np.uint64), es)
    wok = np.array_equal(w.cpu().numpy().view(np.uint32), ew)
    print(f"variant {v} bs {bs}: {'OK' if ok else 'MISMATCH'} (weak {'ok' if wok else 'bad'})", flush=True)
