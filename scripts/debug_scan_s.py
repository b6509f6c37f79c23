"""Debug aid for k_scan_s (SYDELTA_SCAN_L1=3): match an identical / shifted copy of a
96 MiB basis with the probe off and report which expected block hits are missing,
by unit (2048 positions) and by lane of the thread that rolled them."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sy_amd.device as gpu  # noqa: E402

os.environ["SYDELTA_PROBE"] = "0"
bs = 4096
n = 96 << 20
basis = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
gpu.synth_fill(basis[:n], 0x5E1D0101)
for mode in ("1", "3"):
    os.environ["SYDELTA_SCAN_L1"] = mode
    for shift in (0, 1, 2048 + 5):
        src = torch.zeros(n + shift + 16, dtype=torch.uint8, device="cuda")
        src[shift:shift + n] = basis[:n]
        w, s = gpu.signature(basis[:n], bs)
        idx = gpu.Index(w, s, bs, bs)
        d = gpu.match(idx, src, length=n + shift)
        idx.close()
        kind = np.asarray(d.kind)
        b = np.asarray(d.b, dtype=np.uint64)
        pos = np.concatenate([[0], np.cumsum(b)[:-1]]).astype(np.int64)
        cp = pos[kind == 0]
        exp = np.arange(n // bs, dtype=np.int64) * bs + shift
        miss = np.setdiff1d(exp, cp)
        print(f"mode {mode} shift {shift}: copies {cp.size} of {exp.size}, missing {miss.size}, stats {d.stats}")
        if miss.size:
            units = miss // 2048
            print("  first missing positions", miss[:12].tolist())
            print("  unit mod 64 histogram", np.bincount(units % 64, minlength=64).tolist())
            print("  position mod 2048 values", np.unique(miss % 2048)[:10].tolist())
