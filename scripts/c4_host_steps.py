"""Host time of each call of bench.py's C4 step (one caller): signature_batch,
BatchIndex, match_batch_handle, stats, batch free, index free -- wall time per call,
with and without a device synchronize before each (the first shows where the host
waits, the second what the host itself spends).  GPU only; not a test.

    python scripts/c4_host_steps.py [--files N] [--steps K]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    import bench
    import sy_amd.device as dev

    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=10000)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    bs = 4096
    basis, new, files = bench.c4_files(dev, 1 << 20, a.files, 0)
    boff, blen, soff, slen = files
    torch.cuda.synchronize()
    for sync in (False, True):
        rows = {}
        for step in range(a.steps + 1):
            t = {}
            def mark(name, t0):
                if sync:
                    torch.cuda.synchronize()
                t[name] = (time.perf_counter() - t0) * 1e3
                return time.perf_counter()
            t00 = t0 = time.perf_counter()
            w, s = dev.signature_batch(basis, boff, blen, bs)
            t0 = mark("signature_batch", t0)
            nblk = (blen + bs - 1) // bs
            last = blen - (nblk - 1) * bs
            idx = dev.BatchIndex(w, s, nblk, last, bs, device=0)
            t0 = mark("index_create_batch", t0)
            res = dev.match_batch_handle(idx, new, soff, slen)
            t0 = mark("match_batch", t0)
            st = res.stats
            t0 = mark("stats", t0)
            res.close()
            t0 = mark("batch_free", t0)
            idx.close()
            t0 = mark("index_free", t0)
            t["step"] = (time.perf_counter() - t00) * 1e3
            if step:
                for k, v in t.items():
                    rows.setdefault(k, []).append(v)
        print(f"== {'synchronized before each mark' if sync else 'no extra synchronization'} "
              f"(median of {a.steps} steps, ms)")
        for k, v in rows.items():
            print(f"  {k:20s} {np.median(v):8.3f}  (min {min(v):.3f} max {max(v):.3f})")


if __name__ == "__main__":
    main()
