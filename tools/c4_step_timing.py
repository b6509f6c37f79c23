"""Host-side timeline of bench.py's C4 step (measurement only): the wall time of each call
for one rank's share of the 10 000 files (--files F), so the host work between kernels is
attributed.

    python tools/c4_step_timing.py [--files 1250] [--steps 20]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=1250)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import torch

    import bench
    import sy_amd.device as dev

    bs = 4096
    basis, new, files = bench.c4_files(dev, 1 << 20, a.files, 0)
    boff, blen, soff, slen = files
    torch.cuda.synchronize()
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    rows = []
    for it in range(a.steps + 3):
        t = [time.perf_counter()]
        w, s = dev.signature_batch(basis, boff, blen, bs, stream=stream)
        t.append(time.perf_counter())
        nblk = (blen + bs - 1) // bs
        last = blen - (nblk - 1) * bs
        idx = dev.BatchIndex(w, s, nblk, last, bs, device=0, stream=stream)
        t.append(time.perf_counter())
        res = dev.match_batch_handle(idx, new, soff, slen, stream=stream)
        t.append(time.perf_counter())
        idx.close()
        _ = res.stats
        res.close()
        t.append(time.perf_counter())
        if it >= 3:
            rows.append([(t[i + 1] - t[i]) * 1e3 for i in range(len(t) - 1)] + [(t[-1] - t[0]) * 1e3])
    names = ["signature", "index", "match", "close", "step"]
    med = [sorted(c)[len(c) // 2] for c in zip(*rows)]
    print("median: " + " ".join(f"{k} {v:.3f}" for k, v in zip(names, med)))


if __name__ == "__main__":
    main()
