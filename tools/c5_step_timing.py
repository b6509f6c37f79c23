"""Host-side timeline of bench.py's C5 step at N=1 (measurement only): the wall time of
each call of the step, so the host work between the kernels is attributed.

    python tools/c5_step_timing.py [--steps 10]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    import torch

    import sy_amd.device as dev
    from sy_amd import shard

    bs, n = 8192, 8 << 30
    basis = torch.empty(n, dtype=torch.uint8, device="cuda")
    dev.synth_fill_range(basis, 0, 0x5E1D0005)
    p0, p1 = shard.chunk_bounds(n, bs, 1, 0)
    new = torch.empty((n + 15) // 16 * 16, dtype=torch.uint8, device="cuda")
    dev.synth_fill_range(new[:n], 0, 0x5E1D0005)
    dev.synth_mutate_blocks(new[:n], new[:n], 0, bs, 0x5E1D0006, 10000)
    torch.cuda.synchronize()
    stream = torch.cuda.Stream() if os.environ.get("C5_NULL_STREAM") != "1" else torch.cuda.current_stream()
    torch.cuda.set_stream(stream)
    rows = []
    for it in range(a.steps + 3):
        t = [time.perf_counter()]
        w, s = dev.signature(basis, bs, stream=stream)
        t.append(time.perf_counter())
        idx = dev.Index(w, s, bs, bs, device=0, stream=stream)
        t.append(time.perf_counter())
        ch = dev.Chunk(idx, new, 0, n, p0, p1, stream=stream)
        t.append(time.perf_counter())
        d, entry = shard.walk_chain(ch, 0, 1, p0, lambda v: [v], lambda v, src: v)
        t.append(time.perf_counter())
        ch.close()
        idx.close()
        t.append(time.perf_counter())
        del d
        t.append(time.perf_counter())
        if it >= 3:
            rows.append([(t[i + 1] - t[i]) * 1e3 for i in range(len(t) - 1)] + [(t[-1] - t[0]) * 1e3])
    names = ["signature", "index", "classify", "walk_chain", "close", "delta free", "step"]
    for r in rows:
        print(" ".join(f"{k} {v:.3f}" for k, v in zip(names, r)))
    med = [sorted(c)[len(c) // 2] for c in zip(*rows)]
    print("median: " + " ".join(f"{k} {v:.3f}" for k, v in zip(names, med)))


if __name__ == "__main__":
    main()
