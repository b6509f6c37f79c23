"""Host-side cost of the match path on the CPU, with the device layer emulated
(tests/csrc/fake_device.cpp) and its time subtracted: what the library's host code
(classification bookkeeping, walks, batch objects) costs per call on the C4 and C5
shapes.  Not product code; it runs in this container without a GPU.

    python tools/host_profile.py [c4|c5|all] [--files N] [--gib G]

Prints, per shape and repetition, the wall time of each C-ABI call, the emulated
kernels' share, and the difference (host time).  SYDELTA_HOST_TIMING=1 adds the
library's own breakdown on stderr.
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def load():
    os.environ.setdefault("EMU_PROFILE", "1")  # copies count as device time (fake_device.cpp)
    import test_host_emulated as T

    lib = ctypes.CDLL(T._build())
    lib.emu_kernel_ms.restype = ctypes.c_double
    lib.emu_kernel_ms.argtypes = [ctypes.c_int]
    lib.sydelta_last_error.restype = ctypes.c_char_p
    return lib


def check(lib, rc):
    if rc:
        raise RuntimeError(lib.sydelta_last_error().decode())


def ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def timed(lib, label, fn, rows):
    lib.emu_kernel_ms(1)
    t0 = time.perf_counter()
    r = fn()
    wall = (time.perf_counter() - t0) * 1e3
    k = lib.emu_kernel_ms(1)
    rows.append((label, wall, k, wall - k))
    return r


def c4(lib, nfiles, fsz=1 << 20, bs=4096):
    from oracle import oracle as O

    rng = np.random.default_rng(4)
    stride = (fsz + 1 + 15) & ~15
    basis = np.zeros(nfiles * stride + 16, np.uint8)
    new = np.zeros(nfiles * stride + 16, np.uint8)
    for k in range(nfiles):
        b = O.synth_bytes(fsz, 0x5E1D0004 + k)
        basis[k * stride:k * stride + fsz] = b
        p = int(rng.integers(0, fsz + 1))
        new[k * stride:k * stride + fsz + 1] = np.concatenate([b[:p], [rng.integers(0, 256)], b[p:]]).astype(np.uint8)
        for q in rng.integers(0, fsz + 1, 16):
            new[k * stride + q] ^= 1 + int(rng.integers(0, 255))
    off = np.arange(nfiles, dtype=np.uint64) * np.uint64(stride)
    blen = np.full(nfiles, fsz, np.uint64)
    slen = np.full(nfiles, fsz + 1, np.uint64)
    nblk = (blen + bs - 1) // bs
    total = int(nblk.sum())
    last = (blen - (nblk - 1) * bs).astype(np.uint64)
    w = np.zeros(total, np.uint32)
    s = np.zeros(total, np.uint64)
    for rep in range(3):
        rows = []
        timed(lib, "signature_batch", lambda: check(lib, lib.sydelta_signature_batch_device(
            0, ptr(basis), ptr(off), ptr(blen), ctypes.c_uint64(nfiles), ctypes.c_uint64(bs), ptr(w), ptr(s), None)),
              rows)
        ix = ctypes.c_void_p()
        timed(lib, "index_create_batch", lambda: check(lib, lib.sydelta_index_create_batch(
            0, ptr(w), ptr(s), ptr(nblk), ptr(last), ctypes.c_uint64(nfiles), ctypes.c_uint64(bs), 1, None,
            ctypes.byref(ix))), rows)
        bt = ctypes.c_void_p()
        timed(lib, "match_batch", lambda: check(lib, lib.sydelta_match_batch_device(
            ix, ptr(new), ptr(off), ptr(slen), ctypes.c_uint64(nfiles), None, ctypes.byref(bt))), rows)
        timed(lib, "batch_free+index_free", lambda: (lib.sydelta_delta_batch_free(bt), lib.sydelta_index_free(ix)),
              rows)
        report(f"C4 shape: {nfiles} x 1 MiB files, rep {rep}", rows)


def c5(lib, gib, bs=8192):
    from oracle import oracle as O

    n = int(gib * (1 << 30)) // bs * bs
    basis = O.synth_bytes(n + 16, 0x5E1D0005)
    src = O.synth_edit_blocks(basis[:n], 0, bs, 0x5E1D0006, 10000)
    src = np.concatenate([src, np.zeros(16, np.uint8)])
    nb = n // bs
    w = np.zeros(nb, np.uint32)
    s = np.zeros(nb, np.uint64)
    npos = n - bs + 1
    for rep in range(3):
        rows = []
        timed(lib, "signature", lambda: check(lib, lib.sydelta_signature_device(
            0, ptr(basis), ctypes.c_uint64(n), ctypes.c_uint64(bs), ptr(w), ptr(s), None)), rows)
        ix = ctypes.c_void_p()
        timed(lib, "index_create", lambda: check(lib, lib.sydelta_index_create(
            0, ptr(w), ptr(s), ctypes.c_uint64(nb), ctypes.c_uint64(bs), ctypes.c_uint64(bs), 1, None,
            ctypes.byref(ix))), rows)
        ch = ctypes.c_void_p()
        timed(lib, "chunk_classify", lambda: check(lib, lib.sydelta_chunk_classify(
            ix, ptr(src), ctypes.c_uint64(0), ctypes.c_uint64(n), ctypes.c_uint64(n), ctypes.c_uint64(0),
            ctypes.c_uint64(npos), None, ctypes.byref(ch))), rows)
        d = ctypes.c_void_p()
        ex = ctypes.c_uint64()
        timed(lib, "chunk_walk", lambda: check(lib, lib.sydelta_chunk_walk(ch, ctypes.c_uint64(0), ctypes.byref(ex),
                                                                             ctypes.byref(d))), rows)
        timed(lib, "free", lambda: (lib.sydelta_delta_free(d), lib.sydelta_chunk_free(ch), lib.sydelta_index_free(ix)),
              rows)
        report(f"C5 shape: one {n / (1 << 30):g} GiB chunk, bs {bs}, 1% of blocks edited, rep {rep}", rows)


def report(title, rows):
    print(title)
    tot = 0.0
    for label, wall, k, host in rows:
        print(f"  {label:24s} wall {wall:9.2f} ms  emulated kernels {k:9.2f} ms  host {host:8.2f} ms")
        tot += host
    print(f"  {'host total':24s} {tot:9.2f} ms")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shape", nargs="?", default="all")
    ap.add_argument("--files", type=int, default=1000)
    ap.add_argument("--gib", type=float, default=1.0)
    a = ap.parse_args()
    lib = load()
    if a.shape in ("c4", "all"):
        c4(lib, a.files)
    if a.shape in ("c5", "all"):
        c5(lib, a.gib)


if __name__ == "__main__":
    main()
