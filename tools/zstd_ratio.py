"""Ratio of the zstd encoder's sequential form (tests/csrc/zstd_ref.cpp: the same block
coder k_zstd_block runs, byte-identical frames) against the system libzstd at level 3
(what sy's compress/mod.rs:71-76 uses) on the synthetic Delta JSON texts of
tests/test_zstd.py; every frame is decoded by libzstd first.  CPU only; not product code.

    python tools/zstd_ratio.py > profiles/r02_cpu_zstd_ratios.txt
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import test_zstd as Z  # noqa: E402

lz = ctypes.CDLL("libzstd.so.1")
lz.ZSTD_compress.restype = ctypes.c_size_t
lz.ZSTD_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
lz.ZSTD_versionString.restype = ctypes.c_char_p
print(f"libzstd {lz.ZSTD_versionString().decode()}; ratio = frame bytes / text bytes")
print(f"{'text':14s} {'bytes':>9s} {'ours':>8s} {'libzstd-3':>10s}")
for name, data in Z._cases():
    if name not in ("copies", "literals", "mixed", "c5-copies", "runs", "len393216", "fibonacci", "all-ascii"):
        continue
    f = Z.ref_compress(data)
    assert Z.zstd_decode(f, len(data)) == data
    out = ctypes.create_string_buffer(len(data) + 1000)
    g = lz.ZSTD_compress(out, len(out), data, len(data), 3)
    print(f"{name:14s} {len(data):9d} {len(f) / len(data):8.4f} {g / len(data):10.4f}")
