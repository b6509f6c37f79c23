"""zstd frames of the Delta JSON (ssh.rs:1009-1017 compresses the
serde_json text with zstd; sy-remote.rs:160-179 decompresses it).

CPU part: the sequential host form of the device encoder (tests/csrc/zstd_ref.cpp over
sy_amd/csrc/sydelta_zstd.hpp: code builder, header writers, match candidates, greedy
parse, predefined-table FSE coding of the sequences) must produce frames that an
independent decoder -- the system's libzstd (ZSTD_decompress) -- turns back into the
input: JSON deltas (copy-heavy ones take the literals + sequences blocks), random and
skewed texts (codes limited to 11 bits), runs, RLE and Raw blocks, block-size edges,
empty input.  The device encoder is compared with
this host form byte for byte in tests/test_gpu_zstd.py."""
import ctypes
import ctypes.util
import json
import os
import random
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "build", "zstd_ref")


def _libzstd():
    for name in ("libzstd.so.1", ctypes.util.find_library("zstd") or ""):
        if not name:
            continue
        try:
            z = ctypes.CDLL(name)
        except OSError:
            continue
        z.ZSTD_decompress.restype = ctypes.c_size_t
        z.ZSTD_decompress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
        z.ZSTD_isError.restype = ctypes.c_uint
        z.ZSTD_isError.argtypes = [ctypes.c_size_t]
        z.ZSTD_getErrorName.restype = ctypes.c_char_p
        z.ZSTD_getErrorName.argtypes = [ctypes.c_size_t]
        return z
    return None


def zstd_decode(frame: bytes, size: int) -> bytes:
    z = _libzstd()
    dst = ctypes.create_string_buffer(max(1, size))
    src = ctypes.create_string_buffer(frame, len(frame))
    r = z.ZSTD_decompress(dst, size, src, len(frame))
    if z.ZSTD_isError(r):
        raise ValueError(z.ZSTD_getErrorName(r).decode())
    return dst.raw[:r]


def build_ref() -> str:
    os.makedirs(OUT, exist_ok=True)
    lib = os.path.join(OUT, "libzstd_ref.so")
    cmd = ["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
           "-I" + os.path.join(ROOT, "sy_amd", "csrc"), os.path.join(ROOT, "tests", "csrc", "zstd_ref.cpp"), "-o", lib]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return lib


def frame_bound(n: int) -> int:
    nb = max(1, -(-n // (128 << 10)))
    return 14 + 3 * nb + n


_REF = None


def ref_compress(data: bytes) -> bytes:
    global _REF
    if _REF is None:
        _REF = ctypes.CDLL(build_ref())
        _REF.zstd_ref_compress.restype = ctypes.c_size_t
        _REF.zstd_ref_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
    cap = frame_bound(len(data))
    out = ctypes.create_string_buffer(cap)
    src = ctypes.create_string_buffer(data, max(1, len(data)))
    n = _REF.zstd_ref_compress(src, len(data), out, cap)
    assert n > 0
    return out.raw[:n]


def delta_json(rng: random.Random, nops: int, lit_frac: float) -> bytes:
    ops = []
    for _ in range(nops):
        if rng.random() < lit_frac:
            ops.append({"Data": [rng.randrange(256) for _ in range(rng.randint(0, 300))]})
        else:
            ops.append({"Copy": {"offset": rng.randrange(1 << 36) // 4096 * 4096, "size": 4096}})
    return json.dumps({"ops": ops, "source_size": 123456789, "block_size": 4096}, separators=(",", ":")).encode()


def _cases():
    rng = random.Random(1)
    yield "empty", b""
    yield "one", b"{"
    yield "rle", b"7" * 300000
    yield "raw-binary", bytes(rng.randrange(256) for _ in range(5000))
    yield "copies", delta_json(rng, 20000, 0.01)
    yield "literals", delta_json(rng, 3000, 0.9)
    yield "mixed", delta_json(rng, 8000, 0.3)
    yield "small", delta_json(rng, 3, 0.5)
    # the C5 shape: consecutive block Copies (offsets k * 8192), a literal block now and then
    c5 = [{"Copy": {"offset": k * 8192, "size": 8192}} if k % 97 else {"Data": [k % 256] * 300}
          for k in range(60000)]
    yield "c5-copies", json.dumps({"ops": c5, "source_size": 60000 * 8192, "block_size": 8192},
                                  separators=(",", ":")).encode()
    # block-size edges: 1023/1024 (one vs four streams), 128 KiB +- 1
    base = delta_json(rng, 20000, 0.5)
    for n in (1022, 1023, 1024, 1025, (128 << 10) - 1, 128 << 10, (128 << 10) + 1, 3 * (128 << 10)):
        yield f"len{n}", base[:n]
    # skewed: counts like a Fibonacci sequence force Huffman depths above 11 (folded back)
    fib = [1, 1]
    while len(fib) < 26:
        fib.append(fib[-1] + fib[-2])
    syms = b"".join(bytes([48 + i % 70]) * f for i, f in enumerate(fib))
    yield "fibonacci", bytes(random.Random(2).sample(syms, len(syms)))[:120000]
    yield "two-symbols", bytes(rng.choice(b"01") for _ in range(70000))
    yield "runs", b"".join(bytes([rng.randrange(40, 100)]) * rng.randint(1, 300) for _ in range(2000))
    yield "all-ascii", bytes(rng.randrange(128) for _ in range(200000))


@pytest.mark.skipif(shutil.which("g++") is None or _libzstd() is None or
                    not os.path.exists("/opt/rocm/include/hip/hip_runtime.h"),
                    reason="needs g++, the HIP headers and the system libzstd")
@pytest.mark.parametrize("case", list(_cases()), ids=lambda c: c[0])
def test_ref_frames_decode(case):
    name, data = case
    frame = ref_compress(data)
    assert frame[:4] == b"\x28\xb5\x2f\xfd"
    assert zstd_decode(frame, len(data)) == data
    # libzstd level 3 on the same texts: copies 0.181, literals 0.391, mixed 0.366, the C5
    # shape 0.047; here 0.169, 0.392, 0.364, 0.049 (candidate distances from the JSON
    # skeleton and sampled repeats, hash candidates, block-local repeat offsets: DESIGN.md §11)
    bound = {"copies": 0.175, "literals": 0.395, "mixed": 0.37, "c5-copies": 0.051}.get(name)
    if bound:
        assert len(frame) < bound * len(data), (name, len(frame) / len(data))
    if name == "rle":
        assert len(frame) < 64


@pytest.mark.skipif(shutil.which("g++") is None or _libzstd() is None, reason="needs g++ and libzstd")
def test_ref_random_texts():
    rng = np.random.default_rng(3)
    for it in range(60):
        n = int(rng.integers(0, 400000))
        alpha = int(rng.integers(2, 128))
        p = rng.dirichlet(np.full(alpha, float(rng.choice([0.05, 0.5, 5.0]))))
        data = rng.choice(alpha, size=n, p=p).astype(np.uint8).tobytes()
        assert zstd_decode(ref_compress(data), n) == data, it


@pytest.mark.skipif(shutil.which("g++") is None or _libzstd() is None, reason="needs g++ and libzstd")
def test_ref_structured_texts():
    """Texts built from a few repeated units (some cut short, some behind '{' or closed
    by '}', runs between them): matches at skeleton gaps, sampled repeat distances and
    hash distances, back-to-back matches (literal length 0) and repeat offsets in every
    form -- each frame decoded by libzstd."""
    rng = random.Random(5)
    for it in range(120):
        units = [bytes(rng.randrange(97, 97 + rng.randint(2, 20)) for _ in range(rng.randint(1, 60)))
                 for _ in range(rng.randint(1, 6))]
        target = rng.randint(1000, 300000)
        parts, size = [], 0
        while size < target:
            u = rng.choice(units)
            k = rng.random()
            if k < 0.3:
                piece = b"{" + u
            elif k < 0.5:
                piece = u[:rng.randint(0, len(u))]
            elif k < 0.6:
                piece = bytes([rng.randrange(256)]) * rng.randint(1, 9)
            else:
                piece = b"{" + u + b"}"
            parts.append(piece)
            size += len(piece)
        data = b"".join(parts)
        assert zstd_decode(ref_compress(data), len(data)) == data, it
