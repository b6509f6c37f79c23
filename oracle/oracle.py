"""CPU oracle for sy's delta hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may
import this module, and only as the checker (or the reported CPU baseline).
The product path (``sy_amd``) never imports it and fails loudly when its HIP
library is missing.

Two restatements of nijaru/sy v0.0.43 ``src/delta`` live here:

* a pure-Python one (``py_*``), line-by-line after the Rust source, used for
  small cases and to generate the golden fixtures (tests/golden/make_golden.py);
* ``C`` — a ctypes handle to ``oracle/liboracle.so`` built from
  ``oracle/sydelta_oracle.c`` (same rules, fast enough for MiB-sized parity
  cases and for the CPU baseline).

Primitive pins: Adler-32 is checked against ``zlib.adler32``;
XXH3-64 (crate xxhash-rust 0.8.15, not vendored in the reference) is checked
against python-xxhash 3.8.1 (libxxhash 0.8.2), whose XXH3 output is frozen
since xxHash 0.8.0.  The reference itself (Rust) cannot be built here, so the
op-list semantics are pinned by the reference's own unit-test expectations and
the worked examples of SURVEY.md Appendix B (tests/golden/).
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess
from dataclasses import dataclass

import numpy as np

MOD_ADLER = 65521  # rolling.rs:22
HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


# --------------------------------------------------------------------------
# rolling.rs
# --------------------------------------------------------------------------
def py_adler32(data: bytes) -> int:
    """Adler32::hash, rolling.rs:35-45."""
    a, b = 1, 0
    for x in data:
        a = (a + x) % MOD_ADLER
        b = (b + a) % MOD_ADLER
    return (b << 16) | a


class PyAdler32:
    """struct Adler32, rolling.rs:16-91 (u32 wrap semantics kept)."""

    def __init__(self, block_size: int):  # :26-32
        self.a, self.b, self.block_size = 1, 0, block_size

    def update_block(self, block: bytes):  # :48-56
        self.a, self.b = 1, 0
        for x in block:
            self.a = (self.a + x) % MOD_ADLER
            self.b = (self.b + self.a) % MOD_ADLER

    def roll(self, old: int, new: int):  # :66-79
        n = self.block_size & 0xFFFFFFFF
        self.a = ((self.a + MOD_ADLER * 2 - old + new) & 0xFFFFFFFF) % MOD_ADLER
        n_old = ((n * old) & 0xFFFFFFFF) % MOD_ADLER
        self.b = ((self.b + MOD_ADLER * 3 - n_old + self.a - 1) & 0xFFFFFFFF) % MOD_ADLER

    def digest(self) -> int:  # :82-84
        return (self.b << 16) | self.a

    def reset(self):  # :88-91
        self.a, self.b = 1, 0


def py_xxh3(data: bytes) -> int:
    """Strong hash: xxhash_rust::xxh3::Xxh3 digest (seed 0). python-xxhash is the
    independent pin of the third-party primitive (see module docstring)."""
    import xxhash

    return xxhash.xxh3_64_intdigest(data)


# --------------------------------------------------------------------------
# mod.rs / checksum.rs
# --------------------------------------------------------------------------
def py_calculate_block_size(file_size: int) -> int:
    """mod.rs:20-23: (file_size as f64).sqrt() as usize, clamped to 512..=128 KiB."""
    s = int(math.sqrt(float(file_size)))
    return min(max(s, 512), 128 * 1024)


@dataclass(frozen=True)
class BlockChecksum:
    """checksum.rs:9-21."""

    index: int
    offset: int
    size: int
    weak: int
    strong: int


def py_compute_checksums(data: bytes, block_size: int) -> list[BlockChecksum]:
    """checksum.rs:31-80 on an in-memory file image."""
    if len(data) == 0:  # :36-38
        return []
    n = -(-len(data) // block_size)  # div_ceil, :41
    out = []
    for i in range(n):  # rayon collect keeps index order
        off = i * block_size
        blk = data[off : off + block_size]
        out.append(BlockChecksum(i, off, len(blk), py_adler32(blk), py_xxh3(blk)))
    return out


# Ops: ("C", offset, size) for DeltaOp::Copy, ("D", new_offset, length) for DeltaOp::Data.
def _candidate_map(sigs):
    m: dict[int, list] = {}
    for c in sigs:  # generator.rs:75-81 — Vec in input (index) order
        m.setdefault(c.weak, []).append(c)
    return m


def py_generate_delta(src: bytes, sigs: list[BlockChecksum], bs: int):
    """generator.rs:242-379 (in-memory).  Returns list of op tuples."""
    m = _candidate_map(sigs)
    if len(src) == 0:
        return []
    ops = []
    lit_start, lit_len, pos = 0, 0, 0
    r = PyAdler32(bs)
    if len(src) >= bs:
        r.update_block(src[0:bs])
    L = len(src)
    while pos < L:
        found = False
        remaining = L - pos
        if remaining >= bs:
            cands = m.get(r.digest())
            if cands:
                strong = py_xxh3(src[pos : pos + bs])
                for c in cands:
                    if c.strong == strong:  # no size check, :299
                        if lit_len:
                            ops.append(("D", lit_start, lit_len))
                            lit_len = 0
                        ops.append(("C", c.offset, c.size))
                        pos += bs
                        found = True
                        if pos + bs <= L:
                            r.update_block(src[pos : pos + bs])
                        break
        else:
            part = src[pos:]
            cands = m.get(py_adler32(part))
            if cands:
                strong = py_xxh3(part)
                for c in cands:
                    if c.size == len(part) and c.strong == strong:
                        if lit_len:
                            ops.append(("D", lit_start, lit_len))
                            lit_len = 0
                        ops.append(("C", c.offset, c.size))
                        pos += len(part)
                        found = True
                        break
        if not found:
            if not lit_len:
                lit_start = pos
            lit_len += 1
            pos += 1
            if pos > 0 and pos + bs - 1 < L:
                r.roll(src[pos - 1], src[pos + bs - 1])
    if lit_len:
        ops.append(("D", lit_start, lit_len))
    return ops


def py_generate_delta_streaming(src: bytes, sigs: list[BlockChecksum], bs: int, chunk: int = 256 * 1024):
    """generator.rs:67-228 with CHUNK_SIZE = ``chunk`` (reference: 256 KiB)."""
    m = _candidate_map(sigs)
    L = len(src)
    if L == 0:
        return []
    ops = []
    fpos = 0
    first = src[fpos : fpos + chunk]
    bytes_read = len(first)
    fpos += bytes_read
    wbase, window = 0, bytearray(first)
    r = PyAdler32(bs)
    if len(window) >= bs:
        r.update_block(bytes(window[0:bs]))
    wpos = 0
    lit_start, lit_len = 0, 0
    while wpos < len(window):
        remaining = len(window) - wpos
        found = False
        if remaining >= bs:
            cands = m.get(r.digest())
            if cands:
                strong = py_xxh3(bytes(window[wpos : wpos + bs]))
                for c in cands:
                    if c.strong == strong:
                        if lit_len:
                            ops.append(("D", lit_start, lit_len))
                            lit_len = 0
                        ops.append(("C", c.offset, c.size))
                        wpos += bs
                        found = True
                        if wpos + bs <= len(window):
                            r.update_block(bytes(window[wpos : wpos + bs]))
                        break
        elif remaining > 0:
            part = bytes(window[wpos:])
            cands = m.get(py_adler32(part))
            if cands:
                strong = py_xxh3(part)
                for c in cands:
                    if c.size == len(part) and c.strong == strong:
                        if lit_len:
                            ops.append(("D", lit_start, lit_len))
                            lit_len = 0
                        ops.append(("C", c.offset, c.size))
                        wpos += len(part)
                        found = True
                        break
        if not found and wpos < len(window):
            if not lit_len:
                lit_start = wbase + wpos
            lit_len += 1
            if wpos + bs < len(window):
                r.roll(window[wpos], window[wpos + bs])
            wpos += 1
        if wpos >= bs and bytes_read > 0 and len(window) - wpos < bs:
            del window[0:wpos]
            wbase += wpos
            wpos = 0
            nxt = src[fpos : fpos + chunk]
            bytes_read = len(nxt)
            fpos += bytes_read
            if bytes_read > 0:
                window.extend(nxt)
                if len(window) >= bs:
                    r.update_block(bytes(window[0:bs]))
    if lit_len:
        ops.append(("D", lit_start, lit_len))
    return ops


def py_apply_delta(basis: bytes, src: bytes, ops) -> bytes:
    """applier.rs:22-56 on buffers (Data descriptors index the source)."""
    out = bytearray()
    for k, a, b in ops:
        if k == "C":
            if a + b > len(basis):
                raise ValueError("read_exact past end of basis")
            out += basis[a : a + b]
        else:
            out += src[a : a + b]
    return bytes(out)


def compression_ratio(ops) -> float:
    """Delta::compression_ratio, generator.rs:30-55."""
    lit = sum(b for k, a, b in ops if k == "D")
    cop = sum(b for k, a, b in ops if k == "C")
    tot = lit + cop
    return 1.0 if tot == 0 else lit / tot


# --------------------------------------------------------------------------
# Synthetic inputs: counter-based splitmix64 (parallel-friendly stand-in for §8d PRNG)
# --------------------------------------------------------------------------
def splitmix_words(idx: np.ndarray, seed: int) -> np.ndarray:
    """Counter-based splitmix64 of (seed, idx) (sydelta_device.hpp splitmix_word)."""
    idx = np.asarray(idx, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = idx * np.uint64(0x9E3779B97F4A7C15) + np.uint64(seed & 0xFFFFFFFFFFFFFFFF) * np.uint64(0xD1B54A32D192ED03)
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def synth_bytes(n: int, seed: int, first: int = 0) -> np.ndarray:
    """Deterministic uniform bytes [first, first + n) of the stream; identical to
    sy_amd's device generator (counter-based splitmix64 of (seed, word index),
    little-endian words).  first must be a multiple of 8."""
    assert first % 8 == 0
    nw = (n + 7) // 8
    z = splitmix_words(np.arange(first // 8, first // 8 + nw, dtype=np.uint64), seed)
    return z.view(np.uint8)[:n].copy()


def synth_edit_blocks(src: np.ndarray, first: int, bs: int, seed: int, rate_ppm: int) -> np.ndarray:
    """BASELINE C5 edit model (sydelta_synth_mutate_blocks): in each selected
    block-aligned block one byte is replaced by a different byte."""
    out = np.array(src, dtype=np.uint8, copy=True)
    nb = -(-len(out) // bs)
    k = np.arange(first // bs, first // bs + nb, dtype=np.uint64)
    r = splitmix_words(k, seed)
    thresh = (rate_ppm << 32) // 1000000
    sel = np.nonzero((r & np.uint64(0xFFFFFFFF)) < np.uint64(thresh))[0]
    for t in sel:
        o = int(t) * bs + int(r[t] >> np.uint64(32)) % bs
        if o < len(out):
            x = 1 + int(splitmix_words(np.array([k[t]], dtype=np.uint64), ~seed & 0xFFFFFFFFFFFFFFFF)[0]) % 255
            out[o] ^= x
    return out


# --------------------------------------------------------------------------
# C oracle (ctypes)
# --------------------------------------------------------------------------
def build_c(force: bool = False) -> str:
    src = os.path.join(HERE, "sydelta_oracle.c")
    if force or not os.path.exists(LIB_PATH) or os.path.getmtime(LIB_PATH) < os.path.getmtime(src):
        subprocess.check_call(
            ["gcc", "-O3", "-march=x86-64-v2", "-fPIC", "-shared", "-o", LIB_PATH, src, "-lm", "-lpthread"]
        )
    return LIB_PATH


class _C:
    def __init__(self):
        build_c()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        u32p = ctypes.POINTER(ctypes.c_uint32)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.oracle_adler32.restype = ctypes.c_uint32
        L.oracle_adler32.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.oracle_xxh3_64.restype = ctypes.c_uint64
        L.oracle_xxh3_64.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.oracle_calculate_block_size.restype = ctypes.c_uint64
        L.oracle_calculate_block_size.argtypes = [ctypes.c_uint64]
        L.oracle_compute_checksums.restype = ctypes.c_uint64
        L.oracle_compute_checksums.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.oracle_compute_checksums_file.restype = ctypes.c_int64
        L.oracle_compute_checksums_file.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_void_p,
                                                    ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
        gd_args = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                   ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]
        L.oracle_generate_delta.restype = ctypes.c_int64
        L.oracle_generate_delta.argtypes = gd_args + [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_generate_delta_streaming.restype = ctypes.c_int64
        L.oracle_generate_delta_streaming.argtypes = gd_args + [ctypes.c_uint64] + [ctypes.c_void_p] * 3 + \
            [ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_apply_delta.restype = ctypes.c_int64
        L.oracle_apply_delta.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                         ctypes.c_uint64]
        self.L = L
        del u8p, u32p, u64p

    @staticmethod
    def _buf(data):
        arr = np.frombuffer(data, dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else np.ascontiguousarray(data, dtype=np.uint8)
        return arr, arr.ctypes.data if arr.size else None

    def adler32(self, data) -> int:
        arr, p = self._buf(data)
        return int(self.L.oracle_adler32(p, arr.size))

    def xxh3(self, data) -> int:
        arr, p = self._buf(data)
        return int(self.L.oracle_xxh3_64(p, arr.size))

    def calculate_block_size(self, n: int) -> int:
        return int(self.L.oracle_calculate_block_size(n))

    def compute_checksums(self, data, bs: int, threads: int = 1):
        """Returns (weak u32[], strong u64[], size u64[]) numpy arrays."""
        arr, p = self._buf(data)
        n = -(-arr.size // bs) if arr.size else 0
        weak = np.zeros(max(n, 1), np.uint32)
        strong = np.zeros(max(n, 1), np.uint64)
        size = np.zeros(max(n, 1), np.uint64)
        got = self.L.oracle_compute_checksums(p, arr.size, bs, weak.ctypes.data, strong.ctypes.data,
                                              size.ctypes.data, threads)
        assert got == n
        return weak[:n], strong[:n], size[:n]

    def generate_delta(self, src, weak, strong, size, bs: int, streaming: bool = False,
                       chunk: int = 256 * 1024, stats=None):
        """Returns (kind u8[], a u64[], b u64[]) — kind 0 = Copy{a=offset,b=size}, 1 = Data{a=src off,b=len}."""
        arr, p = self._buf(src)
        weak = np.ascontiguousarray(weak, np.uint32)
        strong = np.ascontiguousarray(strong, np.uint64)
        size = np.ascontiguousarray(size, np.uint64)
        n = weak.size
        bsz = np.uint64(bs)
        offset = np.arange(n, dtype=np.uint64) * bsz
        cap = max(16, arr.size // max(1, min(bs, 1 << 20)) * 2 + 16)
        st = np.zeros(2, np.uint64)
        while True:
            kind = np.zeros(cap, np.uint8)
            a = np.zeros(cap, np.uint64)
            b = np.zeros(cap, np.uint64)
            wp = lambda x: x.ctypes.data if x.size else None
            common = (p, arr.size, wp(weak), wp(strong), wp(offset), wp(size), n, bs)
            if streaming:
                got = self.L.oracle_generate_delta_streaming(*common, chunk, kind.ctypes.data, a.ctypes.data,
                                                             b.ctypes.data, cap, st.ctypes.data)
            else:
                got = self.L.oracle_generate_delta(*common, kind.ctypes.data, a.ctypes.data, b.ctypes.data, cap,
                                                   st.ctypes.data)
            if got < 0:
                raise MemoryError("oracle generate_delta failed")
            if got <= cap:
                if stats is not None:
                    stats["strong_full"] = int(st[0])
                    stats["strong_tail"] = int(st[1])
                return kind[:got], a[:got], b[:got]
            cap = int(got)


_C_INSTANCE = None


def C() -> _C:
    global _C_INSTANCE
    if _C_INSTANCE is None:
        _C_INSTANCE = _C()
    return _C_INSTANCE


def ops_from_arrays(kind, a, b):
    return [("C" if int(k) == 0 else "D", int(x), int(y)) for k, x, y in zip(kind, a, b)]


# --------------------------------------------------------------------------
# Local path: block compare + change-ratio sampling
# --------------------------------------------------------------------------
def py_block_compare(src: bytes, dst: bytes, bs: int):
    """local.rs:541-619 (and :682-760): read block k of both files (full reads of a
    regular file: src_read = min(bs, |src| - k*bs), dst_read likewise, 0 past the end);
    a block matches iff the reads are equal in length and content.  Returns
    (changed flags per source block, changed_blocks, literal_bytes, bytes_written)."""
    flags = []
    literal = 0
    off = 0
    while off < len(src):
        s = src[off:off + bs]
        d = dst[off:off + bs]
        changed = not (len(s) == len(d) and s == d)
        flags.append(1 if changed else 0)
        if changed:
            literal += len(s)
        off += len(s)
    return flags, sum(flags), literal, len(src)


def py_estimate_change_ratio(src: bytes, dst: bytes, bs: int, sample_count=None, threshold=None):
    """ratio.rs:78-192 `estimate_change_ratio` on in-memory bytes (regular-file reads
    are full).  Returns (change_ratio, blocks_sampled, blocks_changed, use_delta,
    threshold)."""
    sample_count = 20 if sample_count is None else sample_count
    threshold = 0.75 if threshold is None else threshold
    ssize, dsize = len(src), len(dst)
    total_blocks = -(-dsize // bs)
    sample_count = min(sample_count, total_blocks)
    size_diff = abs(ssize - dsize) / dsize if dsize > 0 else 1.0
    if size_diff > 0.5:
        r = min(size_diff, 1.0)
        return r, 0, 0, r <= threshold, threshold
    step = total_blocks // (sample_count - 1) if sample_count > 1 else 0
    pos = [min(i * step, max(total_blocks - 1, 0)) if sample_count > 1 else 0 for i in range(sample_count)]
    changed = 0
    for k in pos:
        off = k * bs
        s = src[off:off + bs]
        d = dst[off:off + bs]
        if len(s) != len(d):
            changed += 1
            continue
        if py_xxh3(s) != py_xxh3(d):
            changed += 1
    ratio = changed / sample_count if sample_count > 0 else 0.0
    return ratio, sample_count, changed, ratio <= threshold, threshold


# --------------------------------------------------------------------------
# integrity/xxhash3.rs
# --------------------------------------------------------------------------
def py_hash_file(data: bytes, chunk: int = 1 << 20) -> int:
    """XxHash3Hasher::hash_file (integrity/xxhash3.rs:17-33): Xxh3::new(), update with
    1 MiB reads, digest.  Streamed through python-xxhash's XXH3 state, the independent
    pin of xxhash-rust 0.8.15's Xxh3 (module docstring)."""
    import xxhash

    h = xxhash.xxh3_64()
    for o in range(0, len(data), chunk):
        h.update(data[o:o + chunk])
    return h.intdigest()
