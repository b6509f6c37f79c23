"""Host-side mirror of nijaru/sy v0.0.43 ``src/delta``'s public API.

Same names, argument meaning and error behaviour as the Rust re-exports at
``src/delta/mod.rs:9-23``; the work is done by libsydelta.so (gfx950 HIP
kernels behind the C ABI in include/sydelta.h).  Errors surface as
``SyDeltaError`` (an ``OSError``), like the reference's ``io::Result``.

Reference functions and where they are mirrored:

=======================================  =====================================
``compute_checksums``  checksum.rs:31    ``compute_checksums``
``generate_delta_streaming`` gen.rs:67   ``generate_delta_streaming``
``generate_delta``     generator.rs:242  ``generate_delta``
``apply_delta``        applier.rs:22     ``apply_delta`` (host file I/O)
``calculate_block_size`` mod.rs:20       ``calculate_block_size``
``estimate_change_ratio`` ratio.rs:78    ``estimate_change_ratio`` (sampled blocks hashed
                                         on the device)
``Adler32``            rolling.rs:16     ``Adler32``
``BlockChecksum``/``Delta``/``DeltaOp``  dataclasses below
=======================================  =====================================
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field
from typing import Sequence, Union

from . import _lib
from ._lib import SyDeltaError, check, lib

MOD_ADLER = 65521


# ---------------------------------------------------------------------------
# types
# ---------------------------------------------------------------------------
@dataclass(frozen=True)
class BlockChecksum:
    """checksum.rs:9-21."""

    index: int
    offset: int
    size: int
    weak: int
    strong: int


@dataclass(frozen=True)
class Copy:
    """DeltaOp::Copy { offset, size } (generator.rs:12)."""

    offset: int
    size: int


@dataclass(frozen=True)
class Data:
    """DeltaOp::Data(Vec<u8>) (generator.rs:14)."""

    data: bytes


DeltaOp = Union[Copy, Data]


@dataclass
class Delta:
    """generator.rs:19-25."""

    ops: list = field(default_factory=list)
    source_size: int = 0
    block_size: int = 0

    def compression_ratio(self) -> float:
        """generator.rs:30-55."""
        lit = sum(len(o.data) for o in self.ops if isinstance(o, Data))
        cop = sum(o.size for o in self.ops if isinstance(o, Copy))
        tot = lit + cop
        return 1.0 if tot == 0 else lit / tot


@dataclass(frozen=True)
class DeltaStats:
    """applier.rs:9-13."""

    operations_count: int
    literal_bytes: int
    bytes_written: int


class Adler32:
    """rolling.rs:16-92 (host utility; the device computes the same values)."""

    def __init__(self, block_size: int):
        self.a, self.b, self.block_size = 1, 0, block_size

    @staticmethod
    def hash(data: bytes) -> int:
        buf = (ctypes.c_uint8 * len(data)).from_buffer_copy(data) if data else None
        return int(lib.sydelta_adler32_hash(buf, len(data)))

    def update_block(self, block: bytes) -> None:
        h = Adler32.hash(block)
        self.a, self.b = h & 0xFFFF, h >> 16

    def roll(self, old_byte: int, new_byte: int) -> None:
        n = self.block_size & 0xFFFFFFFF
        self.a = ((self.a + MOD_ADLER * 2 - old_byte + new_byte) & 0xFFFFFFFF) % MOD_ADLER
        n_old = ((n * old_byte) & 0xFFFFFFFF) % MOD_ADLER
        self.b = ((self.b + MOD_ADLER * 3 - n_old + self.a - 1) & 0xFFFFFFFF) % MOD_ADLER

    def digest(self) -> int:
        return (self.b << 16) | self.a

    def reset(self) -> None:
        self.a, self.b = 1, 0


def calculate_block_size(file_size: int) -> int:
    """mod.rs:20-23."""
    return int(lib.sydelta_calculate_block_size(file_size))


# ---------------------------------------------------------------------------
# conversions
# ---------------------------------------------------------------------------
def _sigs_to_c(sigs: Sequence[BlockChecksum]):
    arr = (_lib.BlockChecksumC * max(1, len(sigs)))()
    for i, c in enumerate(sigs):
        arr[i].index, arr[i].offset, arr[i].size = c.index, c.offset, c.size
        arr[i].weak, arr[i].strong = c.weak, c.strong
    return arr


def _delta_from_handle(h: ctypes.c_void_p, with_literals: bool = True) -> Delta:
    try:
        n = int(lib.sydelta_delta_num_ops(h))
        ops_p = lib.sydelta_delta_ops(h)
        ops = []
        for i in range(n):
            o = ops_p[i]
            if o.kind == _lib.OP_COPY:
                ops.append(Copy(int(o.a), int(o.b)))
            else:
                lp = lib.sydelta_delta_literal(h, i) if with_literals else None
                ops.append(Data(ctypes.string_at(lp, int(o.b)) if lp else b""))
        return Delta(ops, int(lib.sydelta_delta_source_size(h)), int(lib.sydelta_delta_block_size(h)))
    finally:
        lib.sydelta_delta_free(h)


def _pathb(p) -> bytes:
    return os.fsencode(os.fspath(p))


# ---------------------------------------------------------------------------
# src/delta public functions
# ---------------------------------------------------------------------------
def compute_checksums(path, block_size: int) -> list[BlockChecksum]:
    """checksum.rs:31-80 ``compute_checksums(path, block_size)``."""
    out = ctypes.POINTER(_lib.BlockChecksumC)()
    n = ctypes.c_uint64(0)
    check(lib.sydelta_compute_checksums(_pathb(path), block_size, ctypes.byref(out), ctypes.byref(n)))
    try:
        return [BlockChecksum(int(out[i].index), int(out[i].offset), int(out[i].size), int(out[i].weak),
                              int(out[i].strong)) for i in range(n.value)]
    finally:
        if out:
            lib.sydelta_checksums_free(ctypes.cast(out, ctypes.c_void_p))


def compute_checksums_bytes(data: bytes, block_size: int, device: int = -1) -> list[BlockChecksum]:
    """compute_checksums on an in-memory file image."""
    nb = -(-len(data) // block_size) if (data and block_size) else 0
    arr = (_lib.BlockChecksumC * max(1, nb))()
    got = ctypes.c_uint64(0)
    buf = ctypes.c_char_p(bytes(data)) if data else None
    check(lib.sydelta_compute_checksums_buf(device, ctypes.cast(buf, ctypes.c_void_p), len(data), block_size, arr,
                                            nb, ctypes.byref(got)))
    return [BlockChecksum(int(arr[i].index), int(arr[i].offset), int(arr[i].size), int(arr[i].weak),
                          int(arr[i].strong)) for i in range(got.value)]


def generate_delta_streaming(source_path, dest_checksums: Sequence[BlockChecksum], block_size: int) -> Delta:
    """generator.rs:67-228 ``generate_delta_streaming``."""
    h = ctypes.c_void_p()
    check(lib.sydelta_generate_delta_streaming(_pathb(source_path), _sigs_to_c(dest_checksums), len(dest_checksums),
                                               block_size, ctypes.byref(h)))
    return _delta_from_handle(h)


def generate_delta(source_path, dest_checksums: Sequence[BlockChecksum], block_size: int) -> Delta:
    """generator.rs:242-379 ``generate_delta``."""
    h = ctypes.c_void_p()
    check(lib.sydelta_generate_delta(_pathb(source_path), _sigs_to_c(dest_checksums), len(dest_checksums),
                                     block_size, ctypes.byref(h)))
    return _delta_from_handle(h)


def generate_delta_bytes(src: bytes, dest_checksums: Sequence[BlockChecksum], block_size: int,
                         device: int = -1) -> Delta:
    """generate_delta on an in-memory source."""
    h = ctypes.c_void_p()
    buf = ctypes.c_char_p(bytes(src)) if src else None
    check(lib.sydelta_generate_delta_buf(device, ctypes.cast(buf, ctypes.c_void_p), len(src),
                                         _sigs_to_c(dest_checksums), len(dest_checksums), block_size,
                                         ctypes.byref(h)))
    return _delta_from_handle(h)


def apply_delta(old_file, delta: Delta, new_file) -> DeltaStats:
    """applier.rs:22-56 (receiver side: seek/read the basis, write literals)."""
    literal = written = 0
    with open(old_file, "rb") as old, open(new_file, "wb") as new:
        for op in delta.ops:
            if isinstance(op, Copy):
                old.seek(op.offset)
                buf = old.read(op.size)
                if len(buf) != op.size:  # read_exact
                    raise SyDeltaError(_lib.SYDELTA_E_IO, "failed to fill whole buffer")
                new.write(buf)
                written += op.size
            else:
                new.write(op.data)
                literal += len(op.data)
                written += len(op.data)
    return DeltaStats(len(delta.ops), literal, written)


@dataclass(frozen=True)
class ChangeRatioResult:
    """ratio.rs:11-27."""

    change_ratio: float
    blocks_sampled: int
    blocks_changed: int
    use_delta: bool
    threshold: float

    def change_ratio_percent(self) -> str:
        """ratio.rs:47-50."""
        return f"{self.change_ratio * 100.0:.1f}%"


def estimate_change_ratio(source, dest, block_size: int, sample_count: int | None = None,
                          threshold: float | None = None) -> ChangeRatioResult:
    """ratio.rs:78-192: sample evenly spaced blocks of both files and compare their
    XXH3-64 (computed on the device); I/O errors raise SyDeltaError."""
    r = _lib.ChangeRatioC()
    check(lib.sydelta_estimate_change_ratio(_pathb(source), _pathb(dest), block_size,
                                            -1 if sample_count is None else sample_count,
                                            -1.0 if threshold is None else threshold, ctypes.byref(r)))
    return ChangeRatioResult(r.change_ratio, r.blocks_sampled, r.blocks_changed, bool(r.use_delta), r.threshold)
