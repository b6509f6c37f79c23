"""Wire formats of the delta path: serde_json's compact text of
Vec<BlockChecksum> (sy-remote.rs:146-147, ssh.rs:967-973) and of Delta
(ssh.rs:1003, sy-remote.rs:175), written and parsed by libsydelta (sydelta_wire.cpp;
the Delta writer also on the device)."""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import check, lib

_OP_DTYPE = np.dtype([("kind", "<u4"), ("reserved", "<u4"), ("a", "<u8"), ("b", "<u8")])
_SIG_DTYPE = np.dtype([("index", "<u8"), ("offset", "<u8"), ("size", "<u8"), ("weak", "<u4"),
                       ("reserved", "<u4"), ("strong", "<u8")])


def sig_array(index, offset, size, weak, strong) -> np.ndarray:
    a = np.zeros(len(index), dtype=_SIG_DTYPE)
    a["index"], a["offset"], a["size"], a["weak"], a["strong"] = index, offset, size, weak, strong
    return a


def checksums_to_json(sigs: np.ndarray) -> bytes:
    """sigs: structured array (sig_array)."""
    sigs = np.ascontiguousarray(sigs, dtype=_SIG_DTYPE)
    n = lib.sydelta_checksums_to_json(sigs.ctypes.data if len(sigs) else None, len(sigs), None, 0)
    buf = ctypes.create_string_buffer(n)
    lib.sydelta_checksums_to_json(sigs.ctypes.data if len(sigs) else None, len(sigs), buf, n)
    return buf.raw[:n]


def checksums_from_json(text: bytes) -> np.ndarray:
    out = ctypes.POINTER(_lib.BlockChecksumC)()
    n = ctypes.c_uint64()
    check(lib.sydelta_checksums_from_json(text, len(text), ctypes.byref(out), ctypes.byref(n)))
    try:
        if not n.value:
            return np.zeros(0, dtype=_SIG_DTYPE)
        raw = ctypes.string_at(out, n.value * _SIG_DTYPE.itemsize)
        return np.frombuffer(raw, dtype=_SIG_DTYPE).copy()
    finally:
        if n.value:
            lib.sydelta_checksums_free(out)


def _delta_handle(kind, a, b, source_size: int, block_size: int):
    n = len(kind)
    ops = np.zeros(n, dtype=_OP_DTYPE)
    if n:
        ops["kind"], ops["a"], ops["b"] = kind, a, b
    h = lib.sydelta_delta_from_ops(ops.ctypes.data if n else None, n, source_size, block_size)
    if not h:
        raise ValueError("bad op array")
    return h


def delta_to_json(kind, a, b, source_size: int, block_size: int, lit: bytes | np.ndarray) -> bytes:
    """Delta text from an op table whose Data ops index `lit` (host bytes)."""
    lit = np.ascontiguousarray(np.frombuffer(bytes(lit), dtype=np.uint8) if isinstance(lit, (bytes, bytearray))
                               else lit, dtype=np.uint8)
    h = _delta_handle(kind, a, b, source_size, block_size)
    try:
        n = ctypes.c_uint64()
        lp = lit.ctypes.data if lit.size else ctypes.c_void_p(1)  # non-NULL: use lit even when empty
        check(lib.sydelta_delta_to_json(h, lp, lit.size, None, 0, ctypes.byref(n)))
        buf = ctypes.create_string_buffer(n.value)
        check(lib.sydelta_delta_to_json(h, lp, lit.size, buf, n.value, ctypes.byref(n)))
        return buf.raw[:n.value]
    finally:
        lib.sydelta_delta_free(h)


def delta_to_json_device(kind, a, b, source_size: int, block_size: int, d_lit, stream=None):
    """The same text written on the device from literal bytes in HBM (torch uint8
    tensor); returns the text as a uint8 device tensor."""
    import torch

    from .device import _ptr, _stream

    h = _delta_handle(kind, a, b, source_size, block_size)
    try:
        n = ctypes.c_uint64()
        check(lib.sydelta_delta_to_json_device(h, _ptr(d_lit), d_lit.numel(), None, 0, ctypes.byref(n),
                                               _stream(stream)))
        out = torch.empty(n.value + 16, dtype=torch.uint8, device=d_lit.device)
        check(lib.sydelta_delta_to_json_device(h, _ptr(d_lit), d_lit.numel(), _ptr(out), out.numel(),
                                               ctypes.byref(n), _stream(stream)))
        return out[:n.value]
    finally:
        lib.sydelta_delta_free(h)


def checksums_to_json_device(d_weak, d_strong, block_size: int, last_size: int, stream=None):
    """serde_json::to_string(&Vec<BlockChecksum>) of a signature in HBM (the weak/strong
    tensors of device.signature), written on the device (sy-remote.rs:146-147); returns
    the text as a uint8 device tensor."""
    import torch

    from .device import _ptr, _stream

    nb = d_weak.numel()
    if d_strong.numel() != nb:
        raise ValueError("weak and strong arrays differ in length")
    n = ctypes.c_uint64()
    wp, sp = (_ptr(d_weak), _ptr(d_strong)) if nb else (None, None)
    check(lib.sydelta_checksums_to_json_device(wp, sp, nb, block_size, last_size, None, 0, ctypes.byref(n),
                                               _stream(stream)))
    out = torch.empty(n.value + 16, dtype=torch.uint8, device=d_weak.device)
    check(lib.sydelta_checksums_to_json_device(wp, sp, nb, block_size, last_size, _ptr(out), out.numel(),
                                               ctypes.byref(n), _stream(stream)))
    return out[:n.value]


def checksums_from_json_device(d_text, stream=None):
    """serde_json::from_str::<Vec<BlockChecksum>> of a compact text in HBM (uint8 device
    tensor) parsed on the device; returns the entries as a uint8 device tensor of
    n * 40 bytes (sydelta_block_checksum records) and n.  Raises SyDeltaError for text in
    any other spelling (parse that with checksums_from_json)."""
    import torch

    from .device import _ptr, _stream

    n = ctypes.c_uint64()
    check(lib.sydelta_checksums_from_json_device(_ptr(d_text), d_text.numel(), None, 0, ctypes.byref(n),
                                                 _stream(stream)))
    out = torch.empty(max(1, n.value) * _SIG_DTYPE.itemsize, dtype=torch.uint8, device=d_text.device)
    check(lib.sydelta_checksums_from_json_device(_ptr(d_text), d_text.numel(), _ptr(out), n.value, ctypes.byref(n),
                                                 _stream(stream)))
    return out[:n.value * _SIG_DTYPE.itemsize], n.value


def delta_from_json_device(d_text, stream=None):
    """serde_json::from_str::<Delta> of a compact Delta JSON text in HBM (uint8 device
    tensor) parsed on the device: returns (ops as [(kind, a, b)] with Data ops indexing the
    literal tensor, the literal bytes as a uint8 device tensor, source_size, block_size).
    Raises SyDeltaError for text in any other spelling (parse that with delta_from_json)."""
    import torch

    from .device import _ptr, _stream

    n = ctypes.c_uint64()
    check(lib.sydelta_delta_from_json_device(_ptr(d_text), d_text.numel(), None, 0, ctypes.byref(n), None,
                                             _stream(stream)))
    lit = torch.empty(max(1, n.value), dtype=torch.uint8, device=d_text.device)
    h = ctypes.c_void_p()
    check(lib.sydelta_delta_from_json_device(_ptr(d_text), d_text.numel(), _ptr(lit), lit.numel(), ctypes.byref(n),
                                             ctypes.byref(h), _stream(stream)))
    try:
        cnt = lib.sydelta_delta_num_ops(h)
        ops_p = lib.sydelta_delta_ops(h)
        ops = [(int(ops_p[i].kind), int(ops_p[i].a), int(ops_p[i].b)) for i in range(cnt)]
        return ops, lit[:n.value], int(lib.sydelta_delta_source_size(h)), int(lib.sydelta_delta_block_size(h))
    finally:
        lib.sydelta_delta_free(h)


def zstd_compress_device(d_text, stream=None, device: int | None = None):
    """zstd frame (Huffman literals, FSE-coded sequences) of the bytes of a uint8 device tensor, as a uint8
    device tensor: the compression ssh.rs:1009-1017 applies to the Delta JSON.  The
    tensor must start 16-byte aligned (torch allocations and views at offset 0 do)."""
    import torch

    from .device import _ptr, _stream

    if device is None:
        device = d_text.device.index or 0
    n = d_text.numel()
    out = torch.empty(int(lib.sydelta_zstd_bound(n)) + 16, dtype=torch.uint8, device=d_text.device)
    got = ctypes.c_uint64()
    check(lib.sydelta_zstd_compress_device(device, _ptr(d_text) if n else None, n, _ptr(out), out.numel(),
                                           ctypes.byref(got), _stream(stream)))
    return out[:got.value]


def delta_from_json(text: bytes):
    """-> (ops as [("C", offset, size) | ("D", literal bytes)], source_size, block_size)."""
    h = ctypes.c_void_p()
    check(lib.sydelta_delta_from_json(text, len(text), ctypes.byref(h)))
    try:
        nops = int(lib.sydelta_delta_num_ops(h))
        ops = []
        for i in range(nops):
            o = lib.sydelta_delta_ops(h)[i]
            if o.kind == _lib.OP_COPY:
                ops.append(("C", int(o.a), int(o.b)))
            else:
                p = lib.sydelta_delta_literal(h, i)
                ops.append(("D", ctypes.string_at(p, int(o.b)) if o.b else b""))
        return ops, int(lib.sydelta_delta_source_size(h)), int(lib.sydelta_delta_block_size(h))
    finally:
        lib.sydelta_delta_free(h)
