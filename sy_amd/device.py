"""Device-resident entry points (HBM buffers held by torch tensors).

torch is plumbing here: it owns the device memory and the stream; every
computation is a libsydelta.so kernel.  Used by bench.py and the GPU tests.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from ._lib import check, lib


def _stream(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)


def _ptr(t: torch.Tensor) -> int:
    assert t.is_cuda and t.is_contiguous()
    return t.data_ptr()


def signature(buf: torch.Tensor, block_size: int, stream=None):
    """compute_checksums' per-block loop on a device buffer -> (weak int32[n], strong int64[n])
    (bit patterns of u32 / u64)."""
    assert buf.dtype == torch.uint8
    n = buf.numel()
    nb = -(-n // block_size) if n else 0
    weak = torch.empty(max(nb, 1), dtype=torch.int32, device=buf.device)
    strong = torch.empty(max(nb, 1), dtype=torch.int64, device=buf.device)
    check(lib.sydelta_signature_device(buf.device.index or 0, _ptr(buf) if n else None, n, block_size,
                                       _ptr(weak), _ptr(strong), _stream(stream)))
    return weak[:nb], strong[:nb]


def signature_batch(buf: torch.Tensor, offs, lens, block_size: int, stream=None):
    """Batched signature over many files packed in one device buffer."""
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    total = int(((lens + np.uint64(block_size - 1)) // np.uint64(block_size)).sum()) if len(lens) else 0
    weak = torch.empty(max(total, 1), dtype=torch.int32, device=buf.device)
    strong = torch.empty(max(total, 1), dtype=torch.int64, device=buf.device)
    check(lib.sydelta_signature_batch_device(buf.device.index or 0, _ptr(buf), offs.ctypes.data, lens.ctypes.data,
                                             len(lens), block_size, _ptr(weak), _ptr(strong), _stream(stream)))
    return weak[:total], strong[:total]


class Index:
    """Device probe table for a basis signature (generator.rs:75-81)."""

    def __init__(self, weak, strong, block_size: int, last_size: int, device: int = 0, stream=None):
        self.h = ctypes.c_void_p()
        n = int(weak.numel()) if isinstance(weak, torch.Tensor) else len(weak)
        self.nblocks, self.block_size, self.last_size = n, block_size, last_size
        if isinstance(weak, torch.Tensor) and weak.is_cuda:
            check(lib.sydelta_index_create(device, _ptr(weak) if n else None, _ptr(strong) if n else None, n,
                                           block_size, last_size, 1, _stream(stream), ctypes.byref(self.h)))
        else:
            w = np.ascontiguousarray(np.asarray(weak, dtype=np.uint64).astype(np.uint32))
            s = np.ascontiguousarray(np.asarray(strong, dtype=np.uint64))
            check(lib.sydelta_index_create(device, w.ctypes.data if n else None, s.ctypes.data if n else None, n,
                                           block_size, last_size, 0, None, ctypes.byref(self.h)))

    def close(self):
        if self.h:
            lib.sydelta_index_free(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BatchIndex(Index):
    """Per-file probe tables for a batch of basis signatures (concatenated in file
    order, as signature_batch returns them)."""

    def __init__(self, weak: torch.Tensor, strong: torch.Tensor, nblocks, last_sizes, block_size: int,
                 device: int = 0, stream=None):
        self.h = ctypes.c_void_p()
        nb = np.ascontiguousarray(nblocks, dtype=np.uint64)
        ls = np.ascontiguousarray(last_sizes, dtype=np.uint64)
        self.nfiles, self.block_size = len(nb), block_size
        n = int(nb.sum())
        check(lib.sydelta_index_create_batch(device, _ptr(weak) if n else None, _ptr(strong) if n else None,
                                             nb.ctypes.data, ls.ctypes.data, len(nb), block_size, 1,
                                             _stream(stream), ctypes.byref(self.h)))


@dataclass
class DeviceDelta:
    kind: np.ndarray   # 0 Copy, 1 Data
    a: np.ndarray      # Copy: basis offset; Data: source offset
    b: np.ndarray      # size / length
    source_size: int
    block_size: int
    stats: dict
    handle: object = None  # the library's sydelta_delta (when the ops are its zero-copy view)

    def tuples(self):
        return [("C" if int(k) == 0 else "D", int(x), int(y)) for k, x, y in zip(self.kind, self.a, self.b)]


_OP_DTYPE = np.dtype([("kind", "<u4"), ("reserved", "<u4"), ("a", "<u8"), ("b", "<u8")])


class _DeltaHandle:
    """Owns a sydelta_delta* whose op array numpy views borrow."""

    def __init__(self, h):
        self.h = h

    def __del__(self):
        try:
            lib.sydelta_delta_free(self.h)
        except Exception:
            pass


def _device_delta(h, owner=None) -> DeviceDelta:
    nops = int(lib.sydelta_delta_num_ops(h))
    if nops:
        p = lib.sydelta_delta_ops(h)
        if owner is not None:  # zero-copy view of the library's sydelta_op array
            buf = (ctypes.c_uint8 * (24 * nops)).from_address(ctypes.addressof(p.contents))
            buf._owner = owner  # the handle is freed when the last view goes away
            raw = np.frombuffer(buf, dtype=_OP_DTYPE)
        else:
            raw = np.frombuffer((ctypes.c_uint8 * (24 * nops)).from_address(ctypes.addressof(p.contents)),
                                dtype=_OP_DTYPE).copy()
        kind, a, b = raw["kind"], raw["a"], raw["b"]
    else:
        kind = np.zeros(0, np.uint8)
        a = np.zeros(0, np.uint64)
        b = np.zeros(0, np.uint64)
    st = _lib.MatchStatsC()
    check(lib.sydelta_delta_stats(h, ctypes.byref(st)))
    stats = {f: int(getattr(st, f)) for f, _ in _lib.MatchStatsC._fields_}
    return DeviceDelta(kind, a, b, int(lib.sydelta_delta_source_size(h)), int(lib.sydelta_delta_block_size(h)), stats,
                       owner)


class DeltaBatch:
    """The library's per-file deltas of one batched match (sydelta_delta_batch), kept
    in host memory until freed; `delta(f)` / `deltas()` copy them out on demand."""

    def __init__(self, h):
        self.h = h
        self.count = int(lib.sydelta_delta_batch_count(h))
        st = _lib.MatchStatsC()
        check(lib.sydelta_delta_batch_stats(h, ctypes.byref(st)))
        self.stats = {f: int(getattr(st, f)) for f, _ in _lib.MatchStatsC._fields_}

    def delta(self, f: int) -> DeviceDelta:
        return _device_delta(lib.sydelta_delta_batch_get(self.h, f))

    def deltas(self) -> list:
        return [self.delta(f) for f in range(self.count)]

    def close(self):
        if self.h:
            lib.sydelta_delta_batch_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def match_batch_handle(index: BatchIndex, buf: torch.Tensor, offs, lens, stream=None) -> DeltaBatch:
    """Batched rolling match: source f = buf[offs[f] : offs[f]+lens[f]] against basis f,
    results left in the library (DeltaBatch)."""
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint64)
    h = ctypes.c_void_p()
    check(lib.sydelta_match_batch_device(index.h, _ptr(buf), offs.ctypes.data, lens.ctypes.data, len(lens),
                                         _stream(stream), ctypes.byref(h)))
    return DeltaBatch(h)


def delta_pairs_handle(basis: torch.Tensor, boffs, blens, src: torch.Tensor, soffs, slens, block_size: int,
                       stream=None) -> DeltaBatch:
    """Signature + match of every (basis f, source f) pair in one call (sydelta_delta_pairs_device);
    results left in the library (DeltaBatch)."""
    arrs = [np.ascontiguousarray(x, dtype=np.uint64) for x in (boffs, blens, soffs, slens)]
    h = ctypes.c_void_p()
    check(lib.sydelta_delta_pairs_device(basis.device.index or 0, _ptr(basis), arrs[0].ctypes.data, arrs[1].ctypes.data,
                                         _ptr(src), arrs[2].ctypes.data, arrs[3].ctypes.data, len(arrs[3]), block_size,
                                         _stream(stream), ctypes.byref(h)))
    return DeltaBatch(h)


def delta_pairs(basis: torch.Tensor, boffs, blens, src: torch.Tensor, soffs, slens, block_size: int, stream=None):
    """(list of DeviceDelta, batch totals) of delta_pairs_handle."""
    b = delta_pairs_handle(basis, boffs, blens, src, soffs, slens, block_size, stream)
    try:
        return b.deltas(), b.stats
    finally:
        b.close()


def match_batch(index: BatchIndex, buf: torch.Tensor, offs, lens, stream=None):
    """Batched rolling match: source f = buf[offs[f] : offs[f]+lens[f]] against basis f.
    Returns (list of DeviceDelta, batch totals)."""
    b = match_batch_handle(index, buf, offs, lens, stream)
    try:
        return b.deltas(), b.stats
    finally:
        b.close()


def match(index: Index, src: torch.Tensor, stream=None, length: int | None = None) -> DeviceDelta:
    """Greedy rolling match of a device-resident source (generator.rs:242-379)."""
    n = src.numel() if length is None else length
    h = ctypes.c_void_p()
    check(lib.sydelta_match_device(index.h, _ptr(src) if n else None, n, _stream(stream), ctypes.byref(h)))
    return _device_delta(h, _DeltaHandle(h))


class Chunk:
    """One rank's share of a chunk-sharded match of a single file (BASELINE C5):
    full-window positions [pos_begin, pos_end) classified against the all-gathered
    signature held by `index`.  `buf` holds source bytes [buf_pos, buf_pos + numel)."""

    def __init__(self, index: Index, buf: torch.Tensor, buf_pos: int, file_len: int, pos_begin: int, pos_end: int,
                 stream=None):
        self.h = ctypes.c_void_p()
        self.buf = buf  # must outlive the chunk (on-demand rescans read it)
        check(lib.sydelta_chunk_classify(index.h, _ptr(buf), buf_pos, buf.numel(), file_len, pos_begin, pos_end,
                                          _stream(stream), ctypes.byref(self.h)))

    def walk(self, entry: int):
        """Greedy walk from `entry` -> (DeviceDelta of [entry, exit), exit)."""
        d = ctypes.c_void_p()
        ex = ctypes.c_uint64()
        check(lib.sydelta_chunk_walk(self.h, entry, ctypes.byref(ex), ctypes.byref(d)))
        return _device_delta(d, _DeltaHandle(d)), int(ex.value)

    def close(self):
        if self.h:
            lib.sydelta_chunk_free(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def join_deltas(parts, source_size: int, block_size: int) -> DeviceDelta:
    """Concatenate chunk deltas in file order, merging a trailing Data op with the
    next chunk's leading Data op when contiguous (sydelta_delta_append's rule)."""
    ks, as_, bs_ = [], [], []
    for p in parts:
        k = np.asarray(p.kind, dtype=np.uint8)
        a = np.array(p.a, dtype=np.uint64)
        b = np.array(p.b, dtype=np.uint64)
        if k.size and ks:
            # the last non-empty part so far
            j = max(i for i in range(len(ks)) if ks[i].size) if any(x.size for x in ks) else -1
            if j >= 0 and ks[j][-1] == 1 and k[0] == 1 and int(as_[j][-1]) + int(bs_[j][-1]) == int(a[0]):
                bs_[j] = bs_[j].copy()
                bs_[j][-1] += b[0]
                k, a, b = k[1:], a[1:], b[1:]
        ks.append(k)
        as_.append(a)
        bs_.append(b)
    kind = np.concatenate(ks) if ks else np.zeros(0, np.uint8)
    a = np.concatenate(as_) if as_ else np.zeros(0, np.uint64)
    b = np.concatenate(bs_) if bs_ else np.zeros(0, np.uint64)
    stats = {"positions": sum(p.stats["positions"] for p in parts),
             "weak_hits": sum(p.stats["weak_hits"] for p in parts),
             "verified_hits": sum(p.stats["verified_hits"] for p in parts),
             "copy_ops": int((kind == 0).sum()), "data_ops": int((kind == 1).sum()),
             "literal_bytes": int(b[kind == 1].sum())}
    return DeviceDelta(kind, a, b, source_size, block_size, stats)


def delta_multi_device(devices, basis_chunks, src_chunks, src_pos, src_len: int, block_size: int) -> DeviceDelta:
    """One file chunk-sharded over `devices` inside the library (sydelta_delta_multi_device):
    basis_chunks[g] / src_chunks[g] are uint8 tensors on devices[g]; src_chunks[g] holds
    source bytes [src_pos[g], src_pos[g] + numel) (its chunk plus the block_size - 1 halo).
    The library synchronizes every stream it uses; the caller's work that filled the
    tensors must be complete (torch.cuda.synchronize)."""
    k = len(devices)
    VP = ctypes.c_void_p * k
    U = ctypes.c_uint64 * k
    h = ctypes.c_void_p()
    check(lib.sydelta_delta_multi_device((ctypes.c_int * k)(*devices), k,
                                         VP(*[_ptr(b) if b.numel() else None for b in basis_chunks]),
                                         U(*[b.numel() for b in basis_chunks]),
                                         VP(*[_ptr(c) if c.numel() else None for c in src_chunks]), U(*src_pos),
                                         U(*[c.numel() for c in src_chunks]), src_len, block_size, ctypes.byref(h)))
    return _device_delta(h, _DeltaHandle(h))


def thread_device() -> int:
    """The device the calling thread's path-level calls are bound to (sydelta_thread_device)."""
    d = ctypes.c_int(-1)
    check(lib.sydelta_thread_device(ctypes.byref(d)))
    return d.value


def synth_fill_range(buf: torch.Tensor, first: int, seed: int, stream=None) -> None:
    """Bytes [first, first + numel) of the synth_fill stream (first % 8 == 0)."""
    check(lib.sydelta_synth_fill_range(_ptr(buf), first, buf.numel(), seed & 0xFFFFFFFFFFFFFFFF, _stream(stream)))


def synth_mutate_blocks(dst: torch.Tensor, src: torch.Tensor, first: int, block_size: int, seed: int, rate_ppm: int,
                        stream=None) -> None:
    """C5 edit model: one substituted byte in each selected block (oracle.synth_edit_blocks)."""
    assert dst.numel() == src.numel()
    check(lib.sydelta_synth_mutate_blocks(_ptr(dst), _ptr(src), first, src.numel(), block_size,
                                          seed & 0xFFFFFFFFFFFFFFFF, rate_ppm, _stream(stream)))


def apply_device(basis: torch.Tensor, delta: DeviceDelta, lit: torch.Tensor, out: torch.Tensor | None = None,
                 stream=None):
    """apply_delta (applier.rs:22-56) on the device: Copy ops from `basis`, Data ops
    from `lit` at the op's source offset.  Returns (out tensor, stats dict)."""
    n = len(delta.kind)
    if out is None:
        total = int(np.asarray(delta.b, dtype=np.uint64).sum()) if n else 0
        out = torch.empty(max(total, 1), dtype=torch.uint8, device=basis.device)
    own = None
    if delta.handle is not None:  # the library's own delta: no copy of the ops
        h = delta.handle.h
    else:
        ops = np.zeros(n, dtype=_OP_DTYPE)
        if n:
            ops["kind"], ops["a"], ops["b"] = delta.kind, delta.a, delta.b
        own = h = lib.sydelta_delta_from_ops(ops.ctypes.data if n else None, n, delta.source_size,
                                             delta.block_size)
        if not h:
            raise ValueError("bad op array")
    st = _lib.DeltaStatsC()
    try:
        check(lib.sydelta_apply_delta_device(basis.device.index or 0, _ptr(basis), basis.numel(), h,
                                             _ptr(lit), lit.numel(), _ptr(out), out.numel(), _stream(stream),
                                             ctypes.byref(st)))
    finally:
        if own:
            lib.sydelta_delta_free(own)
    return out[:st.bytes_written], {f: int(getattr(st, f)) for f, _ in _lib.DeltaStatsC._fields_}


def block_compare(src: torch.Tensor, dst: torch.Tensor, block_size: int, stream=None):
    """The local transport's block-compare loop (local.rs:541-619) on device bytes.
    Returns (changed uint8 tensor with one flag per source block, stats dict with
    blocks / changed_blocks / literal_bytes / bytes_written)."""
    nb = -(-src.numel() // block_size) if block_size > 0 else 0
    changed = torch.empty(max(nb, 1), dtype=torch.uint8, device=src.device)
    st = _lib.BlockCompareStatsC()
    check(lib.sydelta_block_compare_device(src.device.index or 0, _ptr(src), src.numel(), _ptr(dst), dst.numel(),
                                           block_size, _ptr(changed), _stream(stream), ctypes.byref(st)))
    return changed[:nb], {f: int(getattr(st, f)) for f, _ in _lib.BlockCompareStatsC._fields_}


def estimate_change_ratio(src: torch.Tensor, dst: torch.Tensor, block_size: int, sample_count: int | None = None,
                          threshold: float | None = None, stream=None) -> dict:
    """estimate_change_ratio (ratio.rs:78-192) on device bytes: src is the new file,
    dst the existing one.  Returns the ChangeRatioResult fields as a dict."""
    r = _lib.ChangeRatioC()
    check(lib.sydelta_estimate_change_ratio_device(
        src.device.index or 0, _ptr(src), src.numel(), _ptr(dst), dst.numel(), block_size,
        -1 if sample_count is None else sample_count, -1.0 if threshold is None else threshold, _stream(stream),
        ctypes.byref(r)))
    return {"change_ratio": r.change_ratio, "blocks_sampled": r.blocks_sampled, "blocks_changed": r.blocks_changed,
            "use_delta": bool(r.use_delta), "threshold": r.threshold}


def xxh3(buf: torch.Tensor, stream=None) -> int:
    """XxHash3Hasher::hash_file / hash_data (integrity/xxhash3.rs:17-40) of device bytes."""
    out = ctypes.c_uint64()
    check(lib.sydelta_xxh3_device(buf.device.index or 0, _ptr(buf), buf.numel(), _stream(stream), ctypes.byref(out)))
    return out.value


def xxh3_batch(buf: torch.Tensor, offs, lens, stream=None) -> np.ndarray:
    """Whole-file XXH3-64 of files [offs[f], offs[f] + lens[f]) of `buf`."""
    o = np.ascontiguousarray(offs, dtype=np.uint64)
    ln = np.ascontiguousarray(lens, dtype=np.uint64)
    if o.shape != ln.shape:
        raise ValueError("offs and lens differ in length")
    if len(ln) and int((o + ln).max()) > buf.numel():
        raise ValueError("file range outside the buffer")
    out = np.zeros(len(ln), dtype=np.uint64)
    check(lib.sydelta_xxh3_batch_device(buf.device.index or 0, _ptr(buf), buf.numel(), o.ctypes.data, ln.ctypes.data, len(ln),
                                        _stream(stream), out.ctypes.data))
    return out


def synth_fill(buf: torch.Tensor, seed: int, stream=None) -> None:
    check(lib.sydelta_synth_fill(_ptr(buf), buf.numel(), seed & 0xFFFFFFFFFFFFFFFF, _stream(stream)))


def synth_mutate(dst: torch.Tensor, src: torch.Tensor, seed: int, rate_ppm: int, stream=None) -> None:
    assert dst.numel() == src.numel()
    check(lib.sydelta_synth_mutate(_ptr(dst), _ptr(src), src.numel(), seed & 0xFFFFFFFFFFFFFFFF, rate_ppm,
                                   _stream(stream)))


def set_profiling(on: bool) -> None:
    lib.sydelta_set_profiling(1 if on else 0)


def profile(reset: bool = False) -> dict:
    import json

    n = lib.sydelta_profile_json(None, 0, 0)
    buf = ctypes.create_string_buffer(n + 1)
    lib.sydelta_profile_json(buf, n + 1, 1 if reset else 0)
    return json.loads(buf.value.decode())
