"""GPU parity of K10 (k_walk_files): the greedy walk resolved on the device, one wave per
unit (generator.rs:116-221, the tail rule :156-184) -- each file of a batch, or each
segment of a chunk of one file (walked again from its true entry when the previous
segment's last Copy crosses into it).

Every case runs through the C ABI and is compared op for op with the C oracle, and with the
classifier + host walk on the same inputs (SYDELTA_FILE_WALK=0 / SYDELTA_CHUNK_WALK=0)."""
import random

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _oracle_ops(oracle_c, src, basis, bs):
    w, s, z = oracle_c.compute_checksums(basis, bs)
    return O.ops_from_arrays(*oracle_c.generate_delta(src, w, s, z, bs))


def _pack(parts):
    import torch

    offs, pos = [], 0
    for p in parts:
        offs.append(pos)
        pos += (len(p) + 15) & ~15
    host = bytearray(pos + 16)
    for o, p in zip(offs, parts):
        host[o:o + len(p)] = p
    buf = torch.frombuffer(host, dtype=torch.uint8).cuda()
    return buf, np.array(offs, np.uint64), np.array([len(p) for p in parts], np.uint64)


def _batch(gpu, pairs, bs, walk, monkeypatch, dx=""):
    """Batched signature + index + match of (src, basis) pairs; walk: SYDELTA_FILE_WALK; dx:
    SYDELTA_DEVICE_EXPAND (the op lists expanded by k_walk_expand or on the host)."""
    monkeypatch.setenv("SYDELTA_FILE_WALK", walk)
    monkeypatch.setenv("SYDELTA_DEVICE_EXPAND", dx)
    bbuf, boff, blen = _pack([b for _, b in pairs])
    sbuf, soff, slen = _pack([s for s, _ in pairs])
    w, s = gpu.signature_batch(bbuf, boff, blen, bs)
    nblk = [-(-int(x) // bs) for x in blen]
    last = [int(x) - (k - 1) * bs if k else 0 for x, k in zip(blen, nblk)]
    idx = gpu.BatchIndex(w, s, nblk, last, bs)
    gpu.set_profiling(True)
    gpu.profile(reset=True)
    out, tot = gpu.match_batch(idx, sbuf, soff, slen)
    prof = gpu.profile(reset=True)
    gpu.set_profiling(False)
    idx.close()
    return out, tot, prof


def _expanded():
    """Files whose op lists the device expanded so far (sydelta_expand_counters)."""
    import ctypes

    from sy_amd._lib import lib

    f, h = ctypes.c_uint64(), ctypes.c_uint64()
    lib.sydelta_expand_counters(ctypes.byref(f), ctypes.byref(h))
    return f.value, h.value


def _mutate(data: bytes, rng, nops: int) -> bytes:
    b = bytearray(data)
    for _ in range(nops):
        k = rng.randrange(5)
        p = rng.randrange(len(b) + 1) if b else 0
        if k == 0 and b:  # substitution
            b[min(p, len(b) - 1)] ^= rng.randrange(1, 256)
        elif k == 1:  # insertion
            b[p:p] = rng.randbytes(rng.randint(1, 40))
        elif k == 2 and b:  # deletion
            del b[p:p + rng.randint(1, 40)]
        elif k == 3 and len(b) > 64:  # duplication of a run
            q = rng.randrange(len(b) - 32)
            b[p:p] = b[q:q + rng.randint(1, 5000)]
        else:  # block-sized move
            q = rng.randrange(len(b) + 1)
            b[p:p] = b[q:q + 4096]
    return bytes(b)


def _cases(rng, bs, nfiles):
    pairs = []
    for i in range(nfiles):
        kind = i % 10
        if kind == 0:  # empty source
            basis, src = rng.randbytes(rng.randint(0, 3 * bs)), b""
        elif kind == 1:  # empty basis: one Data op
            basis, src = b"", rng.randbytes(rng.randint(1, 3 * bs))
        elif kind == 2:  # the tail rule: the basis's partial last block at the source's end
            basis = rng.randbytes(rng.randint(1, 6) * bs + rng.randint(1, bs - 1))
            src = rng.randbytes(rng.randint(0, bs)) + basis[-(len(basis) % bs):]
        elif kind == 3:  # a source shorter than a block, equal to the basis
            basis = rng.randbytes(rng.randint(1, bs - 1))
            src = basis
        elif kind == 4:  # periodic data: weak hits at many positions, duplicate keys
            pat = rng.randbytes(rng.choice([1, 3, 64, 100]))
            basis = (pat * (40 * bs // len(pat) + 1))[:rng.randint(bs, 40 * bs)]
            src = _mutate(basis, rng, 4)
        elif kind == 5:  # zeros with a few bytes set
            basis = bytearray(rng.randint(bs, 20 * bs))
            for _ in range(3):
                basis[rng.randrange(len(basis))] = rng.randrange(256)
            basis = bytes(basis)
            src = _mutate(basis, rng, 3)
        elif kind == 6:  # the C4 edit shape: one inserted byte + 16 substitutions
            basis = rng.randbytes(rng.randint(8, 64) * bs)
            s = bytearray(basis)
            p = rng.randrange(len(s) + 1)
            s[p:p] = bytes([rng.randrange(256)])
            for _ in range(16):
                s[rng.randrange(len(s))] ^= rng.randrange(1, 256)
            src = bytes(s)
        elif kind == 7:  # low alphabet
            basis = bytes(rng.randrange(2) for _ in range(rng.randint(bs, 12 * bs)))
            src = _mutate(basis, rng, 6)
        else:  # random edits
            basis = rng.randbytes(rng.randint(bs, 40 * bs))
            src = _mutate(basis, rng, 10)
        pairs.append((src, basis))
    return pairs


@pytest.mark.parametrize("dx", ["0", "1"])
@pytest.mark.parametrize("bs", [256, 320, 1024, 4096, 8192])
def test_file_walk_matches_oracle(gpu, oracle_c, monkeypatch, bs, dx):
    rng = random.Random(1000 + bs)
    pairs = _cases(rng, bs, 80)
    x0 = _expanded()
    out, tot, prof = _batch(gpu, pairs, bs, "1", monkeypatch, dx)
    assert "k_walk_files" in prof, prof
    x1 = _expanded()
    # dx 1: the device expanded every file, or (a file needed a re-walk) the host took the batch
    assert (x1[0] - x0[0], x1[1] - x0[1]) in (((len(pairs), 0), (0, 1)) if dx == "1" else ((0, 0),)), (x0, x1)
    for i, ((src, basis), d) in enumerate(zip(pairs, out)):
        assert d.tuples() == _oracle_ops(oracle_c, src, basis, bs), (bs, i)
        assert d.source_size == len(src) and d.block_size == bs
    assert tot["copy_ops"] == sum(d.stats["copy_ops"] for d in out)
    assert tot["literal_bytes"] == sum(d.stats["literal_bytes"] for d in out)
    # the classifier path gives the same lists
    out0, _, prof0 = _batch(gpu, pairs, bs, "0", monkeypatch)
    assert "k_walk_files" not in prof0
    assert [d.tuples() for d in out0] == [d.tuples() for d in out]


@pytest.mark.parametrize("asm", ["1", "4", "5", "16"])
def test_file_walk_asm_threads(gpu, oracle_c, monkeypatch, asm):
    """SYDELTA_ASM_THREADS (per call): the expansion's host threads, and with
    SYDELTA_DEVICE_EXPAND unset the choice it implies (<= 4: the walk kernel expands)."""
    monkeypatch.setenv("SYDELTA_ASM_THREADS", asm)
    bs = 1024
    pairs = _cases(random.Random(77), bs, 80)
    x0 = _expanded()
    out, _, _ = _batch(gpu, pairs, bs, "1", monkeypatch)
    x1 = _expanded()
    dev = int(asm) <= 4
    assert (x1[0] - x0[0], x1[1] - x0[1]) in (((len(pairs), 0), (0, 1)) if dev else ((0, 0),)), (asm, x0, x1)
    for i, ((src, basis), d) in enumerate(zip(pairs, out)):
        assert d.tuples() == _oracle_ops(oracle_c, src, basis, bs), (asm, i)


def test_file_walk_c4_shape_1mib(gpu, oracle_c, monkeypatch):
    """BASELINE C4's files (1 MiB, one inserted byte + 16 substitutions), 128 of them,
    through the default (auto) selection."""
    rng = random.Random(4404)
    pairs = []
    for f in range(128):
        basis = O.synth_bytes(1 << 20, 0x5E1D0004 + f).tobytes()
        s = bytearray(basis)
        p = rng.randrange(len(s) + 1)
        s[p:p] = bytes([rng.randrange(256)])
        for _ in range(16):
            s[rng.randrange(len(s))] ^= rng.randrange(1, 256)
        pairs.append((bytes(s), basis))
    monkeypatch.delenv("SYDELTA_FILE_WALK", raising=False)
    out, _, prof = _batch(gpu, pairs, 4096, "", monkeypatch)
    assert "k_walk_files" in prof
    for f, ((src, basis), d) in enumerate(zip(pairs, out)):
        assert d.tuples() == _oracle_ops(oracle_c, src, basis, 4096), f


def test_file_walk_long_literal_runs(gpu, oracle_c, monkeypatch):
    """Sources with long unmatched runs (several roll passes of 4096 starts between hits
    at bs 8192), matches at every phase, and blocks repeated so that later candidates in
    index order share the weak value."""
    rng = random.Random(77)
    bs = 8192
    pairs = []
    for i in range(16):
        blocks = [rng.randbytes(bs) for _ in range(12)]
        basis = b"".join(blocks + blocks[:3])  # duplicate blocks: the lowest index wins
        src = bytearray()
        for j in range(10):
            src += rng.randbytes(rng.randint(0, 3 * bs))  # a literal run
            src += blocks[rng.randrange(12)]
        pairs.append((bytes(src), basis))
    out, _, _ = _batch(gpu, pairs, bs, "1", monkeypatch)
    for i, ((src, basis), d) in enumerate(zip(pairs, out)):
        assert d.tuples() == _oracle_ops(oracle_c, src, basis, bs), i


def _to_dev(data: bytes, pad: int = 16):
    import torch

    t = torch.zeros(len(data) + pad, dtype=torch.uint8, device="cuda")
    if data:
        t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    return t


def _chunk_walk(gpu, src: bytes, basis: bytes, bs: int, bounds):
    """Signature + index of basis, then the chunks [bounds[g], bounds[g+1]) of src
    classified and walked in order (each from the previous one's exit), joined."""
    b = _to_dev(basis)
    w, s = gpu.signature(b[:len(basis)], bs)
    nb = w.numel()
    idx = gpu.Index(w, s, bs, (len(basis) - (nb - 1) * bs) if nb else 0)
    L = len(src)
    parts, entry, chunks = [], 0, []
    for g in range(len(bounds) - 1):
        p0, p1 = bounds[g], bounds[g + 1]
        final = g == len(bounds) - 2
        buf_pos = p0 & ~15
        end = L if final else min(L, p1 + bs - 1)
        chunks.append(gpu.Chunk(idx, _to_dev(src[buf_pos:end]), buf_pos, L, p0, p1 if not final else max(p1, L)))
    for c in chunks:
        d, entry = c.walk(entry)
        parts.append(d)
    for c in chunks:
        c.close()
    idx.close()
    return gpu.join_deltas(parts, L, bs)


@pytest.mark.parametrize("dx", ["0", "1"])
@pytest.mark.parametrize("bs", [256, 4096, 8192])
@pytest.mark.parametrize("nchunks", [1, 3])
def test_chunk_walk_segments(gpu, oracle_c, monkeypatch, bs, nchunks, dx):
    """K10 over a chunk's segments (128 blocks each): an early insertion shifts every later
    Copy off the block grid, so each segment boundary is crossed and the segments are walked
    again from the true entries; then a deletion realigns, substitutions and a duplicated
    run follow.  Equal to the oracle, and to the classifier + host walk; the ops written on the
    host or (dx 1, SYDELTA_DEVICE_EXPAND) by k_chunk_write."""
    rng = random.Random(bs + nchunks)
    nblk = 700
    basis = rng.randbytes(nblk * bs + rng.randint(1, bs - 1))
    s = bytearray(basis)
    s[5 * bs + 7:5 * bs + 7] = b"XY"                      # shifted by 2 from here
    del s[400 * bs + 3:400 * bs + 5]                        # realigned
    for _ in range(30):
        s[rng.randrange(len(s))] ^= rng.randrange(1, 256)
    q = rng.randrange(len(s) - 3 * bs)
    s[q:q] = s[q:q + 3 * bs]                                # a duplicated run
    src = bytes(s)
    npos = len(src) - bs + 1
    nb = -(-npos // bs)
    cuts = sorted(rng.sample(range(1, nb), nchunks - 1))
    bounds = [0] + [c * bs for c in cuts] + [npos]
    monkeypatch.delenv("SYDELTA_CHUNK_WALK", raising=False)
    monkeypatch.delenv("SYDELTA_PROBE", raising=False)
    monkeypatch.setenv("SYDELTA_DEVICE_EXPAND", dx)
    gpu.set_profiling(True)
    gpu.profile(reset=True)
    d = _chunk_walk(gpu, src, basis, bs, bounds)
    prof = gpu.profile(reset=True)
    gpu.set_profiling(False)
    assert "k_walk_files" in prof
    assert ("k_chunk_write" in prof) == (dx == "1"), prof
    exp = _oracle_ops(oracle_c, src, basis, bs)
    assert d.tuples() == exp
    monkeypatch.setenv("SYDELTA_CHUNK_WALK", "0")
    assert _chunk_walk(gpu, src, basis, bs, bounds).tuples() == exp


@pytest.mark.parametrize("dx", ["0", "1"])
@pytest.mark.parametrize("bs", [256, 4096])
@pytest.mark.parametrize("segs", ["2", "5", "16"])
def test_file_walk_in_segments(gpu, oracle_c, monkeypatch, bs, segs, dx):
    """Files cut into segments of >= 8 blocks (SYDELTA_FILE_SEGS): each segment walked from its
    start; a Copy that crosses into the next segment is absorbed by cutting that segment's
    leading literal run, or the segment is walked again from the exit.  Equal to the oracle."""
    rng = random.Random(2000 + bs + int(segs))
    pairs = _cases(rng, bs, 80)
    monkeypatch.setenv("SYDELTA_FILE_SEGS", segs)
    out, tot, prof = _batch(gpu, pairs, bs, "1", monkeypatch, dx)
    assert "k_walk_files" in prof
    for i, ((src, basis), d) in enumerate(zip(pairs, out)):
        assert d.tuples() == _oracle_ops(oracle_c, src, basis, bs), (bs, segs, i)
    assert tot["literal_bytes"] == sum(d.stats["literal_bytes"] for d in out)


def test_file_walk_c4_shape_few_files(gpu, oracle_c, monkeypatch):
    """An 8-GPU rank's share of C4 (few 1 MiB files): the auto mode cuts each file into
    segments (file_segs); every op list equals the oracle's."""
    rng = random.Random(4405)
    pairs = []
    for f in range(96):
        basis = O.synth_bytes(1 << 20, 0x5E1D0104 + f).tobytes()
        s = bytearray(basis)
        p = rng.randrange(len(s) + 1)
        s[p:p] = bytes([rng.randrange(256)])
        for _ in range(16):
            s[rng.randrange(len(s))] ^= rng.randrange(1, 256)
        pairs.append((bytes(s), basis))
    monkeypatch.delenv("SYDELTA_FILE_SEGS", raising=False)
    for dx in ("0", "1"):
        x0 = _expanded()
        out, _, prof = _batch(gpu, pairs, 4096, "", monkeypatch, dx)
        assert "k_walk_files" in prof
        assert _expanded()[0] - x0[0] == (len(pairs) if dx == "1" else 0)  # the C4 shape: no re-walks
        for f, ((src, basis), d) in enumerate(zip(pairs, out)):
            assert d.tuples() == _oracle_ops(oracle_c, src, basis, 4096), (dx, f)


# (SYDELTA_PREROLL, SYDELTA_SLIM_WALK, SYDELTA_CHUNK_SEG, SYDELTA_CHUNK_SEG_LAST): every
# output-affecting setting of the chunk pipeline, read per call
PIPE_KNOBS = [("1", "1", "", ""), ("0", "1", "", ""), ("1", "0", "", ""), ("2", "1", "", ""), ("2", "0", "", ""),
              ("1", "1", "64", "8"), ("0", "1", "1024", "")]


@pytest.mark.parametrize("dx", ["0", "1"])
@pytest.mark.parametrize("preroll,slim,seg,seg_last", PIPE_KNOBS)
def test_chunk_pipeline_two_parts(gpu, oracle_c, monkeypatch, preroll, slim, seg, seg_last, dx):
    """A chunk large enough for the two-part pipeline (>= 512 segments: 70 % / 30 %, the last
    part re-cut into shorter segments, the parts' walks on two streams), with insertions and
    deletions that shift the data across segment and part boundaries (re-walk rounds), a
    duplicated run and substitutions: equal to the oracle and to the classifier path, under
    every pre-roll / slim-walk / segment-size setting, each of which must launch the kernels
    it names; the ops written on the host or (dx 1) by k_chunk_write, the re-walked units'
    by the host after it."""
    rng = random.Random(512)
    bs = 256
    nblk = 600 * 128  # 600 segments of 128 blocks: 19.2 MB
    basis = O.synth_bytes(nblk * bs + 77, 0x5E1D0A01).tobytes()
    s = bytearray(basis)
    for _ in range(40):  # substitutions
        s[rng.randrange(len(s))] ^= rng.randrange(1, 256)
    split = int(600 * 0.7) * 128 * bs  # near the first part's end
    for p in sorted([3 * bs + 5, split - 7, split + 3 * bs + 1, len(s) - 50 * bs], reverse=True):
        s[p:p] = rng.randbytes(rng.randint(1, 9))  # each shifts everything after it
    del s[200 * 128 * bs:200 * 128 * bs + 11]
    q = rng.randrange(len(s) - 4 * bs)
    s[q:q] = s[q:q + 4 * bs]
    src = bytes(s)
    npos = len(src) - bs + 1
    monkeypatch.delenv("SYDELTA_CHUNK_WALK", raising=False)
    monkeypatch.delenv("SYDELTA_PROBE", raising=False)
    monkeypatch.delenv("SYDELTA_CHUNK_PIPE", raising=False)
    for k, v in (("SYDELTA_PREROLL", preroll), ("SYDELTA_SLIM_WALK", slim), ("SYDELTA_CHUNK_SEG", seg),
                 ("SYDELTA_CHUNK_SEG_LAST", seg_last), ("SYDELTA_DEVICE_EXPAND", dx)):
        monkeypatch.setenv(k, v)
    gpu.set_profiling(True)
    gpu.profile(reset=True)
    d = _chunk_walk(gpu, src, basis, bs, [0, npos])
    prof = gpu.profile(reset=True)
    gpu.set_profiling(False)
    nseg = -(-(npos // bs + 1) // int(seg or 128))
    parts = 2 if nseg >= 512 else 1  # (chunk_pipe_parts)
    assert prof["k_walk_files"]["count"] >= parts, prof  # the parts (and any re-walks)
    nparts_pre = {"0": 0, "1": 1, "2": parts}[preroll]
    assert prof.get("k_preroll", {}).get("count", 0) == nparts_pre, prof
    assert prof.get("k_walk_files_slim", {}).get("count", 0) == (nparts_pre if slim == "1" else 0), prof
    assert ("k_chunk_write" in prof) == (dx == "1"), prof
    exp = _oracle_ops(oracle_c, src, basis, bs)
    assert d.tuples() == exp
    if preroll == "1" and slim == "1" and not seg and dx == "0":
        monkeypatch.setenv("SYDELTA_CHUNK_WALK", "0")
        assert _chunk_walk(gpu, src, basis, bs, [0, npos]).tuples() == exp


@pytest.mark.late
def test_chunk_exact_buffers(gpu, oracle_c):
    """Non-final chunks whose source buffers end exactly where sydelta.h lets them (the last
    window byte, min(file_len, p1 + n - 1), in its 16-byte granule) at the END of a raw
    hipMalloc: the walk's and the pre-roll's loads must stay inside (they were
    bounded by the file length, ~4 KiB past a non-final chunk's buffer).  Three chunks at bs
    256 with shifted data (misses everywhere, rolls near each chunk's end), joined: equal to
    the oracle."""
    import ctypes

    import torch

    from sy_amd._lib import check, lib

    hip = ctypes.CDLL("libamdhip64.so")
    rng = random.Random(9090)
    bs = 256
    basis = rng.randbytes(3000 * bs + 77)
    s = bytearray(basis)
    for p in sorted(rng.sample(range(len(s)), 60), reverse=True):
        s[p:p] = bytes([rng.randrange(256)])  # insertions: every block after them is off the grid
    src = bytes(s)
    L = len(src)
    npos = L - bs + 1
    b = _to_dev(basis)
    w, st = gpu.signature(b[:len(basis)], bs)
    nb = w.numel()
    idx = gpu.Index(w, st, bs, len(basis) - (nb - 1) * bs)
    torch.cuda.synchronize()
    bounds = [0, 1000 * bs, 2100 * bs, npos]
    ptrs, parts, entry = [], [], 0
    try:
        for g in range(3):
            p0, p1 = bounds[g], bounds[g + 1]
            final = g == 2
            bpos = p0 & ~15
            end = L if final else min(L, p1 + bs - 1)
            blen = end - bpos
            alloc = (((blen + 15) & ~15) + 4095) & ~4095
            raw = ctypes.c_void_p()
            assert hip.hipMalloc(ctypes.byref(raw), ctypes.c_size_t(alloc)) == 0
            ptrs.append(raw)
            dptr = raw.value + alloc - ((blen + 15) & ~15)  # the buffer's granules end the allocation
            host = np.frombuffer(src[bpos:end], np.uint8)
            assert hip.hipMemcpy(ctypes.c_void_p(dptr), host.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(blen),
                                 1) == 0
            ch = ctypes.c_void_p()
            check(lib.sydelta_chunk_classify(idx.h, ctypes.c_void_p(dptr), bpos, blen, L, p0, max(p1, L) if final else p1,
                                             None, ctypes.byref(ch)))
            dh = ctypes.c_void_p()
            ex = ctypes.c_uint64()
            check(lib.sydelta_chunk_walk(ch, entry, ctypes.byref(ex), ctypes.byref(dh)))
            lib.sydelta_chunk_free(ch)
            parts.append(gpu._device_delta(dh, gpu._DeltaHandle(dh)))
            entry = int(ex.value)
        assert torch.cuda.synchronize() is None
        assert gpu.join_deltas(parts, L, bs).tuples() == _oracle_ops(oracle_c, src, basis, bs)
    finally:
        idx.close()
        for p in ptrs:
            hip.hipFree(p)


@pytest.mark.parametrize("dx", ["0", "1"])
@pytest.mark.parametrize("bs,nfiles", [(256, 80), (4096, 130), (1024, 200)])
def test_delta_pairs_matches_oracle(gpu, oracle_c, monkeypatch, bs, nfiles, dx):
    """sydelta_delta_pairs_device: signature + match of every pair in one call (two groups of
    files from 128 on, the second's signature beside the first's walks; no index): every op
    list equals the oracle's, and the three-call form's."""
    rng = random.Random(3000 + bs + nfiles)
    pairs = _cases(rng, bs, nfiles)
    monkeypatch.setenv("SYDELTA_DEVICE_EXPAND", dx)
    bbuf, boff, blen = _pack([b for _, b in pairs])
    sbuf, soff, slen = _pack([s for s, _ in pairs])
    gpu.set_profiling(True)
    gpu.profile(reset=True)
    out, tot = gpu.delta_pairs(bbuf, boff, blen, sbuf, soff, slen, bs)
    prof = gpu.profile(reset=True)
    gpu.set_profiling(False)
    assert prof["k_walk_files"]["count"] >= (2 if nfiles >= 128 else 1), prof
    assert "k_idx_insert" not in prof, prof
    for i, ((src, basis), d) in enumerate(zip(pairs, out)):
        assert d.tuples() == _oracle_ops(oracle_c, src, basis, bs), (bs, i)
        assert d.source_size == len(src) and d.block_size == bs
    assert tot["copy_ops"] == sum(d.stats["copy_ops"] for d in out)
    assert tot["literal_bytes"] == sum(d.stats["literal_bytes"] for d in out)


def test_delta_pairs_refuses(gpu):
    """The one-call form's limits: block sizes K10 does not take, bases above 1024 blocks."""
    import torch

    from sy_amd._lib import SyDeltaError

    buf = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    with pytest.raises(SyDeltaError):
        gpu.delta_pairs(buf, [0], [4096], buf, [0], [4096], 320 + 1)
    with pytest.raises(SyDeltaError):
        gpu.delta_pairs(buf, [0], [1025 * 256], buf, [0], [4096], 256)


@pytest.mark.parametrize("nfiles", [130, 1250])
def test_delta_pairs_c4_shape_on_stream(gpu, nfiles):
    """The bench's C4 step through the one-call form, repeated on a torch stream of its own:
    every file's op list equals the three-call form's (signature_batch + index + match_batch)."""
    import torch

    import bench

    basis, new, (boff, blen, soff, slen) = bench.c4_files(gpu, basis_bytes=1 << 20, nfiles=nfiles, first=77)
    torch.cuda.synchronize()
    w, s = gpu.signature_batch(basis, boff, blen, 4096)
    nblk = (blen + 4095) // 4096
    idx = gpu.BatchIndex(w, s, nblk, blen - (nblk - 1) * 4096, 4096)
    ref, _ = gpu.match_batch(idx, new, soff, slen)
    idx.close()
    exp = [d.tuples() for d in ref]
    stream = torch.cuda.Stream()
    for rep in range(3):
        with torch.cuda.stream(stream):
            b = gpu.delta_pairs_handle(basis, boff, blen, new, soff, slen, 4096, stream=stream)
        got = [d.tuples() for d in b.deltas()]
        b.close()
        bad = [f for f in range(nfiles) if got[f] != exp[f]]
        assert not bad, (rep, len(bad), bad[:10])
