"""GPU parity for the aligned-window probe (k_probe + on-demand block scans) and
the chunk-sharded single-file match (BASELINE C5).

Both must reproduce generator.rs's op list exactly: the probe only changes which
window starts are classified before the walk (the walk scans a block on demand
when an unaligned hit jumps into it), and chunking only splits the walk at
block-aligned boundaries.  The oracle is the C restatement of generator.rs."""
import os
import random

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["0", "1", "1c"], ids=["scan-only", "probe", "probe-classifier"])
def probe_mode(request):
    """SYDELTA_PROBE=0: every window scanned.  "1": the aligned probe; chunked matches walk
    on the device (K10 over segments).  "1c": the probe with chunks classified and walked
    on the host (SYDELTA_CHUNK_WALK=0)."""
    old = {k: os.environ.get(k) for k in ("SYDELTA_PROBE", "SYDELTA_CHUNK_WALK")}
    os.environ["SYDELTA_PROBE"] = request.param[0]
    if request.param == "1c":
        os.environ["SYDELTA_CHUNK_WALK"] = "0"
    yield request.param[0]
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def _to_dev(data: bytes, pad: int = 16):
    import torch

    t = torch.zeros(len(data) + pad, dtype=torch.uint8, device="cuda")
    if data:
        t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    return t


def _index(gpu, basis: bytes, bs: int):
    b = _to_dev(basis)
    w, s = gpu.signature(b[:len(basis)], bs)
    nb = w.numel()
    last = (len(basis) - (nb - 1) * bs) if nb else 0
    return gpu.Index(w, s, bs, last)


def _oracle_ops(oracle_c, src, basis, bs):
    w, s, z = oracle_c.compute_checksums(basis, bs)
    return O.ops_from_arrays(*oracle_c.generate_delta(src, w, s, z, bs))


def _shift_edits(basis: bytes, rng, bs: int, pairs: int) -> bytes:
    """Insertions each followed later by a deletion of the same length: the source
    is shifted between them (unaligned hits) and realigned after (aligned hits), so
    a walk leaving a shifted hit jumps into a block whose aligned window hit."""
    src = bytearray(basis)
    for _ in range(pairs):
        a = rng.randrange(0, max(1, len(src) - 4 * bs))
        k = rng.randint(1, 3)
        src[a:a] = rng.randbytes(k)
        b = a + k + rng.randint(bs // 2 + 1, 3 * bs)
        del src[b:b + k]
    return bytes(src)


def test_probe_random_small(probe_mode, gpu, oracle_c):
    rng = random.Random(77)
    for it in range(150):
        alpha = rng.choice([2, 4, 256])
        basis = bytes(rng.randrange(alpha) for _ in range(rng.randint(0, 3000)))
        src = bytearray(basis)
        for _ in range(rng.randint(0, 5)):
            op, p = rng.randint(0, 2), rng.randint(0, max(0, len(src) - 1))
            if op == 0 and src:
                src[p] = rng.randrange(256)
            elif op == 1:
                src[p:p] = bytes(rng.randrange(alpha) for _ in range(rng.randint(1, 9)))
            else:
                del src[p:p + rng.randint(1, 9)]
        src = bytes(src)
        bs = rng.choice([1, 3, 7, 16, 33, 64, 100, 241, 256, 300, 512])
        idx = _index(gpu, basis, bs)
        d = gpu.match(idx, _to_dev(src), length=len(src))
        idx.close()
        assert d.tuples() == _oracle_ops(oracle_c, src, basis, bs), (it, bs)


@pytest.mark.parametrize("bs", [256, 512, 1000, 4096, 8192])
def test_probe_shifted_regions(bs, probe_mode, gpu, oracle_c):
    """Shift/realign edits: exercises the on-demand block scans of the probe path."""
    rng = random.Random(bs)
    basis = rng.randbytes(rng.randint(1 << 20, 2 << 20))
    src = _shift_edits(basis, rng, bs, 60)
    src = bytearray(src)
    for _ in range(20):
        src[rng.randrange(len(src))] ^= 0x77
    src = bytes(src)
    idx = _index(gpu, basis, bs)
    d = gpu.match(idx, _to_dev(src), length=len(src))
    idx.close()
    expect = _oracle_ops(oracle_c, src, basis, bs)
    assert d.tuples() == expect
    assert O.py_apply_delta(basis, src, d.tuples()) == src


@pytest.mark.parametrize("pattern", [b"\x00", b"ABC", b"0123456789" * 7])
def test_probe_degenerate(pattern, probe_mode, gpu, oracle_c):
    basis = (pattern * (200000 // len(pattern) + 1))[:200000]
    for src in (basis, basis[5:] + b"xyz", b"q" + basis[:150000]):
        for bs in (4096, 1000):
            idx = _index(gpu, basis, bs)
            d = gpu.match(idx, _to_dev(src), length=len(src))
            idx.close()
            assert d.tuples() == _oracle_ops(oracle_c, src, basis, bs)


def test_probe_auto_mode_c1(gpu, oracle_c):
    """Auto mode on the C1 shape (two small edits in 50 MB): the 1-in-16 sample
    hits, so the probe path runs; result identical to the oracle."""
    os.environ.pop("SYDELTA_PROBE", None)
    n = 52_428_800
    old = O.synth_bytes(n, 0x5E1D0001)
    new = old.copy()
    new[1 << 20:(1 << 20) + 18] = np.frombuffer(b"MODIFIED DATA HERE", np.uint8)
    new[0:20] = np.frombuffer(b"HEADER DATA AT START", np.uint8)
    idx = _index(gpu, old.tobytes(), 4096)
    d = gpu.match(idx, _to_dev(new.tobytes()), length=n)
    idx.close()
    assert d.tuples() == _oracle_ops(oracle_c, new, old, 4096)
    # only the two edited blocks' window starts were scanned
    assert d.stats["weak_hits"] < 4 * 4096


def _chunked(gpu, src: bytes, idx, bs: int, bounds):
    """Classify chunk g = positions [bounds[g], bounds[g+1]) from its own buffer
    (chunk bytes + window halo), then chain the walks."""
    L = len(src)
    chunks = []
    for g in range(len(bounds) - 1):
        p0, p1 = bounds[g], bounds[g + 1]
        final = g == len(bounds) - 2
        buf_pos = p0 & ~15
        end = L if final else min(L, p1 + bs - 1)
        buf = _to_dev(src[buf_pos:end])
        chunks.append(gpu.Chunk(idx, buf, buf_pos, L, p0, p1 if not final else max(p1, L)))
    parts, entry = [], 0
    for c in chunks:
        d, entry = c.walk(entry)
        parts.append(d)
    for c in chunks:
        c.close()
    return gpu.join_deltas(parts, L, bs)


@pytest.mark.parametrize("bs", [64, 1000, 4096, 8192])
@pytest.mark.parametrize("nchunks", [1, 2, 3, 8])
def test_chunked_equals_whole(bs, nchunks, probe_mode, gpu, oracle_c):
    rng = random.Random(bs * 31 + nchunks)
    nblk = rng.randint(40, 300)
    basis = rng.randbytes(nblk * bs + rng.randint(0, bs - 1))
    src = _shift_edits(basis, rng, bs, 8)
    src = bytearray(src)
    for _ in range(10):
        src[rng.randrange(len(src))] ^= 0x11
    src = bytes(src)
    idx = _index(gpu, basis, bs)
    npos = max(0, len(src) - bs + 1)
    nb = -(-npos // bs)
    cuts = sorted(rng.sample(range(1, max(2, nb)), min(nchunks - 1, max(0, nb - 1))))
    bounds = [0] + [c * bs for c in cuts] + [npos]
    d = _chunked(gpu, src, idx, bs, bounds)
    idx.close()
    assert d.tuples() == _oracle_ops(oracle_c, src, basis, bs)


def test_chunked_copy_crosses_boundary(probe_mode, gpu, oracle_c):
    """A 1-byte insertion before a chunk boundary: the last Copy of chunk 0 ends
    inside chunk 1, whose walk must start at that exit, not at its first position."""
    bs = 4096
    rng = random.Random(5)
    basis = rng.randbytes(64 * bs + 123)
    src = basis[:10 * bs] + b"Z" + basis[10 * bs:]
    idx = _index(gpu, basis, bs)
    npos = len(src) - bs + 1
    for cut in (20, 31, 32, 40):
        d = _chunked(gpu, src, idx, bs, [0, cut * bs, npos])
        assert d.tuples() == _oracle_ops(oracle_c, src, basis, bs), cut
    idx.close()


def test_chunk_rejects_bad_layout(gpu):
    import sy_amd._lib as L

    bs = 4096
    basis = bytes(range(256)) * 64
    idx = _index(gpu, basis, bs)
    buf = _to_dev(basis)
    with pytest.raises(L.SyDeltaError):
        gpu.Chunk(idx, buf, 0, len(basis), 100, 2 * bs)  # pos_begin not block-aligned
    with pytest.raises(L.SyDeltaError):
        gpu.Chunk(idx, buf[:1000], 0, 10 * bs, 0, 2 * bs)  # buffer too short for the windows
    idx.close()


def test_synth_ranges_match_oracle(gpu):
    import torch

    n, first, bs = 1 << 20, 3 << 16, 8192
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    gpu.synth_fill_range(t, first, 0x5E1D0005)
    ref = O.synth_bytes(n, 0x5E1D0005, first)
    assert np.array_equal(t.cpu().numpy(), ref)
    u = torch.empty_like(t)
    gpu.synth_mutate_blocks(u, t, first, bs, 0x5E1D0006, 100000)
    exp = O.synth_edit_blocks(ref, first, bs, 0x5E1D0006, 100000)
    got = u.cpu().numpy()
    assert np.array_equal(got, exp)
    changed = np.nonzero(got != ref)[0] // bs
    assert 4 <= len(set(changed.tolist())) <= 30 and len(changed) == len(set(changed.tolist()))


# ---------------------------------------------------------------------------
# apply_delta on the device (applier.rs:22-56)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("bs", [7, 64, 1000, 4096, 8192])
def test_apply_device_round_trip(bs, gpu, oracle_c):
    """apply(match(basis, src)) == src byte for byte, with unaligned Copy/Data
    offsets (odd block sizes, shifted regions) and ops longer than a 64 KiB slice."""
    import torch

    rng = random.Random(bs + 11)
    basis = rng.randbytes(rng.randint(200 * bs, 300 * bs) + rng.randint(0, bs - 1))
    src = bytearray(_shift_edits(basis, rng, bs, 6))
    for _ in range(8):
        p = rng.randrange(len(src))
        src[p:p] = rng.randbytes(rng.randint(1, 3 * bs))
    src = bytes(src)
    idx = _index(gpu, basis, bs)
    s_dev = _to_dev(src)
    d = gpu.match(idx, s_dev, length=len(src))
    idx.close()
    assert d.tuples() == _oracle_ops(oracle_c, src, basis, bs)
    b_dev = _to_dev(basis)
    out, st = gpu.apply_device(b_dev[:len(basis)], d, s_dev[:len(src)])
    torch.cuda.synchronize()
    assert bytes(out.cpu().numpy()) == src
    assert st["bytes_written"] == len(src) and st["operations_count"] == len(d.kind)
    assert st["literal_bytes"] == sum(int(b) for k, b in zip(d.kind, d.b) if int(k) == 1)


@pytest.mark.parametrize("offs", [(1, 3, 5), (15, 0, 9), (0, 7, 1), (8, 8, 8)])
def test_apply_device_misaligned_views(offs, gpu, oracle_c):
    """basis, literal and output buffers that are views at byte
    offsets (basis[1:], lit[3:], out[5:]) rebuild the source exactly."""
    import torch

    ob, ol, oo = offs
    bs = 1000
    rng = random.Random(sum(offs) + 5)
    basis = rng.randbytes(300 * bs + 123)
    src = bytearray(_shift_edits(basis, rng, bs, 6))
    for _ in range(6):
        p = rng.randrange(len(src))
        src[p:p] = rng.randbytes(rng.randint(1, 200 * 1024))  # Data ops longer than a slice
    src = bytes(src)
    idx = _index(gpu, basis, bs)
    d = gpu.match(idx, _to_dev(src), length=len(src))
    idx.close()
    assert d.tuples() == _oracle_ops(oracle_c, src, basis, bs)
    bbuf = torch.zeros(len(basis) + ob + 32, dtype=torch.uint8, device="cuda")
    bbuf[ob:ob + len(basis)] = torch.frombuffer(bytearray(basis), dtype=torch.uint8).cuda()
    lbuf = torch.zeros(len(src) + ol + 32, dtype=torch.uint8, device="cuda")
    lbuf[ol:ol + len(src)] = torch.frombuffer(bytearray(src), dtype=torch.uint8).cuda()
    obuf = torch.full((len(src) + oo + 32,), 0xEE, dtype=torch.uint8, device="cuda")
    out, st = gpu.apply_device(bbuf[ob:ob + len(basis)], d, lbuf[ol:ol + len(src)], out=obuf[oo:oo + len(src)])
    torch.cuda.synchronize()
    assert st["bytes_written"] == len(src)
    got = obuf.cpu().numpy()
    assert bytes(got[oo:oo + len(src)]) == src
    assert (got[:oo] == 0xEE).all() and (got[oo + len(src):] == 0xEE).all()  # nothing written outside


def test_apply_device_rejects_copy_past_end(gpu):
    import torch
    import sy_amd._lib as L

    b = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    bad = gpu.DeviceDelta(np.array([0], np.uint32), np.array([4000], np.uint64), np.array([200], np.uint64),
                          200, 4096, {})
    with pytest.raises(L.SyDeltaError):
        gpu.apply_device(b, bad, b)
    # the bad Copy after many good ones (the whole op list is checked before any copy)
    k = np.zeros(100, np.uint32)
    a = np.zeros(100, np.uint64)
    ln = np.full(100, 40, np.uint64)
    a[77] = 4090
    late = gpu.DeviceDelta(k, a, ln, 4000, 4096, {})
    out = torch.zeros(8192, dtype=torch.uint8, device="cuda")
    with pytest.raises(L.SyDeltaError, match="past the end of the basis"):
        gpu.apply_device(b, late, b, out=out)


@pytest.fixture(params=[2, 3, 8], ids=lambda t: f"walk{t}")
def par_walk(request, monkeypatch):
    """Force the parallel speculative walk (Classifier::walk_parallel) at any size."""
    monkeypatch.setenv("SYDELTA_WALK_THREADS", str(request.param))
    monkeypatch.setenv("SYDELTA_WALK_PAR_MIN", "1")
    return request.param


@pytest.mark.parametrize("bs", [64, 1000, 4096])
def test_parallel_walk_equals_oracle(bs, par_walk, probe_mode, gpu, oracle_c):
    """Split points land inside literal runs, inside unaligned-copy stretches (exits
    differ from the speculative entries: segments re-walked) and between aligned
    copies; the joined op list must equal the sequential one."""
    rng = random.Random(bs + 7 * par_walk)
    basis = rng.randbytes(rng.randint(200, 400) * bs + rng.randint(0, bs - 1))
    src = _shift_edits(basis, rng, bs, 12)
    src = bytearray(src)
    a = rng.randrange(len(src) // 2)
    src[a:a + 5 * bs] = rng.randbytes(5 * bs)  # a long literal run
    for _ in range(15):
        src[rng.randrange(len(src))] ^= 0x3C
    src = bytes(src)
    idx = _index(gpu, basis, bs)
    d = gpu.match(idx, _to_dev(src), length=len(src))
    idx.close()
    assert d.tuples() == _oracle_ops(oracle_c, src, basis, bs)


def test_parallel_walk_all_literal_and_identical(par_walk, gpu, oracle_c):
    bs = 512
    rng = random.Random(3)
    basis = rng.randbytes(300 * bs + 17)
    for src in (rng.randbytes(len(basis)), basis, basis[:-100] + rng.randbytes(100)):
        idx = _index(gpu, basis, bs)
        d = gpu.match(idx, _to_dev(src), length=len(src))
        idx.close()
        assert d.tuples() == _oracle_ops(oracle_c, src, basis, bs)


@pytest.mark.parametrize("nchunks", [2, 3])
def test_parallel_walk_in_chunks(nchunks, par_walk, gpu, oracle_c):
    bs = 1000
    rng = random.Random(nchunks)
    basis = rng.randbytes(250 * bs + 321)
    src = _shift_edits(basis, rng, bs, 6)
    idx = _index(gpu, basis, bs)
    npos = len(src) - bs + 1
    nb = -(-npos // bs)
    cuts = sorted(rng.sample(range(1, nb), nchunks - 1))
    d = _chunked(gpu, src, idx, bs, [0] + [c * bs for c in cuts] + [npos])
    idx.close()
    assert d.tuples() == _oracle_ops(oracle_c, src, basis, bs)


@pytest.mark.parametrize("phase", ["0", "1"], ids=["scan-runs", "phase-probe"])
@pytest.mark.parametrize("bs", [256, 1000, 4096])
def test_phase_probe_shifted_runs(bs, phase, gpu, oracle_c, monkeypatch):
    """Long runs of aligned misses (C4 shape: one insertion, then substitutions and a
    second insertion/deletion inside the shifted region): the phase probe classifies
    one window per block at the run's phase; the op list equals the oracle's."""
    monkeypatch.setenv("SYDELTA_PROBE", "1")
    monkeypatch.setenv("SYDELTA_PHASE_PROBE", phase)
    rng = random.Random(bs * 3 + int(phase))
    for case in range(6):
        basis = rng.randbytes(rng.randint(60, 200) * bs + rng.randint(0, bs - 1))
        src = bytearray(basis)
        a = rng.randrange(len(src) // 4)
        src[a:a] = rng.randbytes(rng.randint(1, 3))                    # phase shift
        for _ in range(rng.randint(0, 12)):                            # substitutions
            src[rng.randrange(a, len(src))] ^= 0x5A
        if case % 2:
            b = rng.randrange(a + 20 * bs, len(src) - 2 * bs)          # second shift in the run
            if rng.random() < 0.5:
                src[b:b] = rng.randbytes(rng.randint(1, 5))
            else:
                del src[b:b + rng.randint(1, 5)]
        if case == 5:
            src[-3 * bs:] = rng.randbytes(3 * bs)                      # literal tail
        src = bytes(src)
        idx = _index(gpu, basis, bs)
        d = gpu.match(idx, _to_dev(src), length=len(src))
        idx.close()
        assert d.tuples() == _oracle_ops(oracle_c, src, basis, bs), case


def test_phase_probe_batch_c4_shape(gpu, oracle_c, monkeypatch):
    """Batched match of 64 files with one insertion + 16 substitutions each (BASELINE
    C4's edit shape, 64 KiB files): every file's op list equals the oracle's."""
    import torch

    monkeypatch.setenv("SYDELTA_PROBE", "1")
    monkeypatch.setenv("SYDELTA_FILE_WALK", "0")  # the classifier's phase probe, not K10
    bs = 4096
    rng = random.Random(44)
    bases, news = [], []
    for f in range(64):
        b = rng.randbytes(64 * 1024)
        s = bytearray(b)
        p = rng.randrange(len(s) + 1)
        s[p:p] = bytes([rng.randrange(256)])
        for _ in range(16):
            s[rng.randrange(len(s))] ^= rng.randrange(1, 256)
        bases.append(b)
        news.append(bytes(s))

    def pack(files):
        offs, pos = [], 0
        for f in files:
            offs.append(pos)
            pos += (len(f) + 15) // 16 * 16
        buf = bytearray(pos + 16)
        for o, f in zip(offs, files):
            buf[o:o + len(f)] = f
        return torch.frombuffer(buf, dtype=torch.uint8).cuda(), offs, [len(f) for f in files]

    bbuf, boff, blen = pack(bases)
    sbuf, soff, slen = pack(news)
    w, s = gpu.signature_batch(bbuf, boff, blen, bs)
    nblk = [-(-x // bs) for x in blen]
    last = [x - (k - 1) * bs for x, k in zip(blen, nblk)]
    idx = gpu.BatchIndex(w, s, nblk, last, bs)
    ds, _ = gpu.match_batch(idx, sbuf, soff, slen)
    idx.close()
    for f in range(64):
        assert ds[f].tuples() == _oracle_ops(oracle_c, news[f], bases[f], bs), f
