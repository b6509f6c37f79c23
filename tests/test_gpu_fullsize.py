"""BASELINE configs C4 and C5 at their configured sizes on one GPU (one MI355X holds
both in HBM), through the same C ABI calls the bench makes.

* C4: 10 000 x 1 MiB basis files, each source with one inserted byte and 16 byte
  substitutions (bench.c4_files), one batched signature + index + match.  For every
  file: the ops tile the source, Data ops name their own source bytes, Copy ops name
  whole basis blocks, and apply_delta on the device rebuilds the source bit-exactly.
  Every file's op list equals the C oracle's (generator.rs:242-379), the oracle run on the
  host's cores (the last files' batch offsets lie past 2^32).
* C5: one 64 GiB file, bs 8192, 1 % of blocks with one substituted byte, matched as 8
  block-aligned chunks (shard.chunk_bounds) classified against the whole signature
  and walked in a chain (each chunk from the previous chunk's exit,
  generator.rs:116-221); the joined op list tiles the file, apply_delta rebuilds it
  (compared on the device in 4 GiB pieces), the whole 8 Mi-op list equals the analytic one
  (each edited block's bytes a literal run -- consecutive ones one Data op -- every other
  block a Copy of itself: random 8 KiB blocks share no weak+strong pair and no window
  straddling an edited block matches), and the 7 chunk-boundary neighbourhoods are
  re-derived by the C oracle from an op start before each boundary.
"""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.late]

GIB = 1 << 30


def _check_tiling(kind, a, b, length, bs, basis_len):
    """Ops tile [0, length); Data ops name their own source range; Copy ops name a
    whole basis block (offset multiple of bs, size bs or the basis's last block)."""
    kind = np.asarray(kind)
    a = np.asarray(a, dtype=np.uint64)
    b = np.asarray(b, dtype=np.uint64)
    assert int(b.sum()) == length
    pos = np.concatenate([[0], np.cumsum(b)[:-1]]).astype(np.uint64)
    data = kind == 1
    assert np.array_equal(a[data], pos[data])
    assert (b[data] > 0).all()
    cp = ~data
    assert (a[cp] % np.uint64(bs) == 0).all()
    last = basis_len - (basis_len - 1) // bs * bs
    ok = (b[cp] == bs) | ((b[cp] == last) & (a[cp] == basis_len - last))
    assert ok.all()
    return pos


def test_c4_full_batch(gpu, oracle_c):
    import torch

    import bench

    bs = 4096
    nfiles = 10000
    fsz = 1 << 20
    basis, new, (boff, blen, soff, slen) = bench.c4_files(gpu, basis_bytes=fsz, nfiles=nfiles, first=0)
    assert int(soff[-1]) > (1 << 32)  # the last files sit past 2^32 in the batch
    w, s = gpu.signature_batch(basis, boff, blen, bs)
    nblk = (blen + bs - 1) // bs
    last = blen - (nblk - 1) * bs
    idx = gpu.BatchIndex(w, s, nblk, last, bs)
    deltas, tot = gpu.match_batch(idx, new, soff, slen)
    idx.close()
    assert len(deltas) == nfiles
    assert tot["copy_ops"] == sum(d.stats["copy_ops"] for d in deltas)
    out = torch.empty(fsz + 1 + 16, dtype=torch.uint8, device="cuda")
    for f, d in enumerate(deltas):
        assert d.source_size == fsz + 1
        _check_tiling(d.kind, d.a, d.b, fsz + 1, bs, fsz)
        # one inserted byte: every block but the one holding it (and those with a
        # substitution) is copied
        assert d.stats["copy_ops"] >= 256 - 1 - 16 - 1
        src_f = new[int(soff[f]):int(soff[f]) + fsz + 1]
        rebuilt, st = gpu.apply_device(basis[int(boff[f]):int(boff[f]) + fsz], d, src_f, out=out)
        assert st["bytes_written"] == fsz + 1
        assert torch.equal(rebuilt, src_f), f
    # every file's op list against the C oracle, on the host's cores (the oracle's calls
    # release the GIL)
    from concurrent.futures import ThreadPoolExecutor

    import bench as B

    hb = basis.cpu().numpy()
    hn = new.cpu().numpy()

    def one(f):
        bh = hb[int(boff[f]):int(boff[f]) + fsz]
        sh = hn[int(soff[f]):int(soff[f]) + fsz + 1]
        wk, st, sz = oracle_c.compute_checksums(bh, bs)
        return O.ops_from_arrays(*oracle_c.generate_delta(sh, wk, st, sz, bs))

    with ThreadPoolExecutor(max(2, B.host_cores()[0])) as ex:
        for f, exp in enumerate(ex.map(one, range(nfiles), chunksize=64)):
            assert deltas[f].tuples() == exp, f


def test_c5_full_chained_chunks(gpu, oracle_c):
    import torch

    from sy_amd import shard

    bs = 8192
    L = 64 * GIB
    world = 8
    basis = torch.empty(L + 16, dtype=torch.uint8, device="cuda")
    src = torch.empty(L + 16, dtype=torch.uint8, device="cuda")
    step = 8 * GIB
    for o in range(0, L, step):  # the bench's C5 generators, rank by rank
        gpu.synth_fill_range(basis[o:o + step], o, 0x5E1D0005)
        gpu.synth_fill_range(src[o:o + step], o, 0x5E1D0005)
        gpu.synth_mutate_blocks(src[o:o + step], src[o:o + step], o, bs, 0x5E1D0006, 10000)
    # each rank signs its basis share; the all-gather is the concatenation
    ws, ss = [], []
    for o in range(0, L, step):
        w, s = gpu.signature(basis[o:o + step], bs)
        ws.append(w)
        ss.append(s)
    w = torch.cat(ws)
    s = torch.cat(ss)
    assert w.numel() == L // bs
    idx = gpu.Index(w, s, bs, bs)
    bounds = [shard.chunk_bounds(L, bs, world, g) for g in range(world)]
    chunks = [gpu.Chunk(idx, src[:L], 0, L, p0, p1) for p0, p1 in bounds]
    # the chain: speculative walks from each chunk's first position, redone from the
    # true entry where the previous exit differs (shard.walk_chain's rule, serialized)
    parts, entry, redone = [], 0, 0
    for g, ch in enumerate(chunks):
        d, ex = ch.walk(bounds[g][0])
        if entry != bounds[g][0]:
            d, ex = ch.walk(entry)
            redone += 1
        parts.append(d)
        entry = ex
    for ch in chunks:
        ch.close()
    idx.close()
    assert entry == L
    joined = gpu.join_deltas(parts, L, bs)
    pos = _check_tiling(joined.kind, joined.a, joined.b, L, bs, L)
    nblocks = L // bs
    assert joined.stats["copy_ops"] > 0.985 * nblocks
    # the analytic op list (synth_mutate_blocks' edited-block set, tests/analytic_ops.py)
    from tests.analytic_ops import block_edit_ops, edited_blocks

    exp_kind, exp_a, exp_b = block_edit_ops(edited_blocks(nblocks, 0x5E1D0006, 10000), bs)
    assert np.array_equal(np.asarray(joined.kind, dtype=np.uint8), exp_kind)
    assert np.array_equal(np.asarray(joined.a, dtype=np.uint64), exp_a)
    assert np.array_equal(np.asarray(joined.b, dtype=np.uint64), exp_b)
    out = torch.empty(L + 16, dtype=torch.uint8, device="cuda")
    rebuilt, st = gpu.apply_device(basis[:L], joined, src[:L], out=out)
    assert st["bytes_written"] == L
    for o in range(0, L, 4 * GIB):
        assert torch.equal(rebuilt[o:o + 4 * GIB], src[o:o + 4 * GIB]), o
    del out, rebuilt
    # boundary neighbourhoods against the oracle: from the op start at least 3 blocks
    # before each boundary, the oracle's greedy walk of the next 8 blocks of source
    # (against the whole signature) gives the same ops up to 5 blocks on
    W = w.cpu().numpy()
    S = s.cpu().numpy()
    size = np.full(W.size, bs, np.uint64)
    kind = np.asarray(joined.kind)
    a = np.asarray(joined.a, dtype=np.uint64)
    b = np.asarray(joined.b, dtype=np.uint64)
    for g in range(1, world):
        p = bounds[g][0]
        i = int(np.searchsorted(pos, np.uint64(p - 3 * bs), side="right")) - 1
        x0 = int(pos[i])
        snip = src[x0:x0 + 8 * bs].cpu().numpy().tobytes()
        ok, oa, ob = oracle_c.generate_delta(snip, W, S, size, bs)
        got = []
        j = i
        while j < len(kind) and int(pos[j]) < x0 + 5 * bs:
            got.append(("C" if kind[j] == 0 else "D", int(a[j]) - (x0 if kind[j] == 1 else 0), int(b[j])))
            j += 1
        exp = []
        q = x0
        for k_, x_, y_ in zip(ok, oa, ob):
            if q >= x0 + 5 * bs:
                break
            exp.append(("C" if k_ == 0 else "D", int(x_), int(y_)))
            q += int(y_)
        # a Data run still open at the cut continues in the device list
        if exp and got and exp[-1][0] == "D" and got[-1][0] == "D":
            exp[-1] = exp[-1][:2]
            got[-1] = got[-1][:2]
        assert got == exp, (g, x0)
