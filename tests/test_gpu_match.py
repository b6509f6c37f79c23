"""GPU parity: rolling match (K2-K5 + host op emission) vs the oracle.

Bit-exact op lists (kind, offset/size) against the C/Python restatement of
generator.rs on the same inputs; at BASELINE sizes, size-independent
properties (reconstruction, op-list invariants, idempotence)."""
import os
import random

import numpy as np
import pytest

from golden_io import dec, load_cases
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _to_dev(data: bytes):
    import torch

    t = torch.zeros(len(data) + 16, dtype=torch.uint8, device="cuda")
    if data:
        t[:len(data)] = torch.frombuffer(bytearray(data), dtype=torch.uint8).cuda()
    return t


def _device_ops(gpu, src: bytes, basis: bytes, bs: int):
    import torch

    b = _to_dev(basis)
    w, s = gpu.signature(b[:len(basis)], bs)
    nb = w.numel()
    last = (len(basis) - (nb - 1) * bs) if nb else 0
    idx = gpu.Index(w, s, bs, last)
    d = gpu.match(idx, _to_dev(src), length=len(src))
    idx.close()
    torch.cuda.synchronize()
    return d


def _oracle_ops(oracle_c, src, basis, bs):
    w, s, z = oracle_c.compute_checksums(basis, bs)
    return O.ops_from_arrays(*oracle_c.generate_delta(src, w, s, z, bs))


@pytest.mark.parametrize("case", load_cases("delta"), ids=lambda c: c["name"])
def test_golden_delta_device(case, gpu):
    src, basis, bs = dec(case["src"]), dec(case["basis"]), case["block_size"]
    d = _device_ops(gpu, src, basis, bs)
    assert d.tuples() == [tuple(o) for o in case["expect_ops"]]
    assert d.source_size == len(src) and d.block_size == bs


@pytest.mark.parametrize("case", load_cases("delta"), ids=lambda c: c["name"])
def test_golden_delta_path_api(case, gpu, tmp_path):
    """The src/delta mirror end to end: compute_checksums(dest) ->
    generate_delta_streaming(source) -> apply_delta == source."""
    import sy_amd.delta as D

    src, basis, bs = dec(case["src"]), dec(case["basis"]), case["block_size"]
    ps, pb, pn = tmp_path / "src", tmp_path / "dest", tmp_path / "out"
    ps.write_bytes(src)
    pb.write_bytes(basis)
    sigs = D.compute_checksums(pb, bs)
    for gen in (D.generate_delta_streaming, D.generate_delta):
        delta = gen(ps, sigs, bs)
        got = []
        for op in delta.ops:
            got.append(("C", op.offset, op.size) if isinstance(op, D.Copy) else ("D", len(op.data)))
        exp = [("C", a, b) if k == "C" else ("D", b) for k, a, b in case["expect_ops"]]
        assert got == exp
        assert abs(delta.compression_ratio() - case["compression_ratio"]) == 0.0
        D.apply_delta(pb, delta, pn)
        assert pn.read_bytes() == src


def _mutate(b, rng, nops=6):
    b = bytearray(b)
    for _ in range(rng.randint(0, nops)):
        op, p = rng.randint(0, 3), rng.randint(0, max(0, len(b) - 1))
        if op == 0 and b:
            b[p] = rng.randint(0, 255)
        elif op == 1:
            b[p:p] = bytes(rng.randint(0, 255) for _ in range(rng.randint(1, 20)))
        elif op == 2:
            del b[p:p + rng.randint(1, 20)]
        else:
            q = rng.randint(0, max(0, len(b) - 1))
            b[p:p] = b[q:q + rng.randint(1, 40)]
    return bytes(b)


def test_random_small_differential(gpu, oracle_c):
    rng = random.Random(2024)
    for it in range(250):
        alpha = rng.choice([2, 4, 256])
        basis = bytes(rng.randrange(alpha) for _ in range(rng.randint(0, 1500)))
        src = _mutate(basis, rng)
        bs = rng.choice(list(range(1, 49)) + [64, 100, 241, 256, 300, 512])
        assert _device_ops(gpu, src, basis, bs).tuples() == _oracle_ops(oracle_c, src, basis, bs), (it, bs)


@pytest.mark.parametrize("bs", [512, 1000, 4096, 8192, 65536, 131072])
def test_random_medium_edits(bs, gpu, oracle_c):
    rng = random.Random(bs * 7)
    basis = rng.randbytes(rng.randint(2 << 20, 4 << 20))
    src = bytearray(basis)
    for _ in range(40):  # substitutions, insertions, deletions, block moves
        op, p = rng.randint(0, 3), rng.randrange(len(src))
        if op == 0:
            src[p] ^= 0x5A
        elif op == 1:
            src[p:p] = rng.randbytes(rng.randint(1, 300))
        elif op == 2:
            del src[p:p + rng.randint(1, 300)]
        else:
            q = rng.randrange(len(src))
            src[p:p] = src[q:q + rng.randint(1, 3 * bs)]
    src = bytes(src)
    d = _device_ops(gpu, src, basis, bs)
    assert d.tuples() == _oracle_ops(oracle_c, src, basis, bs)
    assert O.py_apply_delta(basis, src, d.tuples()) == src


@pytest.mark.parametrize("small", ["0", "1"])
@pytest.mark.parametrize("bs", [1024, 4096])
def test_scan_small_index_modes(bs, small, gpu, oracle_c, monkeypatch):
    """SYDELTA_SCAN_SMALL (per call): a small index scanned by k_scan_lds (0) or by the
    register-fed scans' small mode (k_scan_r at bs 4096, k_scan_g elsewhere); every
    position scanned (SYDELTA_PROBE=0)."""
    monkeypatch.setenv("SYDELTA_SCAN_SMALL", small)
    monkeypatch.setenv("SYDELTA_PROBE", "0")
    rng = random.Random(bs + int(small))
    basis = rng.randbytes(rng.randint(1 << 20, 2 << 20))
    src = bytearray(basis)
    for _ in range(30):
        op, p = rng.randint(0, 2), rng.randrange(len(src))
        if op == 0:
            src[p] ^= 0x3C
        elif op == 1:
            src[p:p] = rng.randbytes(rng.randint(1, 200))
        else:
            q = rng.randrange(len(src))
            src[p:p] = src[q:q + rng.randint(1, 2 * bs)]
    src = bytes(src)
    gpu.set_profiling(True)
    gpu.profile(reset=True)
    try:
        d = _device_ops(gpu, src, basis, bs)
        prof = gpu.profile(reset=True)
    finally:
        gpu.set_profiling(False)
    want = "k_scan_lds" if small == "0" else ("k_scan_r" if bs == 4096 else "k_scan_g")
    assert want in prof, prof
    assert d.tuples() == _oracle_ops(oracle_c, src, basis, bs)


@pytest.mark.parametrize("pattern", [b"\x00", b"ABC", b"ABCD", b"0123456789" * 7])
def test_degenerate_repetitive_data(pattern, gpu, oracle_c):
    """All-zero / periodic data: every window matches (dense hits, the chain
    must still follow the reference's greedy jumps and lowest-index rule)."""
    basis = (pattern * (300000 // len(pattern) + 1))[:300000]
    for src in (basis, basis[5:] + b"xyz", b"q" + basis[: 150000]):
        for bs in (4096, 1000, 7):
            assert _device_ops(gpu, src, basis, bs).tuples() == _oracle_ops(oracle_c, src, basis, bs)


def test_tail_rule_cases(gpu, oracle_c):
    rng = random.Random(99)
    for _ in range(40):
        bs = rng.choice([8, 64, 300, 4096])
        basis = rng.randbytes(rng.randint(1, 5) * bs + rng.randint(1, bs - 1))
        pre = rng.randbytes(rng.randint(0, 3 * bs))
        src = pre + basis[-(len(basis) % bs):]  # the partial last block at the end
        if rng.random() < 0.5:
            src = pre + basis
        assert _device_ops(gpu, src, basis, bs).tuples() == _oracle_ops(oracle_c, src, basis, bs)


def test_source_shorter_than_block(gpu, oracle_c):
    basis = b"0123456789"
    for src in (b"", b"789", b"6789", b"89", b"0123", b"x789"):
        assert _device_ops(gpu, src, basis, 4).tuples() == _oracle_ops(oracle_c, src, basis, 4)
        assert _device_ops(gpu, src, basis, 64).tuples() == _oracle_ops(oracle_c, src, basis, 64)


def test_config1_delta_bench_50mb(gpu, oracle_c):
    """BASELINE config 1 (delta_bench.rs:18,25 edits on non-sparse data), bs 4096."""
    n = 52_428_800
    old = O.synth_bytes(n, 0x5E1D0001)
    new = old.copy()
    new[1 << 20:(1 << 20) + 18] = np.frombuffer(b"MODIFIED DATA HERE", np.uint8)
    new[0:20] = np.frombuffer(b"HEADER DATA AT START", np.uint8)
    d = _device_ops(gpu, new.tobytes(), old.tobytes(), 4096)
    assert d.tuples() == _oracle_ops(oracle_c, new, old, 4096)
    assert d.stats["copy_ops"] == n // 4096 - 2


def test_config3_property_1gib(gpu):
    """BASELINE config 3 shape at 1 GiB: Bernoulli(5%) byte substitutions leave no
    4 KiB window intact, so the exact result is one Data op over the whole source;
    every weak hit must have failed strong verification."""
    import torch

    n = 1 << 30
    bs = 4096
    basis = torch.empty(n, dtype=torch.uint8, device="cuda")
    new = torch.empty(n, dtype=torch.uint8, device="cuda")
    gpu.synth_fill(basis, 0x5E1D0002)
    gpu.synth_mutate(new, basis, 0x5E1D0003, 50000)
    frac = (new != basis).float().mean().item()
    assert 0.049 < frac < 0.051
    w, s = gpu.signature(basis, bs)
    idx = gpu.Index(w, s, bs, bs)
    d = gpu.match(idx, new)
    assert d.tuples() == [("D", 0, n)]
    assert d.stats["verified_hits"] == 0 and d.stats["positions"] == n - bs + 1
    d2 = gpu.match(idx, basis)  # identical source: all Copy, in order
    assert d2.tuples() == [("C", i * bs, bs) for i in range(n // bs)]
    idx.close()


def _batch_device(gpu, pairs, bs):
    """Batched signature + index + match of (src, basis) pairs packed in two buffers
    (16-byte aligned file starts)."""
    import torch

    def pack(parts):
        offs, pos = [], 0
        for p in parts:
            offs.append(pos)
            pos += (len(p) + 15) & ~15
        buf = torch.zeros(pos + 16, dtype=torch.uint8, device="cuda")
        host = bytearray(pos + 16)
        for o, p in zip(offs, parts):
            host[o:o + len(p)] = p
        buf.copy_(torch.frombuffer(host, dtype=torch.uint8).cuda())
        return buf, np.array(offs, np.uint64), np.array([len(p) for p in parts], np.uint64)

    bbuf, boff, blen = pack([b for _, b in pairs])
    sbuf, soff, slen = pack([s for s, _ in pairs])
    w, s = gpu.signature_batch(bbuf, boff, blen, bs)
    nblk = [-(-int(l) // bs) for l in blen]
    last = [int(l) - (k - 1) * bs if k else 0 for l, k in zip(blen, nblk)]
    idx = gpu.BatchIndex(w, s, nblk, last, bs)
    out, tot = gpu.match_batch(idx, sbuf, soff, slen)
    idx.close()
    return out, tot


def test_batch_matches_per_file_oracle(gpu, oracle_c):
    """BASELINE config 4 path: many independent pairs in one launch give, per file,
    exactly the op list sy's generate_delta would (generator.rs:242-379), including
    empty sources, empty bases, sources shorter than a block and tail-rule files."""
    rng = random.Random(4)
    for bs in (4096, 64, 1000):
        pairs = []
        for i in range(120):
            kind = i % 6
            if kind == 0:
                basis = rng.randbytes(rng.randint(0, 3 * bs))
                src = b""
            elif kind == 1:
                basis = b""
                src = rng.randbytes(rng.randint(0, 3 * bs))
            elif kind == 2:
                basis = rng.randbytes(rng.randint(1, 6) * bs + rng.randint(1, bs - 1))
                src = rng.randbytes(rng.randint(0, bs)) + basis[-(len(basis) % bs):]
            else:
                basis = rng.randbytes(rng.randint(bs, 40 * bs))
                src = _mutate(basis, rng, nops=10)
            pairs.append((src, basis))
        out, tot = _batch_device(gpu, pairs, bs)
        assert len(out) == len(pairs)
        for i, ((src, basis), d) in enumerate(zip(pairs, out)):
            assert d.tuples() == _oracle_ops(oracle_c, src, basis, bs), (bs, i)
            assert d.source_size == len(src)
        assert tot["copy_ops"] == sum(d.stats["copy_ops"] for d in out)


def test_batch_1mib_files_c4_shape(gpu, oracle_c):
    """C4 shape (1 MiB files, one inserted byte + 16 substitutions each), 64 files."""
    rng = random.Random(44)
    pairs = []
    for f in range(64):
        basis = O.synth_bytes(1 << 20, 0x5E1D0004 + f).tobytes()
        src = bytearray(basis)
        p = rng.randrange(len(src))
        src[p:p] = bytes([rng.randrange(256)])
        for _ in range(16):
            q = rng.randrange(len(src))
            src[q] ^= 1 + rng.randrange(255)
        pairs.append((bytes(src), basis))
    out, _ = _batch_device(gpu, pairs, 4096)
    for (src, basis), d in zip(pairs, out):
        assert d.tuples() == _oracle_ops(oracle_c, src, basis, 4096)


def test_match_past_4gib_properties(gpu):
    """A 5 GiB source (positions past 2^32, scan segments past 2^31 positions, a
    partial last block): one 1-byte insertion at 3 GiB and 1% of 8 KiB blocks edited.
    The op list tiles the source, apply(delta) rebuilds it bit-exactly on the device,
    and every block away from an edit is copied."""
    import torch

    bs = 8192
    n = (5 << 30) + 1234
    m = 3 << 30
    basis = torch.empty(n + 16, dtype=torch.uint8, device="cuda")
    gpu.synth_fill_range(basis[:n], 0, 0x5E1D0009)
    src = torch.empty(n + 1 + 16, dtype=torch.uint8, device="cuda")
    src[:m] = basis[:m]
    src[m] = 0x5A
    src[m + 1:n + 1] = basis[m:n]
    gpu.synth_mutate_blocks(src[:n + 1], src[:n + 1], 0, bs, 0x5E1D000A, 10000)
    L = n + 1
    w, s = gpu.signature(basis[:n], bs)
    idx = gpu.Index(w, s, bs, n - (w.numel() - 1) * bs)
    d = gpu.match(idx, src, length=L)
    idx.close()
    kind = np.asarray(d.kind)
    a = np.asarray(d.a, dtype=np.uint64)
    b = np.asarray(d.b, dtype=np.uint64)
    assert int(b.sum()) == L
    pos = np.concatenate([[0], np.cumsum(b)[:-1]]).astype(np.uint64)
    data = kind == 1
    assert np.array_equal(a[data], pos[data])  # Data ops name their own source bytes
    assert d.stats["copy_ops"] > 0.97 * (n // bs)
    assert (pos[~data] > (1 << 32)).any()  # copies found past 4 GiB of positions
    out = torch.empty(L + 16, dtype=torch.uint8, device="cuda")
    rebuilt, st = gpu.apply_device(basis[:n], d, src[:L], out=out)
    assert st["bytes_written"] == L
    assert torch.equal(rebuilt, src[:L])
